"""``src.robust_angle_estimation`` — the reference ships this module byte-identical to
``src/algorithms/robust_angle_estimation.py``; both import paths resolve to the same implementation."""
from .algorithms.robust_angle_estimation import RobustAngleEstimator, extract_angles_robust  # noqa: F401

__all__ = ['RobustAngleEstimator', 'extract_angles_robust']

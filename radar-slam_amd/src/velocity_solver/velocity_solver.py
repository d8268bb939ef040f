"""Two-step ego-velocity solve on MI355X.

Drop-in for ``src/velocity_solver/velocity_solver.py`` of the reference (``VelocitySolver`` :20-415,
``estimate_velocity_from_angles`` :418-467).

The reference minimises f(v, w) = sum (y - 4 pi dt / lambda (v + w x p).d)^2 with differential evolution
(seed 42) inside box bounds (:209-263).  The model is linear in (v, w): k [d, p x d].[v; w], so each DE
step is a box-constrained linear least-squares problem with a unique convex optimum; librsl solves it
exactly in fp64 on the device (``rsl_bvls``: 3 unknowns for step 1 with w = 0, 6 for step 2).  With the
reference's own targets (elevation 0, p = r d, :334-339) the w and v_z columns vanish; those components
are then undetermined by the cost (DE returns arbitrary values for them) and this solver returns 0.
The batched per-frame path (many frames at once) is ``rsl.RadarChain`` / ``rsl_velocity``.
"""
from __future__ import annotations

import logging
from typing import Dict, List, Optional

import numpy as np

from rsl import ops

logger = logging.getLogger(__name__)

_TRANS_BOUNDS = [(-50, 50), (-50, 50), (-10, 10)]                       # velocity_solver.py:216
_FULL_BOUNDS = _TRANS_BOUNDS + [(-10, 10), (-10, 10), (-10, 10)]       # velocity_solver.py:250-251


def _result(x, fun, method):
    from scipy.optimize import OptimizeResult
    return OptimizeResult(x=np.asarray(x, dtype=np.float64), fun=float(fun), success=True, status=0, nit=0,
                          nfev=0, message=f'exact box-constrained linear least squares on the device ({method})')


class VelocitySolver:
    """Reference constructor / attributes / methods (velocity_solver.py:20-415)."""

    def __init__(self, fc: float = 77e9, lambda_c: float = None, num_antennas: int = 8,
                 antenna_spacing: float = None, optimization_method: str = 'differential_evolution',
                 max_iterations: int = 1000, tolerance: float = 1e-6):
        self.fc = fc
        self.c = 3e8
        self.lambda_c = lambda_c or (self.c / self.fc)
        self.num_antennas = num_antennas
        self.antenna_spacing = antenna_spacing or (self.lambda_c / 2)
        self.optimization_method = optimization_method
        self.max_iterations = max_iterations
        self.tolerance = tolerance
        self.antenna_positions = np.arange(self.num_antennas) * self.antenna_spacing
        logger.info("Initialized velocity solver:")
        logger.info(f"  Wavelength: {self.lambda_c * 1000:.2f} mm")
        logger.info(f"  Optimization method: {optimization_method}")

    def _k(self, dt):
        return 4 * np.pi * dt / self.lambda_c

    # -- a25 / a26 / a27 --------------------------------------------------------------------------------
    def compute_phase_difference_model(self, target_positions: np.ndarray, target_angles: np.ndarray,
                                       velocity: np.ndarray, angular_velocity: np.ndarray, dt: float) -> np.ndarray:
        x = np.concatenate([np.asarray(velocity, np.float64).reshape(3), np.asarray(angular_velocity, np.float64).reshape(3)])
        return ops.phase_model(target_positions, target_angles, x, self._k(dt))['pred']

    def compute_observed_phase_differences(self, rds_data: np.ndarray, target_info: List[Dict]) -> np.ndarray:
        """angle(s[1] * conj(s[0])) of each target's spatial signature (velocity_solver.py:115-140)."""
        if len(target_info) == 0:
            return np.array([])
        sigs = np.stack([np.asarray(t['spatial_signature']) for t in target_info])
        _, _, ph = ops.cell_extras(sigs=sigs, want_phase=True)
        return ph

    def cost_function(self, motion_params: np.ndarray, target_positions: np.ndarray, target_angles: np.ndarray,
                      observed_phases: np.ndarray, dt: float) -> float:
        return ops.phase_model(target_positions, target_angles, np.asarray(motion_params, np.float64), self._k(dt),
                               y=observed_phases)['cost']

    # -- a28 ----------------------------------------------------------------------------------------------
    def two_step_optimization(self, target_positions: np.ndarray, target_angles: np.ndarray,
                              observed_phases: np.ndarray, dt: float,
                              initial_guess: Optional[np.ndarray] = None) -> Dict:
        N = len(target_positions)
        if N < 3:
            logger.warning("Insufficient targets for optimization")
            return {'success': False, 'message': 'Insufficient targets'}
        k = self._k(dt)
        bounded = self.optimization_method == 'differential_evolution'
        tb = _TRANS_BOUNDS if bounded else [(-np.inf, np.inf)] * 3
        fb = _FULL_BOUNDS if bounded else [(-np.inf, np.inf)] * 6
        big = 1e300
        lo3 = [max(b[0], -big) for b in tb]
        hi3 = [min(b[1], big) for b in tb]
        lo6 = [max(b[0], -big) for b in fb]
        hi6 = [min(b[1], big) for b in fb]
        logger.info("Step 1: Solving for translational velocity...")
        x3, c3 = ops.bvls(target_positions, target_angles, observed_phases, k, lo3, hi3)
        logger.info(f"Step 1 result: v_trans = {x3}")
        logger.info("Step 2: Refining with full 6-DoF motion...")
        x6, c6 = ops.bvls(target_positions, target_angles, observed_phases, k, lo6, hi6)
        velocity_est, angular_velocity_est = x6[:3].copy(), x6[3:].copy()
        m = ops.phase_model(target_positions, target_angles, x6, k, y=observed_phases)
        predicted, residuals = m['pred'], m['resid']
        rmse = np.sqrt(np.mean(residuals ** 2))
        max_residual = np.max(np.abs(residuals))
        results = {'success': True, 'velocity': velocity_est, 'angular_velocity': angular_velocity_est,
                   'cost': m['cost'], 'rmse': rmse, 'max_residual': max_residual, 'residuals': residuals,
                   'predicted_phases': predicted, 'observed_phases': np.asarray(observed_phases),
                   'num_targets': N, 'step1_result': _result(x3, c3, 'rsl_bvls, 3 unknowns'),
                   'step2_result': _result(x6, m['cost'], 'rsl_bvls, 6 unknowns')}
        logger.info("Optimization complete:")
        logger.info(f"  Velocity: {velocity_est}")
        logger.info(f"  Angular velocity: {angular_velocity_est}")
        logger.info(f"  RMSE: {rmse:.6f}")
        logger.info(f"  Max residual: {max_residual:.6f}")
        return results

    # -- a29 ----------------------------------------------------------------------------------------------
    def solve_velocity(self, rds_data: np.ndarray, target_info: List[Dict], dt: float = 0.1,
                       initial_guess: Optional[np.ndarray] = None) -> Dict:
        pos, ang = [], []
        for t in target_info:  # velocity_solver.py:330-342 (elevation 0)
            r, az, el = t['range_m'], t['azimuth_rad'], 0.0
            pos.append([r * np.cos(el) * np.cos(az), r * np.cos(el) * np.sin(az), r * np.sin(el)])
            ang.append([az, el])
        pos = np.array(pos)
        ang = np.array(ang)
        obs = self.compute_observed_phase_differences(rds_data, target_info)
        return self.two_step_optimization(pos, ang, obs, dt, initial_guess)

    def visualize_results(self, results: Dict, save_path: Optional[str] = None) -> None:
        if not results['success']:
            logger.warning("Cannot visualize failed optimization")
            return
        import matplotlib.pyplot as plt
        fig, axes = plt.subplots(2, 2, figsize=(12, 10))
        axes[0, 0].bar(['vx', 'vy', 'vz'], results['velocity'])
        axes[0, 1].bar(['wx', 'wy', 'wz'], results['angular_velocity'])
        axes[1, 0].plot(results['residuals'], 'o-', alpha=0.7)
        axes[1, 1].scatter(results['observed_phases'], results['predicted_phases'], alpha=0.7)
        plt.tight_layout()
        if save_path:
            plt.savefig(save_path, dpi=150, bbox_inches='tight')
        plt.show()


def estimate_velocity_from_angles(angles_path: str, rds_path: str, output_path: str, radar_params: Dict = None,
                                  dt: float = 0.1) -> Dict:
    """File wrapper (velocity_solver.py:418-467).  Keeps the reference's ``.item()`` on the loaded
    ``targets`` object array, which raises ValueError for more than one target (velocity_solver.py:438)."""
    data = np.load(angles_path, allow_pickle=True)
    target_info = data['targets'].item()
    rds = np.load(rds_path)
    logger.info(f"Loaded {len(target_info)} targets")
    if radar_params is None:
        radar_params = {'fc': 77e9, 'lambda_c': 3e8 / 77e9, 'num_antennas': 8}
    solver = VelocitySolver(**radar_params)
    results = solver.solve_velocity(rds, target_info, dt)
    np.savez(output_path, **results)
    logger.info(f"Velocity estimation complete: {results['success']}")
    return results


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser(description='Estimate velocity from angles')
    ap.add_argument('--angles', required=True)
    ap.add_argument('--rds', required=True)
    ap.add_argument('--out', required=True)
    ap.add_argument('--dt', type=float, default=0.1)
    a = ap.parse_args()
    print(f"Velocity estimation complete: {estimate_velocity_from_angles(a.angles, a.rds, a.out, dt=a.dt)}")

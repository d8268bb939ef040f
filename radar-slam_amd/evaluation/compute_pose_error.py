"""Pose error evaluation (APE / RTE) on MI355X.

Drop-in for ``evaluation/compute_pose_error.py`` of the reference (``PoseErrorEvaluator`` :23-517,
``evaluate_pose_errors`` :520-588), imported by ``scripts/run_ego_motion_pipeline.py:38``.

The trajectory-wide work runs in librsl (``rsl.evaluation``, kernels in ``csrc/rsl_eval.hip``): the Umeyama
alignment (centred cross-covariance + 3x3 SVD, :98-140), the orientation alignment (Rotation.mean of
gt * est^-1 as the principal eigenvector of sum q q^T, :142-169), the per-pose APE errors and statistics
(:171-236) and the RTE segment search and errors (:238-306).  The reference's observable conventions are kept:
columns 3:7 of a pose are read as scipy quaternions (scalar last) whatever the docstring says, the alignment is
recomputed inside ``compute_rte``, a segment length without a segment has no entry, keys are
``f'rte_{L:.0f}m'``.  The reference's aligned quaternions carry LAPACK's eigenvector sign; the device returns the
same rotations with the mean quaternion's w >= 0.  The three small private helpers (``_find_segment_end``,
``_compute_relative_transformation``, ``_compute_transformation_error``) act on one segment at a time and stay
on the host, as plain numpy on a handful of numbers.
"""
from __future__ import annotations

import logging
import os
from typing import Dict, List, Optional, Tuple

import numpy as np

from rsl.evaluation import align_poses

logger = logging.getLogger(__name__)


def _quat_matrix(q):
    """Rotation.from_quat(q).as_matrix() for one scipy quaternion (scalar last, normalised first)."""
    x, y, z, w = np.asarray(q, dtype=np.float64) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


class PoseErrorEvaluator:
    def __init__(self, max_ape_threshold: float = 1.0, max_rte_threshold: float = 0.5,
                 rte_segment_lengths: List[float] = [100, 200, 300, 400, 500, 600, 700, 800]):
        self.max_ape_threshold = max_ape_threshold
        self.max_rte_threshold = max_rte_threshold
        self.rte_segment_lengths = rte_segment_lengths
        logger.info("Initialized pose error evaluator")
        logger.info(f"  Max APE threshold: {max_ape_threshold} m")
        logger.info(f"  Max RTE threshold: {max_rte_threshold} m")
        logger.info(f"  RTE segment lengths: {rte_segment_lengths} m")

    # -- alignment (:51-169) -----------------------------------------------------------------------------------
    @staticmethod
    def _info(al):
        a = al.align.cpu().numpy()
        R, t, Rq = a[0:9].reshape(3, 3), a[9:12], a[12:21].reshape(3, 3)
        T = np.eye(4)
        T[:3, :3], T[:3, 3] = Rq, t
        info = {'position_translation': t, 'position_rotation': R, 'orientation_rotation': Rq,
                'scale_factor': float(a[25])}
        return T, info

    def align_trajectories(self, estimated_poses: np.ndarray,
                           ground_truth_poses: np.ndarray) -> Tuple[np.ndarray, np.ndarray, Dict]:
        al = align_poses(estimated_poses, ground_truth_poses)
        T, info = self._info(al)
        logger.info("Aligned trajectories:")
        logger.info(f"  Translation: {info['position_translation']}")
        logger.info(f"  Scale factor: {info['scale_factor']:.6f}")
        return al.aligned.cpu().numpy(), T, info

    def _umeyama_alignment(self, source: np.ndarray, target: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        n = len(source)
        ident = np.tile([0.0, 0.0, 0.0, 1.0], (n, 1))
        al = align_poses(np.column_stack([source, ident]), np.column_stack([target, ident]))
        a = al.align.cpu().numpy()
        T = np.eye(4)
        T[:3, :3], T[:3, 3] = a[0:9].reshape(3, 3), a[9:12]
        return al.aligned.cpu().numpy()[:, :3], T

    def _align_orientations(self, source_quats: np.ndarray, target_quats: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        n = len(source_quats)
        zero = np.zeros((n, 3))
        al = align_poses(np.column_stack([zero, source_quats]), np.column_stack([zero, target_quats]))
        return al.aligned.cpu().numpy()[:, 3:7], al.align.cpu().numpy()[12:21].reshape(3, 3)

    # -- APE (:171-236) ----------------------------------------------------------------------------------------
    def compute_ape(self, estimated_poses: np.ndarray, ground_truth_poses: np.ndarray) -> Dict:
        al = align_poses(estimated_poses, ground_truth_poses)
        _, info = self._info(al)
        err = al.ape_err.cpu().numpy()
        st = al.ape_stats.cpu().numpy()
        out = {'position_errors': err[0], 'orientation_errors': err[1], 'pose_errors': err[2]}
        for k, pre in enumerate(('position', 'orientation', 'pose')):
            out[f'{pre}_rmse'], out[f'{pre}_mean'], out[f'{pre}_std'], out[f'{pre}_max'] = (float(x) for x in st[k, :4])
        ape = {k: out[k] for k in ('position_errors', 'orientation_errors', 'pose_errors', 'position_rmse',
                                    'orientation_rmse', 'pose_rmse', 'position_mean', 'orientation_mean',
                                    'pose_mean', 'position_std', 'orientation_std', 'pose_std', 'position_max',
                                    'orientation_max', 'pose_max')}
        ape['alignment_info'] = info
        logger.info("APE computation complete:")
        logger.info(f"  Position RMSE: {ape['position_rmse']:.6f} m")
        logger.info(f"  Orientation RMSE: {ape['orientation_rmse']:.6f} rad")
        logger.info(f"  Pose RMSE: {ape['pose_rmse']:.6f}")
        return ape

    # -- RTE (:238-361) ----------------------------------------------------------------------------------------
    def compute_rte(self, estimated_poses: np.ndarray, ground_truth_poses: np.ndarray,
                    timestamps: Optional[np.ndarray] = None) -> Dict:
        al = align_poses(estimated_poses, ground_truth_poses)
        lengths = list(self.rte_segment_lengths)
        err, cnt, st = al.rte(lengths)
        out = {}
        for l, L in enumerate(lengths):
            n = int(cnt[l])
            if n == 0:
                continue
            out[f'rte_{L:.0f}m'] = {'errors': err[l, :n].cpu().numpy(), 'rmse': float(st[l, 0]),
                                    'mean': float(st[l, 1]), 'std': float(st[l, 2]), 'max': float(st[l, 3]),
                                    'num_segments': n}
        logger.info(f"RTE computation complete for {len(out)} segment lengths")
        return out

    def _find_segment_end(self, distances: np.ndarray, start_idx: int, segment_length: float) -> Optional[int]:
        end_idx = np.searchsorted(distances, distances[start_idx] + segment_length)
        return end_idx if end_idx < len(distances) else None

    def _compute_relative_transformation(self, pos1: np.ndarray, pos2: np.ndarray, quat1: np.ndarray,
                                         quat2: np.ndarray) -> np.ndarray:
        T = np.eye(4)
        T[:3, :3] = _quat_matrix(quat2) @ _quat_matrix(quat1).T
        T[:3, 3] = pos2 - pos1
        return T

    def _compute_transformation_error(self, T1: np.ndarray, T2: np.ndarray) -> float:
        T_rel = np.linalg.inv(T1) @ T2
        return float(np.sqrt(np.linalg.norm(T_rel[:3, 3]) ** 2 + np.linalg.norm(T_rel[:3, :3] - np.eye(3)) ** 2))

    # -- reporting (:363-517) ------------------------------------------------------------------------------------
    def visualize_ape_rte(self, ape_metrics: Dict, rte_metrics: Dict, timestamps: Optional[np.ndarray] = None,
                          save_path: Optional[str] = None) -> None:
        import matplotlib.pyplot as plt
        if timestamps is None:
            timestamps = np.arange(len(ape_metrics['pose_errors']))
        fig, axes = plt.subplots(2, 2, figsize=(15, 10))
        ax = axes[0, 0]
        ax.plot(timestamps, ape_metrics['position_errors'], label='Position', linewidth=2)
        ax.plot(timestamps, ape_metrics['orientation_errors'], label='Orientation', linewidth=2)
        ax.plot(timestamps, ape_metrics['pose_errors'], label='Combined', linewidth=2)
        ax.set_title('Absolute Pose Error (APE)')
        ax.legend()
        ax = axes[0, 1]
        ax.hist(ape_metrics['position_errors'], bins=30, alpha=0.7, label='Position', density=True)
        ax.hist(ape_metrics['orientation_errors'], bins=30, alpha=0.7, label='Orientation', density=True)
        ax.set_title('APE Distribution')
        ax.legend()
        lens = [float(k.split('_')[1].replace('m', '')) for k in rte_metrics if k.startswith('rte_')]
        if lens:
            axes[1, 0].errorbar(lens, [m['mean'] for k, m in rte_metrics.items() if k.startswith('rte_')],
                                yerr=[m['std'] for k, m in rte_metrics.items() if k.startswith('rte_')],
                                marker='o', capsize=5, capthick=2)
            axes[1, 0].set_title('Relative Trajectory Error (RTE)')
        axes[1, 1].axis('off')
        plt.tight_layout()
        if save_path:
            plt.savefig(save_path, dpi=150, bbox_inches='tight')
        plt.show()

    def generate_pose_error_report(self, ape_metrics: Dict, rte_metrics: Dict, save_path: Optional[str] = None) -> str:
        lines = ["# Pose Error Evaluation Report", "=" * 50, "", "## Absolute Pose Error (APE)", ""]
        for title, pre, unit in (("Position Errors", 'position', ' m'), ("Orientation Errors", 'orientation', ' rad'),
                                 ("Combined Pose Errors", 'pose', '')):
            lines.append(f"### {title}")
            lines.append(f"RMSE: {ape_metrics[f'{pre}_rmse']:.6f}{unit}")
            lines.append(f"Mean: {ape_metrics[f'{pre}_mean']:.6f}{unit}")
            lines.append(f"Std: {ape_metrics[f'{pre}_std']:.6f}{unit}")
            lines.append(f"Max: {ape_metrics[f'{pre}_max']:.6f}{unit}")
            lines.append("")
        lines += ["## Relative Trajectory Error (RTE)", ""]
        for key, m in rte_metrics.items():
            if key.startswith('rte_'):
                lines.append(f"### {key.split('_')[1].replace('m', '')}m Segments")
                lines.append(f"RMSE: {m['rmse']:.6f} m")
                lines.append(f"Mean: {m['mean']:.6f} m")
                lines.append(f"Std: {m['std']:.6f} m")
                lines.append(f"Max: {m['max']:.6f} m")
                lines.append(f"Number of segments: {m['num_segments']}")
                lines.append("")
        text = "\n".join(lines)
        if save_path:
            with open(save_path, 'w') as f:
                f.write(text)
            logger.info(f"Pose error report saved to {save_path}")
        return text


def evaluate_pose_errors(estimated_path: str, ground_truth_path: str, output_path: str,
                         timestamps_path: Optional[str] = None) -> Dict:
    """File wrapper (:520-588).  The reference imports ``os`` only under ``__main__`` (:594), so an imported module
    raises NameError on a truthy ``timestamps_path``; here (as in compute_velocity_error.py) ``os`` is imported at
    module level and the timestamps load works on both routes.  The PoseIntegrator's Euler 'orientations' [N, 3]
    give [N, 6] poses, whose quaternion columns raise ValueError, as in the reference."""
    est_d = np.load(estimated_path, allow_pickle=True)
    gt_d = np.load(ground_truth_path, allow_pickle=True)
    est = np.column_stack([est_d['positions'], est_d['orientations']])
    gt = np.column_stack([gt_d['positions'], gt_d['orientations']])
    timestamps = np.load(timestamps_path) if timestamps_path and os.path.exists(timestamps_path) else None
    ev = PoseErrorEvaluator()
    ape = ev.compute_ape(est, gt)
    rte = ev.compute_rte(est, gt, timestamps)
    report = ev.generate_pose_error_report(ape, rte, output_path.replace('.npz', '_report.md'))
    ev.visualize_ape_rte(ape, rte, timestamps, output_path.replace('.npz', '_errors.png'))
    np.savez(output_path, ape_metrics=ape, rte_metrics=rte, report=report)
    logger.info(f"Pose error evaluation complete: {output_path}")
    return {'ape_metrics': ape, 'rte_metrics': rte}


if __name__ == "__main__":
    import argparse

    p = argparse.ArgumentParser(description='Evaluate pose errors')
    p.add_argument('--est', required=True, help='Path to estimated poses')
    p.add_argument('--gt', required=True, help='Path to ground truth poses')
    p.add_argument('--out', required=True, help='Output path for evaluation')
    p.add_argument('--timestamps', help='Path to timestamps file')
    a = p.parse_args()
    res = evaluate_pose_errors(a.est, a.gt, a.out, a.timestamps)
    print(f"Pose error evaluation complete: {res['ape_metrics']['pose_rmse']:.6f}")

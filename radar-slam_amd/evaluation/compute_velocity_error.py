"""Velocity error statistics (host side).

Drop-in for ``evaluation/compute_velocity_error.py`` of the reference (``VelocityErrorEvaluator`` :22-354,
``evaluate_velocity_errors`` :357-427), imported by ``scripts/run_ego_motion_pipeline.py:37``.  Without this
module the pipeline script stops at that import once this package shadows the reference's ``evaluation``.

The work is a handful of reductions over an [N, 6] array (N = frames of one run, a few thousand at most), so it
stays on the host as numpy: a device launch would cost more than the arithmetic.  The observable
results follow the reference: per-component rmse / mae / bias / population std plus min / max / median /
quartiles (:84-111), the same over the flattened array (:115-128), the centred moving average with window
``[i - w//2, i + w//2]`` clipped to the run (:154-159), the least-squares drift slope per component (:161-166),
and the report text line for line (:197-240).  One deviation: the reference reads ``os.path`` in
``evaluate_velocity_errors`` without importing ``os`` at module level (:390), a NameError whenever a
timestamps path is given; here it works.
"""
from __future__ import annotations

import logging
import os
from typing import Dict, List, Optional

import numpy as np

logger = logging.getLogger(__name__)

_COMPONENTS = ['vx', 'vy', 'vz', 'wx', 'wy', 'wz']
_METRICS = ['rmse', 'mae', 'bias', 'std']


def _stats(e: np.ndarray, wanted: List[str]) -> Dict:
    fns = {'rmse': lambda x: np.sqrt(np.mean(x * x)), 'mae': lambda x: np.mean(np.abs(x)),
           'bias': np.mean, 'std': np.std}
    return {k: fns[k](e) for k in _METRICS if k in wanted}


class VelocityErrorEvaluator:
    def __init__(self, velocity_components: List[str] = _COMPONENTS, error_metrics: List[str] = _METRICS):
        self.velocity_components = velocity_components
        self.error_metrics = error_metrics
        logger.info("Initialized velocity error evaluator")
        logger.info(f"  Components: {velocity_components}")
        logger.info(f"  Metrics: {error_metrics}")

    def compute_velocity_errors(self, estimated_velocities: np.ndarray, ground_truth_velocities: np.ndarray,
                                timestamps: Optional[np.ndarray] = None) -> Dict:
        """Errors est - gt [N, C] and their statistics (reference :46-136)."""
        if estimated_velocities.shape != ground_truth_velocities.shape:
            raise ValueError("Estimated and ground truth velocities must have the same shape")
        n, c = estimated_velocities.shape
        if c != len(self.velocity_components):
            raise ValueError(f"Expected {len(self.velocity_components)} components, got {c}")
        errors = estimated_velocities - ground_truth_velocities
        out = {'num_samples': n, 'components': self.velocity_components, 'errors': errors,
               'estimated_velocities': estimated_velocities, 'ground_truth_velocities': ground_truth_velocities}
        if timestamps is not None:
            out['timestamps'] = timestamps
        per = {}
        for i, name in enumerate(self.velocity_components):
            e = errors[:, i]
            m = _stats(e, self.error_metrics)
            m.update(min_error=np.min(e), max_error=np.max(e), median_error=np.median(e),
                     q25_error=np.percentile(e, 25), q75_error=np.percentile(e, 75))
            per[name] = m
        out['component_metrics'] = per
        overall = _stats(errors, self.error_metrics)
        out['overall_metrics'] = overall
        logger.info(f"Computed velocity errors for {n} samples")
        logger.info(f"Overall RMSE: {overall.get('rmse', 0):.6f}")
        logger.info(f"Overall MAE: {overall.get('mae', 0):.6f}")
        return out

    def analyze_error_trends(self, error_results: Dict, window_size: int = 10) -> Dict:
        """Centred moving average, drift slope and variance per component (reference :138-180)."""
        errors = error_results['errors']
        n = len(errors)
        ts = error_results.get('timestamps', np.arange(n))
        h = window_size // 2
        # moving average through a prefix sum: window [max(0, i-h), min(n, i+h+1))
        csum = np.concatenate([np.zeros((1,) + errors.shape[1:]), np.cumsum(errors, axis=0)])
        lo = np.maximum(np.arange(n) - h, 0)
        hi = np.minimum(np.arange(n) + h + 1, n)
        moving = (csum[hi] - csum[lo]) / (hi - lo)[:, None]
        drift = np.array([np.polyfit(ts, errors[:, i], 1)[0] for i in range(errors.shape[1])])
        logger.info(f"Analyzed error trends with window size {window_size}")
        return {'moving_avg_errors': moving, 'drift_coefficients': drift,
                'error_variance': np.var(errors, axis=0), 'window_size': window_size}

    def generate_error_report(self, error_results: Dict, trend_analysis: Optional[Dict] = None,
                              save_path: Optional[str] = None) -> str:
        """Markdown report (reference :182-251)."""
        o = error_results['overall_metrics']
        lines = ["# Velocity Estimation Error Report", "=" * 50, "", "## Overall Metrics",
                 f"Number of samples: {error_results['num_samples']}"]
        lines += [f"{lab}: {o.get(k, 0):.6f}" for lab, k in (('RMSE', 'rmse'), ('MAE', 'mae'), ('Bias', 'bias'),
                                                             ('Std', 'std'))]
        lines += ["", "## Component-wise Metrics", ""]
        for name, m in error_results['component_metrics'].items():
            lines.append(f"### {name.upper()}")
            lines += [f"{lab}: {m[k]:.6f}" for lab, k in (('RMSE', 'rmse'), ('MAE', 'mae'), ('Bias', 'bias'),
                                                          ('Std', 'std'), ('Min error', 'min_error'),
                                                          ('Max error', 'max_error'),
                                                          ('Median error', 'median_error'))]
            lines.append("")
        if trend_analysis is not None:
            lines += ["## Error Trend Analysis", ""]
            for i, name in enumerate(error_results['components']):
                lines += [f"### {name.upper()}",
                          f"Drift coefficient: {trend_analysis['drift_coefficients'][i]:.6f}",
                          f"Error variance: {trend_analysis['error_variance'][i]:.6f}", ""]
        text = "\n".join(lines)
        if save_path:
            with open(save_path, 'w') as f:
                f.write(text)
            logger.info(f"Error report saved to {save_path}")
        return text

    def visualize_errors(self, error_results: Dict, trend_analysis: Optional[Dict] = None,
                         save_path: Optional[str] = None) -> None:
        """Error time series per component and the error-magnitude histogram (reference :253-309)."""
        import matplotlib.pyplot as plt
        errors = error_results['errors']
        ts = error_results.get('timestamps', np.arange(len(errors)))
        fig, axes = plt.subplots(2, 3, figsize=(15, 10))
        axes = axes.flatten()
        for i, name in enumerate(error_results['components']):
            ax = axes[i]
            ax.plot(ts, errors[:, i], alpha=0.7, linewidth=1)
            if trend_analysis is not None:
                ax.plot(ts, trend_analysis['moving_avg_errors'][:, i], 'r-', linewidth=2, label='Moving Avg')
            ax.axhline(y=0, color='k', linestyle='--', alpha=0.5)
            ax.set_xlabel('Time (s)')
            ax.set_ylabel('Error')
            ax.set_title(f'{name.upper()} Error')
            ax.grid(True, alpha=0.3)
            if trend_analysis is not None:
                ax.legend()
        ax = axes[5]   # the reference draws the histogram over the sixth panel
        ax.hist(np.linalg.norm(errors, axis=1), bins=30, alpha=0.7, edgecolor='black')
        ax.set_xlabel('Error Magnitude')
        ax.set_ylabel('Frequency')
        ax.set_title('Error Magnitude Distribution')
        ax.grid(True, alpha=0.3)
        plt.tight_layout()
        if save_path:
            plt.savefig(save_path, dpi=150, bbox_inches='tight')
        plt.show()

    def compare_velocities(self, error_results: Dict, save_path: Optional[str] = None) -> None:
        """Estimated-vs-truth scatter per component with the correlation coefficient (reference :311-354)."""
        import matplotlib.pyplot as plt
        est, gt = error_results['estimated_velocities'], error_results['ground_truth_velocities']
        fig, axes = plt.subplots(2, 3, figsize=(15, 10))
        axes = axes.flatten()
        for i, name in enumerate(error_results['components']):
            ax = axes[i]
            ax.scatter(gt[:, i], est[:, i], alpha=0.6, s=20)
            lo, hi = min(gt[:, i].min(), est[:, i].min()), max(gt[:, i].max(), est[:, i].max())
            ax.plot([lo, hi], [lo, hi], 'r--', alpha=0.8)
            ax.set_xlabel('Ground Truth')
            ax.set_ylabel('Estimated')
            ax.set_title(f'{name.upper()} Comparison')
            ax.grid(True, alpha=0.3)
            r = np.corrcoef(gt[:, i], est[:, i])[0, 1]
            ax.text(0.05, 0.95, f'R = {r:.3f}', transform=ax.transAxes, verticalalignment='top',
                    bbox=dict(boxstyle='round', facecolor='wheat'))
        plt.tight_layout()
        if save_path:
            plt.savefig(save_path, dpi=150, bbox_inches='tight')
        plt.show()


def evaluate_velocity_errors(estimated_path: str, ground_truth_path: str, output_path: str,
                             timestamps_path: Optional[str] = None) -> Dict:
    """File-level entry (reference :357-427): the pipeline's velocity .npz files -> report, plots, results .npz."""
    est_d = np.load(estimated_path, allow_pickle=True)
    gt_d = np.load(ground_truth_path, allow_pickle=True)
    est = np.column_stack([est_d['velocity'], est_d['angular_velocity']])
    gt = np.column_stack([gt_d['velocity'], gt_d['angular_velocity']])
    ts = np.load(timestamps_path) if timestamps_path and os.path.exists(timestamps_path) else None
    logger.info("Loaded velocity data:")
    logger.info(f"  Estimated: {est.shape}")
    logger.info(f"  Ground truth: {gt.shape}")
    ev = VelocityErrorEvaluator()
    res = ev.compute_velocity_errors(est, gt, ts)
    trend = ev.analyze_error_trends(res)
    report = ev.generate_error_report(res, trend, output_path.replace('.npz', '_report.md'))
    ev.visualize_errors(res, trend, output_path.replace('.npz', '_errors.png'))
    ev.compare_velocities(res, output_path.replace('.npz', '_comparison.png'))
    np.savez(output_path, error_results=res, trend_analysis=trend, report=report)
    logger.info(f"Velocity error evaluation complete: {output_path}")
    return res


if __name__ == "__main__":
    import argparse

    p = argparse.ArgumentParser(description='Evaluate velocity errors')
    p.add_argument('--est', required=True, help='Path to estimated velocities')
    p.add_argument('--gt', required=True, help='Path to ground truth velocities')
    p.add_argument('--out', required=True, help='Output path for evaluation')
    p.add_argument('--timestamps', help='Path to timestamps file')
    a = p.parse_args()
    print(f"Velocity error evaluation complete: "
          f"{evaluate_velocity_errors(a.est, a.gt, a.out, a.timestamps)['overall_metrics']}")

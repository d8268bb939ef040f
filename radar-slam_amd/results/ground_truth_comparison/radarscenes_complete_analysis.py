"""The configs[3] analyzer on MI355X: drop-in for results/ground_truth_comparison/radarscenes_complete_analysis.py
(``CompleteRadarScenesAnalyzer`` :36-491, ``main`` :494-534) of the reference.

Same constructor, attributes, methods, printed progress and result dict as the reference.  The per-frame work runs
through ``rsl.replay.SceneReplay``: every (frame, sensor) cube of the requested frames is synthesised, range-Doppler
processed, peak-selected and angle-estimated on the device in one batch, the associations of all frames come from one
launch, and each frame's Advanced solve runs on the device in order (its adaptive bounds are stateful).  The noise of
the synthetic cubes is the device generator's (Philox), statistically but not bitwise the reference's global
np.random stream; the per-frame arithmetic after the cube is checked against the reference in tests/test_replay.py.

Reference quirks kept: frames without odometry within 1 s are skipped; the association mixes metres and radians and
reuses previous targets (:274-305); a frame without a velocity estimate records the ground-truth pose as its
estimate (:226-231); and ``_compute_error_metrics`` truth-tests the converted numpy arrays (:309), so
``analyze_sequence_with_ego_motion`` ends with the reference's ValueError once a frame has been processed.
``processing_times`` are the batch's wall time split evenly over the processed frames.
"""
import json
import logging
import os
import sys
import time
from pathlib import Path
from typing import Dict, List

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from src.datasets.radarscenes_loader import RadarScenesLoader  # noqa: E402
from src.radar_signal.dechirp import SignalPreprocessor  # noqa: E402
from src.algorithms.robust_angle_estimation import RobustAngleEstimator  # noqa: E402
from src.algorithms.advanced_velocity_optimization import AdvancedVelocityOptimizer  # noqa: E402

logger = logging.getLogger(__name__)


class CompleteRadarScenesAnalyzer:
    def __init__(self, dataset_path: str):
        from rsl.replay import SceneReplay
        self.dataset_path = Path(dataset_path)
        self.loader = RadarScenesLoader(dataset_path)
        self.radar_params = {'fc': 77e9, 'bandwidth': 1e9, 'chirp_duration': 40e-6, 'pri': 100e-6, 'num_chirps': 32,
                             'num_antennas': 8, 'sampling_rate': 10e6, 'noise_power': 0.01}
        rp = self.radar_params
        self.preprocessor = SignalPreprocessor(fc=rp['fc'], bandwidth=rp['bandwidth'],
                                               chirp_duration=rp['chirp_duration'], pri=rp['pri'],
                                               num_chirps=rp['num_chirps'], sampling_rate=rp['sampling_rate'])
        self.angle_estimator = RobustAngleEstimator(fc=rp['fc'], antenna_spacing=3e8 / (2 * rp['fc']),
                                                    num_antennas=rp['num_antennas'], search_resolution=2.0,
                                                    temporal_window=3, confidence_threshold=0.6, max_targets=50)
        self.velocity_optimizer = AdvancedVelocityOptimizer(fc=rp['fc'], lambda_c=3e8 / rp['fc'],
                                                            num_antennas=rp['num_antennas'],
                                                            antenna_spacing=3e8 / (2 * rp['fc']), max_velocity=30.0,
                                                            max_angular_velocity=5.0, regularization_weight=0.01,
                                                            num_optimization_runs=2, use_parallel=False)
        # the device engine shares the analyzer's estimator state
        self.replay = SceneReplay(radar_params=rp, angle_estimator=self.angle_estimator,
                                  velocity_optimizer=self.velocity_optimizer)
        self.estimated_trajectory = []
        self.ground_truth_trajectory = []
        self.velocity_estimates = []
        self.ground_truth_velocities = []
        self.seed = 0  # device noise stream of the synthesised cubes
        logger.info("Initialized complete RadarScenes analyzer with ego-motion estimation")

    def analyze_sequence_with_ego_motion(self, sequence_id: str, max_frames: int = 5) -> Dict:
        print(f"Complete analysis of sequence: {sequence_id}")
        sequence_data = self.loader.load_sequence_data(sequence_id)
        radar_frames = self.loader.extract_radar_frames(sequence_data, frame_duration_ms=100.0)
        if max_frames:
            radar_frames = radar_frames[:max_frames]
        print(f"Processing {len(radar_frames)} frames...")
        results = {'sequence_id': sequence_id, 'frames_processed': 0, 'estimated_trajectory': [],
                   'ground_truth_trajectory': [], 'velocity_estimates': [], 'ground_truth_velocities': [],
                   'processing_times': [], 'frame_results': [], 'error_metrics': {}}
        kept, truths, idxs = [], [], []
        for frame_idx, frame_data in enumerate(radar_frames):
            gt = self.loader.get_odometry_at_time(sequence_data, frame_data['timestamp'])
            if not gt:
                continue
            sc = {sid: self.loader.convert_radar_to_scatterers(frame_data, sid) for sid in frame_data['sensors']}
            kept.append({'timestamp': frame_data['timestamp'], 'scatterers': sc})
            truths.append(gt)
            idxs.append(frame_idx)
        t0 = time.time()
        out = self.replay.run(kept, seed=self.seed) if kept else None
        per_frame = (time.time() - t0) / max(len(kept), 1)
        for n, (frame_idx, gt) in enumerate(zip(idxs, truths)):
            est = out['velocity_estimates'][n]
            tg = out['targets'][n]
            results['frames_processed'] += 1
            results['processing_times'].append(per_frame)
            gt_pose = np.array([gt['x'], gt['y'], gt['yaw']])
            results['ground_truth_trajectory'].append(gt_pose)
            if est:
                results['estimated_trajectory'].append(out['poses'][n].copy())
                results['velocity_estimates'].append(est)
            else:
                results['estimated_trajectory'].append(gt_pose)
            gt_velocity = np.array([gt['vx'], 0.0, gt['yaw_rate']])
            results['ground_truth_velocities'].append(gt_velocity)
            reliable = sum(1 for t in tg if t['is_reliable'])
            results['frame_results'].append({
                'frame_idx': frame_idx, 'timestamp': int(kept[n]['timestamp']), 'total_targets': len(tg),
                'reliable_targets': reliable, 'processing_time': per_frame, 'ground_truth_pose': gt_pose,
                'estimated_pose': out['poses'][n].copy() if est else gt_pose, 'ground_truth_velocity': gt_velocity,
                'estimated_velocity': est['velocity'] if est else gt_velocity[:3],
                'velocity_confidence': est['confidence'] if est else 0.0})
            print(f"  Frame {frame_idx + 1}: {reliable}/{len(tg)} targets, "
                  f"velocity estimate: {est is not None}, time: {per_frame:.3f}s")
        for key in ('estimated_trajectory', 'ground_truth_trajectory', 'velocity_estimates',
                    'ground_truth_velocities'):
            if results[key]:
                results[key] = np.array(results[key])
        results['error_metrics'] = self._compute_error_metrics(results)
        print(f"Sequence analysis complete: {results['frames_processed']} frames")
        return results

    def _create_target_associations(self, current_targets: List[Dict], previous_targets: List[Dict]) -> List[Dict]:
        """:274-305 for one frame pair, on the device (rsl_associate_nearest)."""
        return self.replay.associate([list(previous_targets), list(current_targets)])[1]

    def _compute_error_metrics(self, results: Dict) -> Dict:
        """:307-351, including its truth test of the converted arrays."""
        if not results['estimated_trajectory'] or not results['ground_truth_trajectory']:
            return {'error': 'No trajectory data for comparison'}
        est, gt = results['estimated_trajectory'], results['ground_truth_trajectory']
        pos_err = np.linalg.norm(est[:, :2] - gt[:, :2], axis=1)
        yaw_err = np.abs(est[:, 2] - gt[:, 2])
        vel_err = []
        if results['velocity_estimates'] and results['ground_truth_velocities']:
            for e, g in zip(results['velocity_estimates'], results['ground_truth_velocities']):
                v = e['velocity'] if isinstance(e, dict) else e
                vel_err.append(np.linalg.norm(v - g[:3]))
        if len(est) > 1 and len(gt) > 1:
            le = np.sum(np.linalg.norm(np.diff(est[:, :2], axis=0), axis=1))
            lg = np.sum(np.linalg.norm(np.diff(gt[:, :2], axis=0), axis=1))
            length_error = abs(le - lg) / max(lg, 1e-6)
        else:
            length_error = 0.0
        return {'position_rmse': np.sqrt(np.mean(pos_err ** 2)), 'position_mae': np.mean(pos_err),
                'position_max_error': np.max(pos_err), 'yaw_rmse': np.sqrt(np.mean(yaw_err ** 2)),
                'yaw_mae': np.mean(yaw_err), 'yaw_max_error': np.max(yaw_err),
                'velocity_rmse': np.sqrt(np.mean(vel_err ** 2)) if vel_err else 0.0,
                'velocity_mae': np.mean(vel_err) if vel_err else 0.0, 'trajectory_length_error': length_error,
                'successful_estimates': len([v for v in results['velocity_estimates'] if v is not None]),
                'total_frames': results['frames_processed']}

    def create_comprehensive_visualization(self, results: Dict, save_path: str = 'radarscenes_complete_analysis.png'):
        """:353-466 (plots; off the device path)."""
        import matplotlib.pyplot as plt
        fig, axes = plt.subplots(2, 3, figsize=(18, 12))
        if len(results['ground_truth_trajectory']) > 0:
            g = results['ground_truth_trajectory']
            axes[0, 0].plot(g[:, 0], g[:, 1], 'b-', linewidth=3, label='Ground Truth', marker='o')
        if len(results['estimated_trajectory']) > 0:
            e = results['estimated_trajectory']
            axes[0, 0].plot(e[:, 0], e[:, 1], 'r--', linewidth=2, label='Estimated', marker='s')
        axes[0, 0].set_title('Trajectory Comparison')
        axes[0, 0].legend()
        if len(results['estimated_trajectory']) > 0 and len(results['ground_truth_trajectory']) > 0:
            axes[0, 1].plot(np.linalg.norm(results['estimated_trajectory'][:, :2] -
                                           results['ground_truth_trajectory'][:, :2], axis=1), 'r-', marker='o')
        axes[0, 1].set_title('Position Errors Over Time')
        if results['processing_times']:
            axes[1, 1].plot(results['processing_times'], 'g-', marker='o')
        axes[1, 1].set_title('Processing Times')
        axes[1, 2].axis('off')
        plt.tight_layout()
        plt.savefig(save_path, dpi=150, bbox_inches='tight')
        plt.show()
        print(f"Comprehensive analysis visualization saved as '{save_path}'")

    def save_complete_results(self, results: Dict, output_path: str = 'radarscenes_complete_results.json'):
        """:468-491: numpy / dict / list conversion, then JSON."""
        def conv(o):
            if isinstance(o, np.integer):
                return int(o)
            if isinstance(o, np.floating):
                return float(o)
            if isinstance(o, np.ndarray):
                return o.tolist()
            if isinstance(o, dict):
                return {str(k): conv(v) for k, v in o.items()}
            if isinstance(o, list):
                return [conv(x) for x in o]
            return o
        with open(output_path, 'w') as f:
            json.dump(conv(results), f, indent=2)
        print(f"Complete analysis results saved to '{output_path}'")


def main():
    """:494-534."""
    import argparse
    ap = argparse.ArgumentParser(description='Complete RadarScenes analysis with ground truth comparison')
    ap.add_argument('--dataset', required=True, help='Path to RadarScenes dataset')
    ap.add_argument('--sequence', default='sequence_9', help='Sequence to analyze')
    ap.add_argument('--max-frames', type=int, default=5, help='Max frames to process')
    ap.add_argument('--output', default='radarscenes_complete_results.json', help='Output file for results')
    args = ap.parse_args()
    analyzer = CompleteRadarScenesAnalyzer(args.dataset)
    t0 = time.time()
    results = analyzer.analyze_sequence_with_ego_motion(args.sequence, args.max_frames)
    total = time.time() - t0
    analyzer.create_comprehensive_visualization(results)
    analyzer.save_complete_results(results, args.output)
    print(f"\nComplete analysis with ground truth comparison finished in {total:.1f}s!")
    print(f"Sequence: {results['sequence_id']}")
    print(f"Frames processed: {results['frames_processed']}")
    return results


if __name__ == "__main__":
    main()

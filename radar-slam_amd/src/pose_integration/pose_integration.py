"""Velocity-to-pose integration (host, NumPy/SciPy) for the drop-in import path.

Drop-in for ``src/pose_integration/pose_integration.py`` of the reference (``PoseIntegrator`` :23-378,
``integrate_velocities_to_pose`` :381-424).  This is the post-gather trajectory reduction (SURVEY §8f
"next" #1): it runs on the host over the gathered per-frame velocities (6 floats per frame).  The
reference's ``integrate_pose`` multiplies norm(omega)[N] by diff(t)[N-1] (:199) and therefore raises
ValueError for N >= 2; that observable behaviour is kept.
"""
from __future__ import annotations

import logging
from typing import Dict, Optional, Tuple

import numpy as np
from scipy.spatial.transform import Rotation

logger = logging.getLogger(__name__)


class PoseIntegrator:
    def __init__(self, initial_position: np.ndarray = np.array([0, 0, 0]),
                 initial_orientation: np.ndarray = np.array([0, 0, 0]), coordinate_frame: str = 'body',
                 integration_method: str = 'trapezoidal', smoothing: bool = True, smoothing_window: int = 5):
        self.initial_position = np.array(initial_position)
        self.initial_orientation = np.array(initial_orientation)
        self.coordinate_frame = coordinate_frame
        self.integration_method = integration_method
        self.smoothing = smoothing
        self.smoothing_window = smoothing_window
        self.current_position = self.initial_position.copy()
        self.current_orientation = self.initial_orientation.copy()
        self.current_rotation = Rotation.from_euler('xyz', self.initial_orientation)

    def integrate_translational_velocity(self, velocities: np.ndarray, timestamps: np.ndarray) -> np.ndarray:
        """Trapezoid / Euler running sum (:67-111), then uniform_filter1d(mode='nearest') smoothing."""
        v = np.asarray(velocities, dtype=np.float64)
        N = len(v)
        dt = np.diff(timestamps)
        if self.integration_method == 'trapezoidal':
            inc = 0.5 * dt[:, None] * (v[:-1] + v[1:])
        elif self.integration_method == 'euler':
            inc = dt[:, None] * v[:-1]
        else:
            raise ValueError(f"Unknown integration method: {self.integration_method}")
        pos = np.zeros((N, 3))
        pos[0] = self.initial_position
        for i in range(1, N):  # sequential sum, same rounding order as the reference loop
            pos[i] = pos[i - 1] + inc[i - 1]
        if self.smoothing and N > self.smoothing_window:
            from scipy.ndimage import uniform_filter1d
            for c in range(3):
                pos[:, c] = uniform_filter1d(pos[:, c], size=self.smoothing_window, mode='nearest')
        return pos

    def integrate_angular_velocity(self, angular_velocities: np.ndarray,
                                   timestamps: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """Right-multiplied rotation-vector increments (:113-167)."""
        w = np.asarray(angular_velocities, dtype=np.float64)
        N = len(w)
        ori = np.zeros((N, 3))
        ori[0] = self.initial_orientation
        rot = np.zeros((N, 3, 3))
        rot[0] = self.current_rotation.as_matrix()
        dt = np.diff(timestamps)
        for i in range(1, N):
            om = w[i - 1]
            mag = np.linalg.norm(om)
            if mag > 1e-12:
                r = Rotation.from_matrix(rot[i - 1]) * Rotation.from_rotvec((om / mag) * (mag * dt[i - 1]))
                rot[i] = r.as_matrix()
                ori[i] = r.as_euler('xyz')
            else:
                rot[i] = rot[i - 1]
                ori[i] = ori[i - 1]
        return ori, rot

    def integrate_pose(self, velocities: np.ndarray, angular_velocities: np.ndarray, timestamps: np.ndarray) -> Dict:
        N = len(velocities)
        if len(angular_velocities) != N or len(timestamps) != N:
            raise ValueError("All input arrays must have the same length")
        positions = self.integrate_translational_velocity(velocities, timestamps)
        orientations, rotations = self.integrate_angular_velocity(angular_velocities, timestamps)
        total_distance = np.sum(np.linalg.norm(np.diff(positions, axis=0), axis=1))
        # [N] * [N-1] as in the reference (:199): broadcasts only for N == 1
        total_rotation = np.sum(np.linalg.norm(angular_velocities, axis=1) * np.diff(timestamps))
        return {'timestamps': timestamps, 'positions': positions, 'orientations': orientations,
                'rotations': rotations, 'velocities': velocities, 'angular_velocities': angular_velocities,
                'total_distance': total_distance, 'total_rotation': total_rotation,
                'duration': timestamps[-1] - timestamps[0], 'num_points': N}

    def transform_to_world_frame(self, trajectory: Dict, initial_world_pose: Optional[Dict] = None) -> Dict:
        if initial_world_pose is None:
            initial_world_pose = {'position': np.array([0, 0, 0]), 'orientation': np.array([0, 0, 0])}
        p0 = initial_world_pose['position']
        r0 = Rotation.from_euler('xyz', initial_world_pose['orientation'])
        wp = np.zeros_like(trajectory['positions'])
        wo = np.zeros_like(trajectory['orientations'])
        wr = np.zeros_like(trajectory['rotations'])
        for i in range(len(trajectory['positions'])):
            wp[i] = p0 + r0.apply(trajectory['positions'][i])
            r = r0 * Rotation.from_matrix(trajectory['rotations'][i])
            wo[i] = r.as_euler('xyz')
            wr[i] = r.as_matrix()
        out = trajectory.copy()
        out.update(positions=wp, orientations=wo, rotations=wr, coordinate_frame='world')
        return out

    def visualize_trajectory(self, trajectory: Dict, save_path: Optional[str] = None,
                             show_orientation: bool = True) -> None:
        import matplotlib.pyplot as plt
        p = trajectory['positions']
        plt.figure(figsize=(8, 6))
        plt.plot(p[:, 0], p[:, 1], 'b-', linewidth=2)
        plt.axis('equal')
        if save_path:
            plt.savefig(save_path, dpi=150, bbox_inches='tight')
        plt.show()

    def save_trajectory(self, trajectory: Dict, output_path: str) -> None:
        np.savez(output_path, **trajectory)
        with open(output_path.replace('.npz', '.txt'), 'w') as f:
            f.write("# Trajectory data\n")
            f.write("# Format: timestamp, x, y, z, roll, pitch, yaw\n")
            for t, p, o in zip(trajectory['timestamps'], trajectory['positions'], trajectory['orientations']):
                f.write(f"{t:.6f}, {p[0]:.6f}, {p[1]:.6f}, {p[2]:.6f}, {o[0]:.6f}, {o[1]:.6f}, {o[2]:.6f}\n")
        logger.info(f"Trajectory saved to {output_path}")


def integrate_velocities_to_pose(velocities_path: str, output_path: str, initial_pose: Optional[Dict] = None,
                                 dt: float = 0.1) -> Dict:
    data = np.load(velocities_path, allow_pickle=True)
    v, w = data['velocity'], data['angular_velocity']
    ts = np.arange(len(v)) * dt
    integ = PoseIntegrator()
    traj = integ.integrate_pose(v, w, ts)
    if initial_pose is not None:
        traj = integ.transform_to_world_frame(traj, initial_pose)
    integ.save_trajectory(traj, output_path)
    return traj

"""Velocity-to-pose integration for the drop-in import path, on the device.

Drop-in for ``src/pose_integration/pose_integration.py`` of the reference (``PoseIntegrator`` :23-378,
``integrate_velocities_to_pose`` :381-424).  ``integrate_translational_velocity`` and
``integrate_angular_velocity`` run the fp64 prefix scans of librsl (``rsl_traj_scan``: trapezoid / Euler
positions and the quaternion product of the rotation-vector increments, with the reference's per-step
``np.diff(timestamps)``) and the ``uniform_filter1d(mode='nearest')`` smoothing (``rsl_traj_smooth``); the host
only converts the device quaternions to the reference's rotation matrices and 'xyz' Euler angles.  Like every
class of this package, it needs the HIP device (no CPU fallback).  The reference's ``integrate_pose`` multiplies
norm(omega)[N] by diff(t)[N-1] (:199) and therefore raises ValueError for N >= 2; that observable behaviour is
kept.
"""
from __future__ import annotations

import logging
from typing import Dict, Optional, Tuple

import numpy as np
from scipy.spatial.transform import Rotation

logger = logging.getLogger(__name__)

_METHODS = {'trapezoidal': 0, 'euler': 1}


def _scan(vel, nv, omega, timestamps, method):
    """Device scan of one frame sequence -> (ctx, pos [N, 3], quat [N, 4]) device tensors, pose 0 = origin / identity."""
    import torch
    import rsl
    from rsl.runtime import _ptr
    ctx = rsl.get_context()
    ts = np.ascontiguousarray(timestamps, dtype=np.float64)
    N = len(ts)
    dv = ctx.to_dev(np.ascontiguousarray(vel, dtype=np.float64).reshape(N, -1))
    dw = ctx.to_dev(np.ascontiguousarray(omega, dtype=np.float64).reshape(N, 3)) if omega is not None else None
    pos, quat = ctx.empty((N, 3), torch.float64), ctx.empty((N, 4), torch.float64)
    ctx._bind()
    ctx.check(ctx.lib.rsl_traj_scan(ctx.h, _ptr(dv), int(dv.shape[1]), int(nv), _ptr(dw), 3, _ptr(ctx.to_dev(ts)),
                                    0.0, N, method, _ptr(pos), _ptr(quat), None), 'rsl_traj_scan')
    return ctx, pos, quat


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
        """Trapezoid / Euler running sum (:67-103) as a device prefix scan, then the :105-109 smoothing."""
        if self.integration_method not in _METHODS:
            raise ValueError(f"Unknown integration method: {self.integration_method}")
        v = np.asarray(velocities, dtype=np.float64)
        N = len(v)
        if N == 0:
            np.zeros((0, 3))[0] = self.initial_position  # the reference's positions[0] = ... on an empty array
        # the reference adds velocities[i] (shape [k], or a scalar for 1-D input) to a 3-vector (:88, :97): a scalar or
        # k = 1 broadcasts to x, y, z; any other k != 3 raises numpy's broadcast error once the loop runs (N >= 2)
        v = v.reshape(N, -1) if v.ndim != 1 else v[:, None]
        k = v.shape[1]
        if k != 3:
            if k != 1 and N >= 2:
                raise ValueError(f'operands could not be broadcast together with shapes (3,) ({k},) ')
            v = np.repeat(v, 3, axis=1) if k == 1 else np.zeros((N, 3))
        ctx, pos, _ = _scan(v, 3, None, timestamps, _METHODS[self.integration_method])
        pos += ctx.torch.as_tensor(self.initial_position, dtype=ctx.torch.float64, device=pos.device)
        if self.smoothing and N > self.smoothing_window:
            from rsl.traj import smooth
            pos = smooth(ctx, pos, int(self.smoothing_window))
        return pos.cpu().numpy()

    def integrate_angular_velocity(self, angular_velocities: np.ndarray,
                                   timestamps: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """Right-multiplied rotation-vector increments (:113-167) as a device quaternion prefix product; a step
        with |omega| <= 1e-12 copies the previous orientation and rotation (:162-165)."""
        w = np.asarray(angular_velocities, dtype=np.float64).reshape(-1, 3)
        N = len(w)
        ori = np.zeros((N, 3))
        ori[0] = self.initial_orientation
        rot = np.zeros((N, 3, 3))
        rot[0] = self.current_rotation.as_matrix()
        if N < 2:
            return ori, rot
        _, _, quat = _scan(w, 0, w, timestamps, 0)
        q = quat.cpu().numpy()
        r = self.current_rotation * Rotation.from_quat(q[1:, [1, 2, 3, 0]])
        moved = np.linalg.norm(w[:-1], axis=1) > 1e-12
        src = np.maximum.accumulate(np.where(np.concatenate([[True], moved]), np.arange(N), 0))
        rot[1:] = r.as_matrix()
        ori[1:] = r.as_euler('xyz')
        rot, ori = rot[src], ori[src]  # unmoved steps repeat the last moved one (or the initial pose) exactly
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

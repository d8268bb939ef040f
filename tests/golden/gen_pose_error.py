#!/usr/bin/env python3
"""Golden vectors for APE / RTE (evaluation half): imports the REFERENCE's
evaluation/compute_pose_error.py (numpy / scipy / matplotlib only; build container only) and records
PoseErrorEvaluator.align_trajectories / compute_ape / compute_rte on synthetic trajectories.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_pose_error.py

Writes tests/golden/golden_pose_error.npz (data only: inputs and outputs).
"""
import os
import sys

import numpy as np

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))


def trajectories():
    """Deterministic (estimated, ground truth) pose pairs [N, 7]; columns 3:7 are read by the reference as
    scipy quaternions (scalar last), whatever its docstring says."""
    from scipy.spatial.transform import Rotation
    cases = {}
    rs = np.random.RandomState(125)
    # planar drive, ~1.3 km: default RTE segment lengths 100 .. 800 m
    N = 1500
    yaw = np.cumsum(0.02 * np.sin(np.arange(N) / 60.0) + 0.002 * rs.randn(N))
    v = 8.5 + 0.5 * np.sin(np.arange(N) / 90.0)
    gt_p = np.zeros((N, 3))
    gt_p[1:, 0] = np.cumsum(v[:-1] * 0.1 * np.cos(yaw[:-1]))
    gt_p[1:, 1] = np.cumsum(v[:-1] * 0.1 * np.sin(yaw[:-1]))
    gt_q = Rotation.from_euler('z', yaw).as_quat()
    off = Rotation.from_euler('z', 0.3)
    est_p = off.apply(gt_p) + np.array([4.0, -2.5, 0.0]) + np.cumsum(0.05 * rs.randn(N, 3) * [1, 1, 0], axis=0)
    est_q = (Rotation.from_euler('xyz', 0.01 * rs.randn(N, 3)) * Rotation.from_euler('z', yaw + 0.3)).as_quat()
    cases['planar'] = (np.column_stack([est_p, est_q]), np.column_stack([gt_p, gt_q]), None)
    # 3-D helix with unnormalised quaternions and short segments
    N = 600
    t = np.arange(N) * 0.05
    gt_p = np.column_stack([20 * np.cos(t / 3), 20 * np.sin(t / 3), 0.8 * t])
    gt_r = Rotation.from_euler('zyx', np.column_stack([t / 3, 0.1 * np.sin(t), 0.05 * np.cos(2 * t)]))
    Rm = Rotation.from_euler('xyz', [0.2, -0.1, 0.7])
    est_p = Rm.apply(gt_p) + [1.0, 2.0, -3.0] + 0.2 * rs.randn(N, 3)
    est_q = (Rotation.from_euler('xyz', 0.05 * rs.randn(N, 3)) * Rm * gt_r).as_quat() * rs.uniform(0.5, 2.0, (N, 1))
    cases['helix'] = (np.column_stack([est_p, est_q]), np.column_stack([gt_p, gt_r.as_quat()]),
                      [5.0, 10.0, 25.0, 50.0, 160.0])
    # short run: segment lengths past the trajectory's length give no entry
    N = 20
    gt_p = np.column_stack([np.arange(N) * 1.0, 0.1 * np.arange(N) ** 1.5, np.zeros(N)])
    gt_q = Rotation.from_euler('z', 0.05 * np.arange(N)).as_quat()
    est_p = gt_p + 0.3 * rs.randn(N, 3)
    est_q = (Rotation.from_euler('xyz', 0.1 * rs.randn(N, 3)) * Rotation.from_quat(gt_q)).as_quat()
    cases['short'] = (np.column_stack([est_p, est_q]), np.column_stack([gt_p, gt_q]), [2.0, 7.5, 100.0, 1000.0])
    return cases


def main():
    sys.dont_write_bytecode = True
    import matplotlib
    matplotlib.use('Agg')
    import logging
    logging.disable(logging.CRITICAL)
    sys.path.insert(0, REF)
    from evaluation.compute_pose_error import PoseErrorEvaluator
    out = {}
    for name, (est, gt, lens) in trajectories().items():
        ev = PoseErrorEvaluator() if lens is None else PoseErrorEvaluator(rte_segment_lengths=lens)
        out[f'{name}_est'], out[f'{name}_gt'] = est, gt
        out[f'{name}_lengths'] = np.array(ev.rte_segment_lengths, dtype=np.float64)
        aligned, T, info = ev.align_trajectories(est, gt)
        out[f'{name}_aligned'], out[f'{name}_T'] = aligned, T
        for k, v in info.items():
            out[f'{name}_info_{k}'] = np.asarray(v)
        ape = ev.compute_ape(est, gt)
        for k, v in ape.items():
            if k != 'alignment_info':
                out[f'{name}_ape_{k}'] = np.asarray(v)
        rte = ev.compute_rte(est, gt)
        out[f'{name}_rte_keys'] = np.array(list(rte.keys()))
        for key, m in rte.items():
            for k, v in m.items():
                out[f'{name}_{key}_{k}'] = np.asarray(v)
    np.savez_compressed(os.path.join(OUT, 'golden_pose_error.npz'), **out)
    print('wrote', len(out), 'arrays')


if __name__ == '__main__':
    main()

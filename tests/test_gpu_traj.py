"""GPU trajectory scans (rsl_traj_scan / stitch / apply / smooth) against the oracle restatement of
pose_integration.py:67-167 on identical inputs (fp64; tolerance 1e-12 absolute, the prefix-scan reordering)."""
import numpy as np
import pytest

import radar_oracle as O

pytestmark = pytest.mark.gpu
DT = 0.1


@pytest.mark.parametrize('F', [1, 7, 1000, 5000])
def test_reducer_steps_match_sequential_integration(ctx, F):
    import torch
    from scipy.spatial.transform import Rotation
    from rsl.traj import TrajectoryReducer
    rs = np.random.RandomState(F)
    steps = 3
    vel = rs.randn(steps * F, 2)
    om = 0.2 * rs.randn(steps * F, 3)
    red = TrajectoryReducer(ctx, F, dt=DT)
    poses = []
    for s in range(steps):
        v = ctx.to_dev(np.ascontiguousarray(vel[s * F:(s + 1) * F]))
        w = ctx.to_dev(np.ascontiguousarray(om[s * F:(s + 1) * F]))
        poses.append(red.step(v, vstride=2, nv=2, omega=w, ostride=3).cpu().numpy().copy())
    poses = np.concatenate(poses)
    ts = np.arange(steps * F) * DT
    v3 = np.concatenate([vel, np.zeros((len(vel), 1))], axis=1)
    ref = O.integrate_positions(v3, ts, smoothing=False)
    assert np.abs(poses[:, :3] - ref).max() < 1e-9 * max(1.0, np.abs(ref).max())
    rot = O.integrate_rotations(om, ts)
    q = poses[:, 3:]
    m = Rotation.from_quat(np.stack([q[:, 1], q[:, 2], q[:, 3], q[:, 0]], axis=1)).as_matrix()
    assert np.abs(m - rot).max() < 1e-9


def test_euler_and_timestamps(ctx):
    from rsl.runtime import _ptr
    import torch
    rs = np.random.RandomState(2)
    F = 300
    ts = np.cumsum(rs.uniform(0.05, 0.15, F))
    v = rs.randn(F, 3)
    pos = ctx.empty((F, 3), torch.float64)
    quat = ctx.empty((F, 4), torch.float64)
    dv, dts = ctx.to_dev(v), ctx.to_dev(ts)
    for method, name in ((0, 'trapezoidal'), (1, 'euler')):
        ctx.check(ctx.lib.rsl_traj_scan(ctx.h, _ptr(dv), 3, 3, None, 3, _ptr(dts), 0.0, F, method, _ptr(pos),
                                        _ptr(quat), None), 'scan')
        ref = O.integrate_positions(v, ts, method=name, smoothing=False)
        assert np.abs(pos.cpu().numpy() - ref).max() < 1e-11


def test_stitch_kernel_matches_host(ctx):
    from rsl.runtime import _ptr
    from rsl.traj import initial_state, stitch_host
    import torch
    rs = np.random.RandomState(9)
    R = 5
    summ = rs.randn(R, 16)
    for r in range(R):
        q = rs.randn(4)
        summ[r, 3:7] = q / np.linalg.norm(q)
    st = initial_state((1.0, 2.0, 3.0))
    for rank in range(R):
        ds, dst, db = ctx.to_dev(summ), ctx.to_dev(st), ctx.empty((7,), torch.float64)
        ctx.check(ctx.lib.rsl_traj_stitch(ctx.h, _ptr(ds), R, rank, DT, 0, _ptr(dst), _ptr(db)), 'stitch')
        hb, hs = stitch_host(summ, st, rank, DT)
        assert np.abs(db.cpu().numpy() - hb).max() < 1e-13
        assert np.abs(dst.cpu().numpy() - hs).max() < 1e-13


def test_smoothing_matches_scipy(ctx):
    from scipy.ndimage import uniform_filter1d
    from rsl.traj import smooth
    rs = np.random.RandomState(4)
    x = rs.randn(103, 3)
    for size in (5, 4, 1):
        got = smooth(ctx, ctx.to_dev(x), size).cpu().numpy()
        ref = np.stack([uniform_filter1d(x[:, c], size=size, mode='nearest') for c in range(3)], axis=1)
        assert np.abs(got - ref).max() < 1e-13

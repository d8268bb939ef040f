"""Multi-rank trajectory reduction protocol on CPU (gloo, world_size 2): per-rank block summaries, all-gather,
stitch (rsl.traj.stitch_host, the numpy mirror of k_traj_stitch) -> identical to integrating the whole frame
sequence in one process (oracle restatement of pose_integration.py:67-167)."""
import os
import socket

import numpy as np
import pytest

import radar_oracle as O

DT = 0.1


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _block_summary(v, w):
    """Local block integration (test side, via the oracle): summary as k_traj_scan's."""
    from rsl.traj import quat_mul, rotvec_quat
    F = len(v)
    ts = np.arange(F) * DT
    pos = O.integrate_positions(v, ts, smoothing=False)
    q = np.array([1.0, 0, 0, 0])
    for i in range(1, F):
        q = quat_mul(q, rotvec_quat(w[i - 1], DT))
    return np.concatenate([pos[-1], q, v[-1], v[0], w[-1]]), pos


def _worker(rank, world, port, steps, F, out):
    import torch
    import torch.distributed as dist
    from rsl.traj import initial_state, stitch_host
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    rs = np.random.RandomState(11)
    vel = rs.randn(steps * world * F, 3)
    om = 0.3 * rs.randn(steps * world * F, 3)
    state = initial_state()
    got = []
    for s in range(steps):
        g0 = (s * world + rank) * F
        summ, pos_local = _block_summary(vel[g0:g0 + F], om[g0:g0 + F])
        allsum = [torch.zeros(16, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(allsum, torch.from_numpy(summ))
        base, state = stitch_host(torch.stack(allsum).numpy(), state, rank, DT)
        mine = torch.from_numpy(pos_local + base[:3])
        allpos = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allpos, mine)
        got.append(torch.cat(allpos).numpy())
    if rank == 0:
        np.save(out, np.concatenate(got))
    dist.destroy_process_group()


def test_two_rank_trajectory_matches_single_process(tmp_path):
    import torch.multiprocessing as mp
    steps, F, world = 3, 7, 2
    out = str(tmp_path / 'pos.npy')
    mp.spawn(_worker, args=(world, _free_port(), steps, F, out), nprocs=world, join=True)
    got = np.load(out)
    rs = np.random.RandomState(11)
    vel = rs.randn(steps * world * F, 3)
    ref = O.integrate_positions(vel, np.arange(len(vel)) * DT, smoothing=False)
    assert np.abs(got - ref).max() < 1e-12


def test_stitch_rotations_match_sequential():
    """Quaternion stitching of blocks == the reference's sequential rotation composition."""
    from scipy.spatial.transform import Rotation
    from rsl.traj import initial_state, quat_mul, rotvec_quat, stitch_host
    rs = np.random.RandomState(5)
    R, F = 3, 6
    om = 0.5 * rs.randn(R * F, 3)
    v = rs.randn(R * F, 3)
    summ = []
    locq = []
    for r in range(R):
        s, _ = _block_summary(v[r * F:(r + 1) * F], om[r * F:(r + 1) * F])
        summ.append(s)
        q = [np.array([1.0, 0, 0, 0])]
        for i in range(1, F):
            q.append(quat_mul(q[-1], rotvec_quat(om[r * F + i - 1], DT)))
        locq.append(q)
    summ = np.array(summ)
    ref = O.integrate_rotations(om, np.arange(R * F) * DT)
    st = initial_state()
    for r in range(R):
        base, _ = stitch_host(summ, st, r, DT)
        for i in range(F):
            q = quat_mul(base[3:], locq[r][i])
            m = Rotation.from_quat([q[1], q[2], q[3], q[0]]).as_matrix()
            assert np.abs(m - ref[r * F + i]).max() < 1e-12


def _scipy_smooth(window):
    from scipy.ndimage import uniform_filter1d

    def f(x):
        return np.stack([uniform_filter1d(x[:, c], size=window, mode='nearest') for c in range(x.shape[1])], axis=1)
    return f


def _worker_gather(rank, world, port, steps, F, window, out):
    """The reducer's protocol as rsl.traj.TrajectoryReducer runs it, on host tensors: summaries all-gathered,
    poses gathered to rank 0 (dist.gather), rank 0 streams them through rsl.traj.StreamingSmoother."""
    import torch
    import torch.distributed as dist
    from rsl.traj import StreamingSmoother, initial_state, stitch_host
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    rs = np.random.RandomState(13)
    vel = rs.randn(steps * world * F, 3)
    om = 0.3 * rs.randn(steps * world * F, 3)
    state = initial_state()
    sm = StreamingSmoother(window, _scipy_smooth(window), np.concatenate) if rank == 0 else None
    got = []
    for s in range(steps):
        g0 = (s * world + rank) * F
        summ, pos_local = _block_summary(vel[g0:g0 + F], om[g0:g0 + F])
        allsum = [torch.zeros(16, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(allsum, torch.from_numpy(summ))
        base, state = stitch_host(torch.stack(allsum).numpy(), state, rank, DT)
        mine = torch.from_numpy(pos_local + base[:3])
        lst = [torch.zeros_like(mine) for _ in range(world)] if rank == 0 else None
        dist.gather(mine, gather_list=lst, dst=0)
        if rank == 0:
            got.append(sm.push(torch.cat(lst).numpy()))
    if rank == 0:
        got.append(sm.finalize())
        np.save(out, np.concatenate(got))
    dist.destroy_process_group()


@pytest.mark.parametrize('steps,F,window', [(3, 7, 5), (2, 1, 5), (4, 2, 4), (2, 30, 9)])
def test_two_rank_gather_and_smoothing(tmp_path, steps, F, window):
    """Poses gathered to rank 0 and smoothed across block edges (rank boundary and step boundary) == the reference's
    uniform_filter1d over the whole sequentially integrated trajectory (pose_integration.py:67-111)."""
    import torch.multiprocessing as mp
    world = 2
    out = str(tmp_path / 'pos.npy')
    mp.spawn(_worker_gather, args=(world, _free_port(), steps, F, window, out), nprocs=world, join=True)
    got = np.load(out)
    rs = np.random.RandomState(13)
    vel = rs.randn(steps * world * F, 3)
    ref = O.integrate_positions(vel, np.arange(len(vel)) * DT, smoothing=True, window=window)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() < 1e-12


def test_streaming_smoother_chunkings():
    """Every chunking of a trajectory through StreamingSmoother gives the one-shot result (or the raw trajectory
    when it has at most `window` frames, pose_integration.py:105)."""
    from rsl.traj import StreamingSmoother
    rs = np.random.RandomState(1)
    for window in (1, 2, 3, 4, 5, 8):
        for N in (1, 3, window, window + 1, 23):
            x = rs.randn(N, 3)
            ref = _scipy_smooth(window)(x) if N > window else x
            for trial in range(4):
                cuts = np.sort(rs.choice(np.arange(1, N), size=min(N - 1, trial), replace=False)) if N > 1 else []
                sm = StreamingSmoother(window, _scipy_smooth(window), np.concatenate)
                parts = [sm.push(c) for c in np.split(x, cuts)] + [sm.finalize()]
                got = np.concatenate(parts)
                assert got.shape == x.shape, (window, N, cuts)
                assert np.abs(got - ref).max() < 1e-13, (window, N, cuts)

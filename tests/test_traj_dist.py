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

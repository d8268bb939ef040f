"""The shipped rsl.TrajectoryReducer at world size 2 on the device: two fresh processes (torch
multiprocessing, spawn context: new interpreters, the pytest process is not re-executed) bind device 0, join a gloo
group and run TrajectoryReducer.step for 4 steps + finalize, i.e. rsl/traj.py's multi-rank branches as shipped: the
summary all-gather, rsl_traj_stitch / rsl_traj_apply, the pose gather to rank 0 and the rank-0 streaming smoothing.
Rank 0's trajectory is checked against the oracle restatement of pose_integration.py:67-167 over the whole
concatenated sequence (step, rank, frame): smoothed positions (integrate_positions(smoothing=True)) and rotations
(integrate_rotations) to 1e-9.

VERDICT r3 next #7: the same at world size 1 over `nccl` (RCCL) in a fresh spawned process, so the device-tensor
collective branches (`all_gather_into_tensor` of the summaries and `gather` of the poses on device tensors,
rsl/traj.py step / _gather) execute as shipped on the one GPU a box has; the test asserts the reducer took them."""
import os
import socket

import numpy as np
import pytest

import radar_oracle as O

pytestmark = pytest.mark.gpu

DT = 0.1
STEPS, F, WINDOW = 4, 37, 5


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(world):
    rs = np.random.RandomState(21)
    n = STEPS * world * F
    return rs.randn(n, 3), 0.3 * rs.randn(n, 3)


def _worker(rank, port, out, backend, world):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, 'radar-slam_amd'))
    import torch
    import torch.distributed as dist
    import rsl
    from rsl.traj import TrajectoryReducer
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if backend == 'nccl':
        dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', 0))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    ctx = rsl.get_context(0)
    vel, om = _inputs(world)
    red = TrajectoryReducer(ctx, F, dt=DT, smoothing_window=WINDOW, keep=True)
    assert red.on and red.gloo == (backend == 'gloo')  # nccl: the device-tensor collective branches
    for s in range(STEPS):
        g0 = (s * world + rank) * F
        v = ctx.to_dev(np.ascontiguousarray(vel[g0:g0 + F]))
        w = ctx.to_dev(np.ascontiguousarray(om[g0:g0 + F]))
        red.step(v, vstride=3, nv=3, omega=w, ostride=3)
    red.finalize()
    torch.cuda.synchronize()
    if rank == 0:
        pos, quat = red.trajectory()
        np.savez(out, pos=pos.cpu().numpy(), quat=quat.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('backend,world', [('gloo', 2), ('nccl', 1)])
def test_reducer_on_device(tmp_path, backend, world):
    import torch.multiprocessing as mp
    from scipy.spatial.transform import Rotation
    out = str(tmp_path / 'traj.npz')
    mp.start_processes(_worker, args=(_free_port(), out, backend, world), nprocs=world, join=True,
                       start_method='spawn')
    z = np.load(out)
    vel, om = _inputs(world)
    ts = np.arange(len(vel)) * DT
    ref_pos = O.integrate_positions(vel, ts, smoothing=True, window=WINDOW)
    ref_rot = O.integrate_rotations(om, ts)
    assert z['pos'].shape == ref_pos.shape and z['quat'].shape == (len(vel), 4)
    assert np.abs(z['pos'] - ref_pos).max() < 1e-9 * max(1.0, np.abs(ref_pos).max())
    rot = Rotation.from_quat(z['quat'][:, [1, 2, 3, 0]]).as_matrix()  # (w, x, y, z) -> scipy's scalar-last
    assert np.abs(rot - ref_rot).max() < 1e-9

"""Trajectory reduction over frame blocks: device prefix scans per block, block
stitching from 16-double summaries, one all-gather of the summaries and one all-gather of the poses.

Reference: src/pose_integration/pose_integration.py:67-167 (trapezoidal / euler positions, rotation
composition R_i = R_{i-1} * exp(omega_{i-1} dt)).  Each GPU integrates its own contiguous frame block with
``rsl_traj_scan`` (positions relative to the block's first frame, orientation quaternions relative to identity),
all ranks all-gather the block summaries over RCCL (16 doubles per rank), every rank stitches with
``rsl_traj_stitch`` (the running state carries the pose across steps), applies its block offset with
``rsl_traj_apply``, and the per-frame poses [F, 7] (x, y, z, qw, qx, qy, qz) are gathered to rank 0, which smooths
the positions (uniform_filter1d, pose_integration.py:105-109) across block edges with a streaming smoother.  These
are the only collectives of the chain: latency-bound (tens of bytes to 56 B per frame), not per-link
bandwidth-bound.

``stitch_host`` is the same stitching rule in numpy (it runs in the gloo tests on CPU and pins the kernel).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

SUMMARY = 16
STATE = 16


def quat_mul(a, b):
    """Hamilton product (w, x, y, z): composition as scipy's Rotation.__mul__."""
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return np.array([aw * bw - ax * bx - ay * by - az * bz, aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx, aw * bz + ax * by - ay * bx + az * bw])


def rotvec_quat(w, dt):
    """Rotation.from_rotvec(axis * |w| dt) with the reference's |w| > 1e-12 gate (pose_integration.py:139-151)."""
    m = float(np.sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]))
    if not m > 1e-12:
        return np.array([1.0, 0.0, 0.0, 0.0])
    s, c = np.sin(0.5 * m * dt) / m, np.cos(0.5 * m * dt)
    return np.array([c, w[0] * s, w[1] * s, w[2] * s])


def initial_state(p0=(0.0, 0.0, 0.0), q0=(1.0, 0.0, 0.0, 0.0)) -> np.ndarray:
    s = np.zeros(STATE)
    s[0:3] = p0
    s[3:7] = q0
    return s


def stitch_host(summaries: np.ndarray, state: np.ndarray, rank: int, dt: float,
                method: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """numpy mirror of k_traj_stitch: (base [7] of block `rank`, new state)."""
    p, q = state[0:3].copy(), state[3:7].copy()
    vl, wl, started = state[7:10].copy(), state[10:13].copy(), state[13] != 0.0
    base = None
    for r, s in enumerate(np.asarray(summaries).reshape(-1, SUMMARY)):
        if started:
            p = p + (0.5 * dt * (vl + s[10:13]) if method == 0 else dt * vl)
            q = quat_mul(q, rotvec_quat(wl, dt))
        if r == rank:
            base = np.concatenate([p, q])
        p = p + s[0:3]
        q = quat_mul(q, s[3:7])
        vl, wl, started = s[7:10].copy(), s[13:16].copy(), True
    new = np.zeros(STATE)
    new[0:3], new[3:7], new[7:10], new[10:13], new[13] = p, q, vl, wl, 1.0
    return base, new


class StreamingSmoother:
    """``uniform_filter1d(x[:, c], size=W, mode='nearest')`` over a trajectory that arrives in consecutive chunks
    (pose_integration.py:105-109), exact for the whole trajectory: a frame is emitted once the ``W - 1 - W // 2``
    frames to its right have arrived (the window's right half), so the chunk edges need a carried tail of the last W
    raw frames and nothing else.  The reference smooths only when the trajectory has more than W frames (:105);
    frames are therefore held back until the trajectory is longer than W, and ``finalize`` returns them unsmoothed
    when it never was.  ``smooth_fn`` smooths one contiguous [n, ncol] array with 'nearest' edges (the device kernel
    ``rsl_traj_smooth`` in the product, scipy in the CPU protocol test); ``cat_fn`` concatenates along frames."""

    def __init__(self, window: int, smooth_fn, cat_fn):
        self.W = int(window)
        self.right = self.W - 1 - self.W // 2
        self.smooth_fn, self.cat_fn = smooth_fn, cat_fn
        self.tail = None
        self.seen = 0     # raw frames pushed
        self.emitted = 0  # frames returned

    def push(self, x):
        """x [n, ncol] raw frames -> the smoothed frames that became final (possibly none)."""
        n = len(x)
        buf = x if self.tail is None else self.cat_fn([self.tail, x])
        b0 = self.seen - (len(buf) - n)          # global index of buf[0]
        self.seen += n
        self.tail = buf[-self.W:].clone() if hasattr(buf, 'clone') else buf[-self.W:].copy()
        if self.seen <= self.W:                 # not yet known whether the reference would smooth at all
            return x[:0]
        sm = self.smooth_fn(buf)
        lo, hi = self.emitted - b0, self.seen - self.right - b0
        self.emitted = self.seen - self.right
        return sm[lo:hi]

    def finalize(self):
        """The frames still held back (the right edge, 'nearest'-padded; or everything, unsmoothed, when the
        trajectory has at most W frames)."""
        if self.tail is None or self.emitted == self.seen:
            return None if self.tail is None else self.tail[:0]
        if self.seen <= self.W:
            out = self.tail[len(self.tail) - self.seen:]
        else:
            b0 = self.seen - len(self.tail)
            out = self.smooth_fn(self.tail)[self.emitted - b0:]
        self.emitted = self.seen
        return out


class TrajectoryReducer:
    """Per-rank device trajectory of consecutive frame blocks (one block per step per rank).

    Each step: ``rsl_traj_scan`` of this rank's block, all-gather of the 16-double block summaries (latency-bound),
    ``rsl_traj_stitch`` + ``rsl_traj_apply`` (absolute poses of the block), then a gather of the per-frame poses
    [F, 7] to rank 0 (``dist.gather`` = ncclSend/Recv to the root over xGMI).  Rank 0 smooths the
    positions as the reference does (``uniform_filter1d(size=smoothing_window, mode='nearest')``,
    pose_integration.py:105-109) with a ``StreamingSmoother`` on the device: the global trajectory is the
    concatenation (step, rank, frame), so a block edge is smoothed with the neighbouring block's frames, and the last
    ``W - 1 - W // 2`` frames of a step are emitted by the next step or by ``finalize``."""

    def __init__(self, ctx, frames: int, *, dt: float = 0.1, method: str = 'trapezoidal', group=None,
                 smoothing: bool = True, smoothing_window: int = 5, keep: bool = False, collective: bool = True):
        """collective=False: this rank's trajectory only, no collective even with a process group up (the bench's
        single-rank sub-measurements)."""
        import torch
        self.ctx, self.F, self.dt = ctx, int(frames), float(dt)
        self.method = 0 if method == 'trapezoidal' else 1
        e = ctx.empty
        self.pos = e((self.F, 3), torch.float64)
        self.quat = e((self.F, 4), torch.float64)
        self.summary = e((SUMMARY,), torch.float64)
        self.base = e((7,), torch.float64)
        self.state = ctx.to_dev(initial_state())
        self.group = group
        import torch.distributed as dist
        self.dist = dist
        # collectives whenever a process group is up (also at world size 1: one rank still runs the RCCL calls)
        self.on = collective and dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.on else 1
        self.rank = dist.get_rank(group) if self.on else 0
        self.gloo = self.on and dist.get_backend(group) == 'gloo'  # gloo gathers host tensors only
        self.summaries = e((self.world, SUMMARY), torch.float64)
        self.poses = e((self.F, 7), torch.float64)
        self.root = self.rank == 0
        self.all_poses = (e((self.world * self.F, 7), torch.float64) if self.on else self.poses) \
            if self.root else None
        self.smoother = StreamingSmoother(smoothing_window, lambda x: smooth(ctx, x, smoothing_window), torch.cat) \
            if (smoothing and self.root) else None
        self.smoothed = None  # rank 0: the smoothed positions that became final in the last step
        self.keep = keep
        self._hist_pos, self._hist_quat = [], []

    def step(self, vel, *, vstride: int, nv: int = 2, omega=None, ostride: int = 3):
        """vel: device f64 rows (v_x, v_y[, v_z], ...) of this rank's block.  Returns, on rank 0, all ranks' raw
        (unsmoothed) poses of this step [R*F, 7] = (x, y, z, qw, qx, qy, qz); None on the other ranks."""
        from .runtime import _ptr
        import torch
        c = self.ctx
        c._bind()
        c.check(c.lib.rsl_traj_scan(c.h, _ptr(vel), int(vstride), int(nv), _ptr(omega), int(ostride), None,
                                    self.dt, self.F, self.method, _ptr(self.pos), _ptr(self.quat),
                                    _ptr(self.summary)), 'rsl_traj_scan')
        if self.on:
            if self.gloo:
                hs = torch.empty((self.world, SUMMARY), dtype=torch.float64)
                self.dist.all_gather_into_tensor(hs.view(-1), self.summary.cpu(), group=self.group)
                self.summaries.copy_(hs)
            else:
                self.dist.all_gather_into_tensor(self.summaries.view(-1), self.summary, group=self.group)
        else:
            self.summaries[0].copy_(self.summary)
        c._bind()
        c.check(c.lib.rsl_traj_stitch(c.h, _ptr(self.summaries), self.world, self.rank, self.dt, self.method,
                                      _ptr(self.state), _ptr(self.base)), 'rsl_traj_stitch')
        c.check(c.lib.rsl_traj_apply(c.h, _ptr(self.pos), _ptr(self.quat), self.F, _ptr(self.base)), 'rsl_traj_apply')
        self.poses[:, 0:3].copy_(self.pos)
        self.poses[:, 3:7].copy_(self.quat)
        if self.on:
            self._gather()
        if not self.root:
            return None
        if self.smoother is not None:
            self.smoothed = self.smoother.push(self.all_poses[:, 0:3].contiguous())
        if self.keep:
            self._hist_pos.append(self.smoothed if self.smoother is not None else self.all_poses[:, 0:3].clone())
            self._hist_quat.append(self.all_poses[:, 3:7].clone())
        return self.all_poses

    def _gather(self):
        import torch
        if self.gloo:
            mine = self.poses.cpu()
            lst = [torch.empty_like(mine) for _ in range(self.world)] if self.root else None
            self.dist.gather(mine, gather_list=lst, dst=0, group=self.group)
            if self.root:
                self.all_poses.copy_(torch.cat(lst))
        else:
            lst = list(self.all_poses.view(self.world, self.F, 7).unbind(0)) if self.root else None
            self.dist.gather(self.poses, gather_list=lst, dst=0, group=self.group)

    def finalize(self):
        """Rank 0: the held-back last smoothed positions (see StreamingSmoother.finalize)."""
        if not self.root or self.smoother is None:
            return None
        tail = self.smoother.finalize()
        if self.keep and tail is not None:
            self._hist_pos.append(tail)
        return tail

    def trajectory(self):
        """Rank 0 with keep=True, after finalize(): (positions [N, 3], quaternions [N, 4]) of the whole run."""
        import torch
        return torch.cat(self._hist_pos), torch.cat(self._hist_quat)


def smooth(ctx, x, size: int = 5):
    """uniform_filter1d(x[:, c], size, mode='nearest') per column on the device (pose_integration.py:105-109)."""
    from .runtime import _ptr
    F, ncol = x.shape
    out = ctx.empty((F, ncol), x.dtype)
    ctx._bind()
    ctx.check(ctx.lib.rsl_traj_smooth(ctx.h, _ptr(x), F, ncol, int(size), _ptr(out)), 'rsl_traj_smooth')
    return out

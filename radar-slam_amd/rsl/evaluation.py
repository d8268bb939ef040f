"""Pose-error evaluation on the device (evaluation half): librsl's rsl_pose_align / rsl_pose_rte.

Reference: evaluation/compute_pose_error.py:51-361 (PoseErrorEvaluator).  Poses are f64 [N, 7]; columns 3:7 are
read as scipy quaternions (scalar last) exactly as the reference's Rotation.from_quat reads them.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from .runtime import Context, _ptr, get_context


def _poses(ctx, x):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    if a.ndim != 2 or a.shape[1] != 7:
        if a.ndim == 2 and a.shape[1] >= 3:  # Rotation.from_quat's message for the quaternion columns
            raise ValueError(f"Expected `quat` to have shape (4,) or (N, 4), got {a[:, 3:7].shape}.")
        raise ValueError(f"poses must be [N, 7], got {a.shape}")
    if len(a) == 0:
        raise ValueError("Found array with 0 sample(s)")
    return ctx.to_dev(a)


class PoseAlignment:
    """Device buffers of one alignment: align [32] (R 9, t 3, Rq 9, q 4, scale 1, means 6), aligned [N, 7],
    ape_err [3, N], ape_stats [3, 5] (rmse, mean, std, max, n)."""

    def __init__(self, ctx: Context, est, gt):
        import torch
        self.ctx = ctx
        self.est, self.gt = _poses(ctx, est), _poses(ctx, gt)
        n = len(self.est)
        if len(self.gt) != n:
            raise ValueError(f"operands could not be broadcast together with shapes ({n},3) ({len(self.gt)},3)")
        self.n = n
        self._scratch_for(8)
        e = ctx.empty
        self.align = e((32,), torch.float64)
        self.aligned = e((n, 7), torch.float64)
        self.ape_err = e((3, n), torch.float64)
        self.ape_stats = e((3, 5), torch.float64)
        ctx._bind()
        ctx.check(ctx.lib.rsl_pose_align(ctx.h, _ptr(self.est), _ptr(self.gt), n, _ptr(self.scratch),
                                         _ptr(self.align), _ptr(self.aligned), _ptr(self.ape_err),
                                         _ptr(self.ape_stats)), 'rsl_pose_align')

    def _scratch_for(self, nlen):
        import torch
        nb = self.ctx.lib.rsl_pose_error_scratch_bytes(self.n, max(nlen, 3))
        if getattr(self, 'scratch', None) is None or self.scratch.numel() * 8 < nb:
            self.scratch = self.ctx.empty(((nb + 7) // 8,), torch.float64)

    def rte(self, lengths: Sequence[float]):
        """-> (err [nlen, N] device, counts [nlen] host, stats [nlen, 5] host)."""
        import torch
        ctx = self.ctx
        L = np.ascontiguousarray(np.asarray(lengths, dtype=np.float64).reshape(-1))
        nlen = len(L)
        if nlen == 0:
            return None, np.zeros(0, np.int64), np.zeros((0, 5))
        self._scratch_for(nlen)
        dl = ctx.to_dev(L)
        err = ctx.empty((nlen, self.n), torch.float64)
        cnt = ctx.empty((nlen,), torch.int64)
        st = ctx.empty((nlen, 5), torch.float64)
        ctx._bind()
        ctx.check(ctx.lib.rsl_pose_rte(ctx.h, _ptr(self.aligned), _ptr(self.gt), self.n, _ptr(dl), nlen,
                                       _ptr(self.scratch), _ptr(err), _ptr(cnt), _ptr(st)), 'rsl_pose_rte')
        return err, cnt.cpu().numpy(), st.cpu().numpy()


def align_poses(est, gt, ctx: Optional[Context] = None) -> PoseAlignment:
    return PoseAlignment(ctx or get_context(), est, gt)

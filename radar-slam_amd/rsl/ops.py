"""Per-call device operations with host (numpy) inputs/outputs, used by the reference-compatible classes.

Each function uploads its operands, launches librsl kernels on the context's device, and returns numpy
arrays in the reference's dtypes (complex128 / float64 upcast from the fp32 device results where the
kernel computes in fp32).  Device tensors (torch) are accepted wherever an RDS/cube is expected and are
then used in place without a copy.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib, tables
from .runtime import Context, get_context, unpack_coord


def _ctx(ctx: Optional[Context]) -> Context:
    return ctx or get_context()


def _is_dev(x) -> bool:
    return hasattr(x, 'is_cuda') and bool(getattr(x, 'is_cuda', False))


def as_dev_c64(ctx: Context, x):
    torch = ctx.torch
    if _is_dev(x):
        return x if x.dtype == torch.complex64 else x.to(torch.complex64)
    a = np.asarray(x)
    if not np.iscomplexobj(a):
        a = a.astype(np.complex128)
    return ctx.to_dev(a.astype(np.complex64))


def to_host(t, dtype=None):
    a = t.cpu().numpy()
    return a.astype(dtype) if dtype is not None else a


# -- a3..a7 --------------------------------------------------------------------------------------------
def preprocess_rows(rows, table: np.ndarray, dc: bool, ctx: Optional[Context] = None) -> np.ndarray:
    """rows [..., S] * table[S], then optional complex-mean removal per row (dechirp.py:108,120,139)."""
    c = _ctx(ctx)
    a = np.asarray(rows)
    shape = a.shape
    S = shape[-1]
    if np.asarray(table).shape[0] != S:
        raise ValueError(f"operands could not be broadcast together with shapes ({S},) ({np.asarray(table).shape[0]},) ")
    d_in = as_dev_c64(c, a.reshape(-1, S))
    d_tab = c.to_dev(np.asarray(table, dtype=np.complex128).astype(np.complex64))
    out = c.empty(d_in.shape, c.torch.complex64)
    c._bind()
    c.check(c.lib.rsl_preprocess_rows(c.h, _ptr(d_in), d_in.shape[0], S, _ptr(d_tab), int(dc), _ptr(out)),
            'rsl_preprocess_rows')
    return to_host(out, np.complex128).reshape(shape)


def _ptr(t):
    from ctypes import c_void_p
    return None if t is None else c_void_p(t.data_ptr())


def range_doppler(frames, table: np.ndarray, *, chirp0=0, num_chirps=None, dc_removal=True,
                  ctx: Optional[Context] = None, keep_on_device=False):
    """frames [A, C, S] or [F, A, C, S] -> RDS [.., A, S, C] (c128 host, or c64 device tensor)."""
    c = _ctx(ctx)
    single = (frames.ndim == 3)
    d = as_dev_c64(c, frames)
    if single:
        d = d.unsqueeze(0)
    d = d.contiguous()
    d_tab = c.to_dev(np.asarray(table).astype(np.complex64))
    rds = c.rds(d, d_tab, chirp0=chirp0, num_chirps=num_chirps, dc_removal=dc_removal)
    if keep_on_device:
        return rds[0] if single else rds
    out = to_host(rds, np.complex128)
    return out[0] if single else out


# -- a8 -------------------------------------------------------------------------------------------------
def detect_peaks(rds, *, threshold_db=-20.0, i_lo=0, i_hi=1 << 30, want_db=True, ctx: Optional[Context] = None):
    """rds [A, S, C] -> (antenna, range_bin, doppler_bin, power_db) arrays in reference order + dB map."""
    c = _ctx(ctx)
    torch = c.torch
    d = as_dev_c64(c, rds)
    if d.dim() == 3:
        d = d.unsqueeze(0)
    d = d.contiguous()
    F, A, S, C = d.shape
    mask, rc, db = c.detect(d, tables.power_threshold(threshold_db), i_lo, i_hi, want_db=want_db)
    offs = c.offsets(mask, rc, C)
    ne = int(offs['entry_base'][F].item())
    nc = int(offs['cell_base'][F].item())
    lists = c.emit(d, mask, offs, ne, nc, want_pdb=True)
    ant, rbin, dbin = unpack_coord(to_host(lists['e_coord'][:ne]))
    res = dict(antenna=ant.astype(np.int64), range_bin=rbin.astype(np.int64), doppler_bin=dbin.astype(np.int64),
               power_db=to_host(lists['e_pdb'][:ne], np.float64),
               entry_base=to_host(offs['entry_base']), cells=nc)
    if want_db:
        res['power_spectrum_db'] = to_host(db, np.float64)
        if F == 1:
            res['power_spectrum_db'] = res['power_spectrum_db'][0]
    return res


# -- signatures as a pseudo-RDS [N, A, 1, 1] -------------------------------------------------------------
def _sig_cells(c: Context, sigs: np.ndarray):
    torch = c.torch
    s = np.atleast_2d(np.asarray(sigs))
    N, A = s.shape
    d = as_dev_c64(c, s.reshape(N, A, 1, 1)).contiguous()
    fr = c.to_dev(np.arange(N, dtype=np.int32))
    rc = c.to_dev(np.zeros(N, dtype=np.int32))
    return d, fr, rc, N


def _rds_cells(c: Context, rds, rbins, dbins):
    d = as_dev_c64(c, rds)
    if d.dim() == 3:
        d = d.unsqueeze(0)
    d = d.contiguous()
    _, A, S, C = d.shape
    rb = np.asarray(rbins, dtype=np.int64)
    db = np.asarray(dbins, dtype=np.int64)
    if rb.size and (rb.min() < 0 or rb.max() >= S or db.min() < 0 or db.max() >= C):
        raise IndexError('range/doppler bin out of bounds')
    fr = c.to_dev(np.zeros(rb.size, dtype=np.int32))
    rc = c.to_dev((rb * C + db).astype(np.int32))
    return d, fr, rc, int(rb.size)


def doa(method: str, steer_c128: np.ndarray, *, sigs=None, rds=None, rbins=None, dbins=None, want_spec=False,
        ctx: Optional[Context] = None):
    """Argmax grid index (+ optional f64 spectrum [N, G]) for MUSIC / beamforming; signatures either given
    explicitly ([N, M], normalised in-kernel as the reference does) or gathered from an RDS."""
    c = _ctx(ctx)
    if sigs is not None:
        d, fr, rc, N = _sig_cells(c, sigs)
    else:
        d, fr, rc, N = _rds_cells(c, rds, rbins, dbins)
    if N == 0:
        return np.zeros(0, np.int64), (np.zeros((0, steer_c128.shape[0])) if want_spec else None)
    st = c.steering(steer_c128)
    m = _lib.METHOD_MUSIC if method == 'music' else _lib.METHOD_BEAMFORMING
    idx, _, spec = c.doa(d, fr, rc, st, m, n=N, want_spec=want_spec)
    return to_host(idx[:N]).astype(np.int64), (to_host(spec[:N], np.float64) if want_spec else None)


def subspace_music(sigs, steer_c128: np.ndarray, num_sources: int, ctx: Optional[Context] = None) -> np.ndarray:
    """MUSIC spectrum f64 [n, G] for any num_sources (angle_estimation.py:109-154; rsl_music_subspace)."""
    c = _ctx(ctx)
    s = np.ascontiguousarray(np.atleast_2d(np.asarray(sigs, dtype=np.complex128)))
    st = np.ascontiguousarray(np.asarray(steer_c128, dtype=np.complex128))
    n, M = s.shape
    G = st.shape[0]
    ds, dst = c.to_dev(s.view(np.float64)), c.to_dev(st.view(np.float64))
    out = c.empty((n, G), c.torch.float64)
    c._bind()
    c.check(c.lib.rsl_music_subspace(c.h, _ptr(ds), n, M, int(num_sources), _ptr(dst), G, _ptr(out)),
            'rsl_music_subspace')
    return to_host(out)


def subspace_esprit(sigs, num_sources: int, esprit_scale: float, ctx: Optional[Context] = None) -> np.ndarray:
    """ESPRIT angles (deg) f64 [n] for any num_sources (angle_estimation.py:178-225; rsl_esprit_subspace)."""
    c = _ctx(ctx)
    s = np.ascontiguousarray(np.atleast_2d(np.asarray(sigs, dtype=np.complex128)))
    n, M = s.shape
    ds = c.to_dev(s.view(np.float64))
    out = c.empty((n,), c.torch.float64)
    c._bind()
    c.check(c.lib.rsl_esprit_subspace(c.h, _ptr(ds), n, M, int(num_sources), float(esprit_scale), _ptr(out)),
            'rsl_esprit_subspace')
    return to_host(out)


def cell_extras(*, sigs=None, rds=None, rbins=None, dbins=None, esprit_scale=1 / math.pi, want_sig=False,
                want_esprit=False, want_phase=False, ctx: Optional[Context] = None):
    c = _ctx(ctx)
    if sigs is not None:
        d, fr, rc, N = _sig_cells(c, sigs)
    else:
        d, fr, rc, N = _rds_cells(c, rds, rbins, dbins)
    if N == 0:
        A = d.shape[1]
        return (np.zeros((0, A), np.complex128) if want_sig else None, np.zeros(0) if want_esprit else None,
                np.zeros(0) if want_phase else None)
    sig, esp, ph, _ = c.cell_extras(d, fr, rc, n=N, esprit_scale=esprit_scale, want_sig=want_sig,
                                    want_esprit=want_esprit, want_phase=want_phase)
    return (to_host(sig[:N], np.complex128) if want_sig else None, to_host(esp[:N]) if want_esprit else None,
            to_host(ph[:N]) if want_phase else None)


def confidence(sigs, az_deg: Sequence[float], antenna_positions, lambda_c, ctx: Optional[Context] = None):
    """compute_angle_confidence for N (signature, angle) pairs (robust_angle_estimation.py:88-138)."""
    c = _ctx(ctx)
    d, fr, rc, N = _sig_cells(c, sigs)
    az = np.atleast_1d(np.asarray(az_deg, dtype=np.float64))
    steer = tables.steering_matrix(az, np.asarray(antenna_positions), lambda_c)
    st = c.steering(steer)
    gi = c.to_dev(np.arange(N, dtype=np.int32))
    conf = c.confidence(d, fr, rc, gi, st, N)
    return to_host(conf[:N])


def phase_model(pos, ang, x6, k, y=None, wrap=False, ridge=0.0, ctx: Optional[Context] = None):
    c = _ctx(ctx)
    pos = np.ascontiguousarray(np.asarray(pos, np.float64).reshape(-1, 3))
    ang = np.ascontiguousarray(np.asarray(ang, np.float64).reshape(-1, 2))
    n = pos.shape[0]
    torch = c.torch
    dp, da = c.to_dev(pos.reshape(-1) if n else np.zeros(3)), c.to_dev(ang.reshape(-1) if n else np.zeros(2))
    dx = c.to_dev(np.asarray(x6, np.float64).reshape(6))
    dy = c.to_dev(np.asarray(y, np.float64)) if y is not None and n else None
    pred = c.empty((max(n, 1),), torch.float64)
    resid = c.empty((max(n, 1),), torch.float64) if dy is not None else None
    cost = c.empty((1,), torch.float64) if dy is not None else None
    c._bind()
    c.check(c.lib.rsl_phase_model(c.h, _ptr(dp), _ptr(da), n, _ptr(dx), float(k), _ptr(dy), int(wrap), float(ridge),
                                  _ptr(pred), _ptr(resid), _ptr(cost)), 'rsl_phase_model')
    out = dict(pred=to_host(pred[:n]))
    if dy is not None:
        out['resid'] = to_host(resid[:n])
        out['cost'] = float(cost.item())
    return out


def bvls(pos, ang, y, k, lo, hi, ridge=0.0, ctx: Optional[Context] = None):
    """Exact box-constrained linear LS of the 3- or 6-DoF phase model; returns (x, cost)."""
    c = _ctx(ctx)
    pos = np.ascontiguousarray(np.asarray(pos, np.float64).reshape(-1, 3))
    ang = np.ascontiguousarray(np.asarray(ang, np.float64).reshape(-1, 2))
    n = pos.shape[0]
    nv = len(lo)
    torch = c.torch
    dp, da, dy = c.to_dev(pos.reshape(-1)), c.to_dev(ang.reshape(-1)), c.to_dev(np.asarray(y, np.float64))
    dlo, dhi = c.to_dev(np.asarray(lo, np.float64)), c.to_dev(np.asarray(hi, np.float64))
    out = c.empty((nv + 1,), torch.float64)
    c._bind()
    c.check(c.lib.rsl_bvls(c.h, _ptr(dp), _ptr(da), n, _ptr(dy), float(k), nv, float(ridge), _ptr(dlo), _ptr(dhi),
                           _ptr(out)), 'rsl_bvls')
    o = to_host(out)
    return o[:nv], float(o[nv])


# -- a30 / a31: cross-frame association and wrapped-phase solve ------------------------------------------
def associate(cur_xy, prev_xy, thr: float, ctx: Optional[Context] = None):
    """Greedy nearest-unused association (velocity_solver_improved.py:74-129) on the device.
    Returns (match int64 [Nc] with -1 for none, dist float64 [Nc])."""
    c = _ctx(ctx)
    torch = c.torch
    cur = np.ascontiguousarray(np.asarray(cur_xy, np.float64).reshape(-1, 2))
    prev = np.ascontiguousarray(np.asarray(prev_xy, np.float64).reshape(-1, 2))
    nc, npv = cur.shape[0], prev.shape[0]
    if nc == 0:
        return np.zeros(0, np.int64), np.zeros(0)
    dc = c.to_dev(cur.reshape(-1))
    dp = c.to_dev(prev.reshape(-1)) if npv else None
    scratch = c.empty((max((npv + 31) // 32, 1),), torch.int32)
    match = c.empty((nc,), torch.int32)
    dist = c.empty((nc,), torch.float64)
    c._bind()
    c.check(c.lib.rsl_associate(c.h, _ptr(dc), nc, _ptr(dp), npv, float(thr), _ptr(scratch), _ptr(match), _ptr(dist)),
            'rsl_associate')
    return to_host(match).astype(np.int64), to_host(dist)


def wrapped_solve(pos, ang, y, k, *, mode: int, lo, hi, nv: int = 6, w: float = 0.01, vmax: float = 50.0,
                  wmax: float = 10.0, prev=None, extra=None, grid_n: int = 512, iters: int = 12,
                  ctx: Optional[Context] = None):
    """Global minimisation of the wrapped-phase cost (rsl_wrapped_solve): mode 0 = Improved regularisation,
    mode 1 = Advanced penalties.  Returns (x6, cost)."""
    from ctypes import c_double
    c = _ctx(ctx)
    torch = c.torch
    pos = np.ascontiguousarray(np.asarray(pos, np.float64).reshape(-1, 3))
    ang = np.ascontiguousarray(np.asarray(ang, np.float64).reshape(-1, 2))
    n = pos.shape[0]
    ex = None if extra is None else np.ascontiguousarray(np.asarray(extra, np.float64).reshape(-1, 6))
    nextra = 0 if ex is None else ex.shape[0]
    nbytes = int(c.lib.rsl_wrapped_scratch_bytes(n, grid_n, nextra))
    scratch = c.empty(((nbytes + 7) // 8,), torch.float64)
    dp, da, dy = c.to_dev(pos.reshape(-1)), c.to_dev(ang.reshape(-1)), c.to_dev(np.asarray(y, np.float64))
    dprev = c.to_dev(np.asarray(prev, np.float64).reshape(6)) if prev is not None else None
    dex = c.to_dev(ex.reshape(-1)) if nextra else None
    out = c.empty((8,), torch.float64)
    lo6 = (c_double * 6)(*[float(v) for v in lo])
    hi6 = (c_double * 6)(*[float(v) for v in hi])
    c._bind()
    c.check(c.lib.rsl_wrapped_solve(c.h, _ptr(dp), _ptr(da), n, _ptr(dy), float(k), int(mode), float(w), float(vmax),
                                    float(wmax), _ptr(dprev), lo6, hi6, int(nv), int(grid_n), _ptr(dex), nextra,
                                    int(iters), _ptr(scratch), nbytes, _ptr(out)), 'rsl_wrapped_solve')
    o = to_host(out)
    return o[:6].copy(), float(o[6])


def wrapped_search(pos, ang, y, k, *, mode: int, lo, hi, nv: int = 6, w: float = 0.01, vmax: float = 50.0,
                   wmax: float = 10.0, prev=None, extra=None, spacing_frac: float = 0.5, nbest: int = 64,
                   iters: int = 12, ctx: Optional[Context] = None):
    """Basin-resolving global minimisation of the wrapped-phase cost (rsl_wrapped_search): 2-D Gauss-Newton in
    (v_x, v_y) from a grid whose spacing is spacing_frac of the wrap period 2 pi / k, then the nv-D refinement from the
    nbest best basins and the extra starts.  Returns (x6, cost)."""
    from ctypes import c_double
    c = _ctx(ctx)
    torch = c.torch
    pos = np.ascontiguousarray(np.asarray(pos, np.float64).reshape(-1, 3))
    ang = np.ascontiguousarray(np.asarray(ang, np.float64).reshape(-1, 2))
    n = pos.shape[0]
    ex = None if extra is None else np.ascontiguousarray(np.asarray(extra, np.float64).reshape(-1, 6))
    nextra = 0 if ex is None else ex.shape[0]
    lo6 = (c_double * 6)(*[float(v) for v in lo])
    hi6 = (c_double * 6)(*[float(v) for v in hi])
    # x[2..5] during the 2-D stage: the regulariser's optimum for them (0; with a previous motion, Advanced's temporal
    # term w 0.1 |x - prev|^2 against 10 w v_z^2: v_z = prev_z / 101, w = prev_w)
    base = np.zeros(6)
    if prev is not None and mode == 1:
        p = np.asarray(prev, np.float64).reshape(6)
        base[2] = p[2] * 0.1 / 10.1
        base[3:] = p[3:] if nv == 6 else 0.0
    b6 = (c_double * 6)(*[float(v) for v in base])
    # at least 64 points per axis (a smooth landscape when k is small, e.g. the pipeline's lambda = fc / c); the width
    # of a collapsed axis (adaptive bounds with lo == hi) does not count: that axis gets one point (search_grid), and
    # the other keeps its own spacing instead of a 32768-point line of starts
    widths = [w for w in (float(hi[0]) - float(lo[0]), float(hi[1]) - float(lo[1])) if w > 1e-9]
    width = min(widths) if widths else 1e-9
    spacing = min(float(spacing_frac) * 2 * math.pi / abs(float(k)), width / 64)
    nbytes = int(c.lib.rsl_wrapped_search_scratch_bytes(n, lo6, hi6, spacing, int(nbest), nextra))
    if nbytes < 0:
        raise ValueError('rsl_wrapped_search_scratch_bytes: bad arguments')
    scratch = c.empty(((nbytes + 7) // 8,), torch.float64)
    dp, da, dy = c.to_dev(pos.reshape(-1)), c.to_dev(ang.reshape(-1)), c.to_dev(np.asarray(y, np.float64))
    dprev = c.to_dev(np.asarray(prev, np.float64).reshape(6)) if prev is not None else None
    dex = c.to_dev(ex.reshape(-1)) if nextra else None
    out = c.empty((8,), torch.float64)
    c._bind()
    c.check(c.lib.rsl_wrapped_search(c.h, _ptr(dp), _ptr(da), n, _ptr(dy), float(k), int(mode), float(w), float(vmax),
                                     float(wmax), _ptr(dprev), lo6, hi6, int(nv), b6, spacing, int(nbest), _ptr(dex),
                                     nextra, int(iters), _ptr(scratch), nbytes, _ptr(out)), 'rsl_wrapped_search')
    o = to_host(out)
    return o[:6].copy(), float(o[6])

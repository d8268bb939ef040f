"""Parity comparators (CPU, numpy): explain every GPU/oracle difference by an fp32 near-tie of the
reference's own fp64 values, or report it as unexplained.  Tolerances are stated here once:

* RDS:      max |rds_gpu - rds_ref| <= RDS_ATOL_REL * max |rds_ref|           (c64 chain measured 1.6e-7)
* peaks:    set equality, except cells whose reference decision margin is below PEAK_RTOL
            (|p - max_neighbour| or |p - threshold| relative to p), which fp32 cannot resolve
* DoA:      same grid index, or a different index whose reference |a^H s|^2 is within DOA_RGAP relative of
            the reference maximum, (g_ref_max - g_ref[gpu_idx]) / g_ref_max < 1e-6 (an fp32 near-tie,
            or the +-90 deg alias, whose gap is 0); the number of such flips is asserted against
            DOA_FLIP_FRAC * N_cells (each flip is a 0.5 deg miss, so it is counted, not just explained)
  Of those flips none may be scan-caused (scan_flips): the GPU index must be the fp64 argmax of the
            GPU's own fp32 signature, up to fp64-level ties (relative gap <= OWN_TIE_RGAP, e.g. the +-90 deg alias);
            the remaining flips are RDS-caused (the fp32 RDS itself moves the argmax)
* ESPRIT:   |deg_gpu - deg_ref| <= ESPRIT_TOL_DEG (= 1e-3 rad, the north-star DoA tolerance)
* velocity: cost within VEL_COST_RTOL relative; (v_x, v_y) within VEL_ATOL m/s when well conditioned
"""
import numpy as np

import radar_oracle as O

RDS_ATOL_REL = 1e-5
PEAK_RTOL = 2e-5
DOA_RGAP = 1e-6
DOA_FLIP_FRAC = 2e-4
OWN_TIE_RGAP = 1e-13
ESPRIT_TOL_DEG = float(np.degrees(1e-3))
VEL_COST_RTOL = 1e-6
VEL_ATOL = 1e-4


def rds_error(gpu, ref):
    return float(np.abs(gpu - ref).max() / np.abs(ref).max())


def _neighbour_max(p):
    A, S, C = p.shape
    pad = np.full((A, S + 2, C + 2), -np.inf)
    pad[:, 1:-1, 1:-1] = p
    m = np.full(p.shape, -np.inf)
    for di in (-1, 0, 1):
        for dj in (-1, 0, 1):
            if di == 0 and dj == 0:
                continue
            m = np.maximum(m, pad[:, 1 + di:1 + di + S, 1 + dj:1 + dj + C])
    return m


def peak_diff(gpu_mask, ref_rds, *, threshold_db=-20.0, gate=(0, 1 << 30)):
    """gpu_mask bool [A, S, C].  Returns (n_gpu, n_ref, n_diff, n_unexplained)."""
    ref_mask, _ = O.peak_mask(ref_rds, threshold_db)
    A, S, C = ref_rds.shape
    g = np.zeros(S, bool)
    g[max(gate[0], 0):min(gate[1], S - 1) + 1] = True
    ref_mask &= g[None, :, None]
    diff = gpu_mask ^ ref_mask
    p = np.abs(ref_rds) ** 2
    nb = _neighbour_max(p)
    thr = 10 ** (threshold_db / 10) - 1e-12
    near_max = np.abs(p - nb) <= PEAK_RTOL * np.maximum(p, nb)
    near_thr = np.abs(p - thr) <= PEAK_RTOL * thr
    unexpl = diff & ~(near_max | near_thr)
    return int(gpu_mask.sum()), int(ref_mask.sum()), int(diff.sum()), int(unexpl.sum())


def doa_flip_budget(n_cells, num_antennas=8, search_resolution=0.5):
    """Largest accepted number of explained flips among n_cells cells: DOA_FLIP_FRAC per cell for an 8-element
    array on the reference's 0.5-degree grid, scaled by 8 / M for smaller arrays (the beam, and with it the band of
    grid points whose power lies within fp32 rounding of the maximum, widens as 1 / M) and by 0.5 / resolution for
    finer grids (more grid points in that band; tests/test_gpu_sweep.py measured 5 / 15692 at 0.25 degrees).  Measured on MI355X (r2): cfg2 4 / 60000 (6.7e-5), a4 (M = 4)
    3 / 10502 (2.9e-4), cfg5 1 / 30000; every flip's reference relative gap <= 8.7e-8."""
    return max(3, int(DOA_FLIP_FRAC * n_cells * max(1.0, 8.0 / num_antennas) * max(1.0, 0.5 / search_resolution)))


def doa_diff(gpu_idx, ref_sigs, steer, method='music', stats=None):
    """gpu_idx [N] grid indices; ref_sigs c128 [N, M] (unit norm, from the fp64 reference RDS).
    Returns (n_mismatch, n_unexplained, ref_idx); with ``stats`` (a dict) also accumulates the largest relative
    gap of an explained flip ('max_rgap') and the alias flips (+-90 deg, gap 0) ('alias')."""
    g = np.abs(ref_sigs @ steer.conj().T) ** 2
    if method == 'music':
        spec = O.music_spectrum_closed(ref_sigs, steer)
        ref_idx = np.argmax(spec, axis=1)
    else:
        ref_idx = np.argmax(g, axis=1)
    n = np.arange(len(gpu_idx))
    mism = gpu_idx != ref_idx
    gref = g[n, ref_idx]
    rgap = (gref - g[n, gpu_idx]) / np.where(gref > 0, gref, 1.0)
    explained = rgap < DOA_RGAP
    if stats is not None and mism.any():
        stats['max_rgap'] = max(stats.get('max_rgap', 0.0), float(rgap[mism].max()))
        stats['alias'] = stats.get('alias', 0) + int((mism & (rgap == 0)).sum())
    return int(mism.sum()), int((mism & ~explained).sum()), ref_idx


def esprit_diff(gpu_deg, ref_deg):
    both_nan = np.isnan(gpu_deg) & np.isnan(ref_deg)
    d = np.abs(gpu_deg - ref_deg)
    d[both_nan] = 0
    return float(np.nanmax(d) if d.size else 0.0), int((np.isnan(gpu_deg) != np.isnan(ref_deg)).sum())


def scan_flips(gpu_idx, gpu_sigs, steer, method='music'):
    """Scan-caused flips: cells whose GPU grid index is not the fp64 argmax of the GPU's OWN signature (gpu_sigs: the
    fp32 RDS values of each cell, any scale), beyond fp64-level ties (gap <= OWN_TIE_RGAP relative).  Returns
    (count, largest relative gap among them)."""
    if len(gpu_idx) == 0:
        return 0, 0.0
    gs = np.asarray(gpu_sigs, np.complex128)
    nrm = np.linalg.norm(gs, axis=1, keepdims=True)
    gs = gs / np.where(nrm > 0, nrm, 1.0)
    g = np.abs(gs @ steer.conj().T) ** 2
    own = np.argmax(O.music_spectrum_closed(gs, steer), axis=1) if method == 'music' else np.argmax(g, axis=1)
    n = np.arange(len(gpu_idx))
    go = g[n, own]
    rgap = (go - g[n, gpu_idx]) / np.where(go > 0, go, 1.0)
    bad = (gpu_idx != own) & (rgap > OWN_TIE_RGAP)
    return int(bad.sum()), float(rgap[bad].max()) if bad.any() else 0.0


def spectrum_argmax_consistent(spec, idx, method='music', atol=2e-5):
    """The grid index is a maximum of the written f32 spectrum up to the scan's precision: exactly the f16 scan's
    argmax where its top-2 gap is clear, the fp64 argmax of the cell's signature where it was re-scanned (a near-tie
    inside the scan's 1e-6 bound), so the written value there is within the den / power tolerance of the row max."""
    n = np.arange(len(idx))
    if method == 'music':
        d = np.where(spec > 0, 1.0 / np.where(spec > 0, spec, 1.0), np.inf)
        return bool(((d[n, idx] - d.min(axis=1)) <= atol).all())
    return bool(((spec.max(axis=1) - spec[n, idx]) <= atol).all())

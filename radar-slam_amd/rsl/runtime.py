"""Device runtime: one librsl handle per (device, stream), torch tensors as device memory (plumbing).

Every function here launches HIP kernels of librsl.so on torch's current stream of the context's
device.  There is no CPU path: constructing a Context without a HIP device raises RuntimeError.
"""
from __future__ import annotations

import ctypes
import math
import threading
from ctypes import byref, c_double, c_float, c_int, c_longlong, c_void_p
from typing import Dict, Optional

import numpy as np

from . import _lib
from . import tables

_P = c_void_p


def unpack_coord(coord: np.ndarray):
    """Host unpack of the emit's packed entries (include/rsl.h RSL_COORD_*): antenna, range_bin, doppler_bin."""
    u = np.asarray(coord).view(np.uint32)
    return ((u >> 26).astype(np.int32), ((u >> 13) & 0x1fff).astype(np.int32), (u & 0x1fff).astype(np.int32))


_HIP = None


def _hip():
    """The HIP runtime (libamdhip64, already loaded by torch-ROCm) for the few calls torch does not expose."""
    global _HIP
    if _HIP is None:
        h = ctypes.CDLL('libamdhip64.so')
        h.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(c_void_p), ctypes.c_size_t, ctypes.c_uint]
        h.hipExtMallocWithFlags.restype = c_int
        h.hipFree.argtypes = [c_void_p]
        h.hipFree.restype = c_int
        _HIP = h
    return _HIP


class _DeviceBlock:
    """Owner of a raw device allocation exposed to torch through __cuda_array_interface__ (torch keeps this object
    alive as long as the tensor's storage; hipFree when it goes)."""
    _TYPESTR = {'float32': '<f4', 'float64': '<f8', 'int32': '<i4', 'int64': '<i8', 'complex64': '<c8', 'uint8': '|u1'}

    def __init__(self, ptr, nbytes, shape, dtype, hip):
        self.ptr, self.nbytes, self.hip = ptr, nbytes, hip
        self.__cuda_array_interface__ = {'shape': tuple(int(d) for d in shape),
                                         'typestr': self._TYPESTR[str(dtype).replace('torch.', '')],
                                         'data': (ptr, False), 'version': 2, 'strides': None}

    def __del__(self):
        if self.ptr:
            self.hip.hipFree(c_void_p(self.ptr))
            self.ptr = 0


def _ptr(t) -> Optional[c_void_p]:
    if t is None:
        return None
    return c_void_p(t.data_ptr())


class Context:
    """A librsl handle bound to one HIP device; launches go to torch's current stream."""

    def __init__(self, device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("rsl: no HIP device visible — the MI355X product path has no CPU fallback")
        self.torch = torch
        self.lib = _lib.load()
        self.device = torch.device('cuda', device)
        h = c_void_p()
        rc = self.lib.rsl_create(byref(h), device)
        if rc != 0:
            raise RuntimeError(f"rsl_create(device={device}) failed with code {rc}")
        self.h = h
        self._steer_cache: Dict = {}

    def __del__(self):
        try:
            if getattr(self, 'h', None):
                self.lib.rsl_destroy(self.h)
        except Exception:
            pass

    # -- plumbing -------------------------------------------------------------------------------
    def _bind(self):
        s = self.torch.cuda.current_stream(self.device).cuda_stream
        self.lib.rsl_set_stream(self.h, c_void_p(s))

    def check(self, rc: int, what: str):
        if rc == 0:
            return
        msg = self.lib.rsl_last_error(self.h).decode(errors='replace')
        if rc in (_lib.RSL_ERR_INVALID, _lib.RSL_ERR_UNSUPPORTED):
            raise ValueError(f"{what}: {msg}")
        raise RuntimeError(f"{what}: {msg}")

    def empty(self, shape, dtype):
        return self.torch.empty(shape, dtype=dtype, device=self.device)

    def empty_contiguous(self, shape, dtype):
        """A device tensor in its own physically contiguous allocation (hipExtMallocWithFlags with
        hipDeviceMallocContiguous), freed when the tensor goes away; None when the driver cannot provide it.  For the
        large streamed outputs whose store rate depends on how the VRAM manager backs them (the configs[1] spectrum:
        DESIGN §5)."""
        torch = self.torch
        n = 1
        for d in shape:
            n *= int(d)
        nbytes = n * torch.empty((), dtype=dtype).element_size()
        hip = _hip()
        p = c_void_p()
        torch.cuda.set_device(self.device)
        if hip.hipExtMallocWithFlags(byref(p), ctypes.c_size_t(max(nbytes, 1)), 0x4) != 0 or not p.value:
            hip.hipGetLastError()
            return None
        owner = _DeviceBlock(p.value, nbytes, shape, dtype, hip)
        return torch.as_tensor(owner, device=self.device)

    def to_dev(self, arr: np.ndarray, dtype=None):
        t = self.torch.from_numpy(np.ascontiguousarray(arr))
        if dtype is not None:
            t = t.to(dtype)
        return t.to(self.device, non_blocking=False)

    def sync(self):
        self._bind()
        self.check(self.lib.rsl_sync(self.h), 'rsl_sync')

    # -- timing ---------------------------------------------------------------------------------
    def timing(self, on: bool = True):
        self.lib.rsl_timing_enable(self.h, int(on))

    def timing_reset(self):
        self.lib.rsl_timing_reset(self.h)

    def timing_read(self) -> Dict[str, tuple]:
        out = {}
        for k, name in enumerate(_lib.K_NAMES):
            ms, n = c_double(), c_longlong()
            self.lib.rsl_timing_read(self.h, k, byref(ms), byref(n))
            out[name] = (ms.value, n.value)
        return out

    def timing_spans(self) -> Dict[str, list]:
        """Per kernel id: [(start_ms, end_ms), ...] of every launch since timing_reset, on one device clock (ms after
        the reset's reference event), in launch order."""
        out = {}
        if not hasattr(self.lib, 'rsl_timing_spans'):  # an older library under RSL_LIBRARY (A/B runs)
            return out
        for k, name in enumerate(_lib.K_NAMES):
            n = self.lib.rsl_timing_spans(self.h, k, 0, None, None)
            if n > 0:
                a, b = (c_double * n)(), (c_double * n)()
                self.lib.rsl_timing_spans(self.h, k, n, a, b)
                out[name] = list(zip(a, b))
        return out

    # -- a7 -------------------------------------------------------------------------------------
    def rds(self, cube, table, *, chirp0: int = 0, num_chirps: Optional[int] = None, dc_removal: bool = True,
            out=None, work=None):
        """cube complex64 [F, A, Ct, S] (device) -> rds complex64 [F, A, S, C]."""
        torch = self.torch
        F, A, Ct, S = cube.shape
        C = Ct - chirp0 if num_chirps is None else num_chirps
        if out is None:
            out = self.empty((F, A, S, C), torch.complex64)
        if work is None:
            work = self.empty((F, A, C, S), torch.complex64)
        self._bind()
        self.check(self.lib.rsl_rds(self.h, _ptr(cube), F, A, Ct, chirp0, C, S, _ptr(table), int(dc_removal),
                                    _ptr(work), _ptr(out)), 'rsl_rds')
        return out

    # -- a7 + a8 fused -----------------------------------------------------------------------------
    def rds_detect(self, cube, table, thr_power: float, i_lo: int, i_hi: int, *, rds, work, mask, row_count,
                   peak_pow=None, db_map=None, chirp0: int = 0, num_chirps: Optional[int] = None,
                   dc_removal: bool = True):
        """cube [F, A, Ct, S] -> rds [F, A, S, C] + detection outputs, Doppler FFT and detection in one kernel.
        Returns the row grouping of ``peak_pow`` (pass it to ``emit``)."""
        F, A, Ct, S = cube.shape
        C = Ct - chirp0 if num_chirps is None else num_chirps
        group = ctypes.c_int(1)
        self._bind()
        self.check(self.lib.rsl_rds_detect(self.h, _ptr(cube), F, A, Ct, chirp0, C, S, _ptr(table),
                                           int(dc_removal), _ptr(work), _ptr(rds), float(thr_power), int(i_lo),
                                           int(i_hi), _ptr(mask), _ptr(row_count), _ptr(db_map), _ptr(peak_pow),
                                           ctypes.byref(group)),
                   'rsl_rds_detect')
        return int(group.value)

    # -- a8 -------------------------------------------------------------------------------------
    def detect(self, rds, thr_power: float, i_lo: int, i_hi: int, want_db: bool = False, out=None):
        torch = self.torch
        F, A, S, C = rds.shape
        W = (C + 63) // 64
        if out is None:
            out = {}
        mask = out.get('mask')
        if mask is None:
            mask = self.empty((F, A, S, W), torch.int64)
        rc = out.get('row_count')
        if rc is None:
            rc = self.empty((F, A, S), torch.int32)
        db = self.empty((F, A, S, C), torch.float32) if want_db else None
        pk = out.get('peak_pow')
        self._bind()
        self.check(self.lib.rsl_detect(self.h, _ptr(rds), F, A, S, C, float(thr_power), int(i_lo), int(i_hi),
                                       _ptr(mask), _ptr(rc), _ptr(db), _ptr(pk)), 'rsl_detect')
        return mask, rc, db

    def offsets(self, mask, row_count, C: int, bufs=None):
        torch = self.torch
        F, A, S, W = mask.shape
        b = bufs or {}
        eo = b.get('entry_row_off') if b.get('entry_row_off') is not None else self.empty((F * A * S,), torch.int32)
        co = b.get('cell_row_off') if b.get('cell_row_off') is not None else self.empty((F * S,), torch.int32)
        sc = b.get('scratch') if b.get('scratch') is not None else self.empty((F * S,), torch.int32)
        eb = b.get('entry_base') if b.get('entry_base') is not None else self.empty((F + 1,), torch.int64)
        cb = b.get('cell_base') if b.get('cell_base') is not None else self.empty((F + 1,), torch.int64)
        fc = b.get('frame_counts') if b.get('frame_counts') is not None else self.empty((2 * F,), torch.int64)
        um = b.get('union_mask') if b.get('union_mask') is not None else self.empty((F, S, W), torch.int64)
        self._bind()
        self.check(self.lib.rsl_peak_offsets(self.h, _ptr(mask), _ptr(row_count), F, A, S, C, _ptr(eo), _ptr(co),
                                             _ptr(sc), _ptr(eb), _ptr(cb), _ptr(fc), _ptr(um)), 'rsl_peak_offsets')
        return dict(entry_row_off=eo, cell_row_off=co, scratch=sc, entry_base=eb, cell_base=cb, frame_counts=fc,
                    union_mask=um)

    def emit(self, rds, mask, offs, entry_cap: int, cell_cap: int, want_pdb: bool = True, bufs=None,
             peak_pow=None, peak_pow_group: int = 1):
        """Compact peak entries and unique cells.  With ``peak_pow`` (from detect, row grouping 1; or rds_detect,
        the grouping it returned) and the offsets' union mask the RDS is not re-read."""
        torch = self.torch
        F, A, S, C = rds.shape
        b = bufs or {}

        def get(name, n, dt):
            t = b.get(name)
            return t if t is not None else self.empty((max(n, 1),), dt)
        # e_coord = antenna << 26 | range_bin << 13 | doppler_bin (u32 bits in an int32 tensor; unpack_coord)
        e_co, e_c = get('e_coord', entry_cap, torch.int32), get('e_cell', entry_cap, torch.int32)
        e_pdb = get('e_pdb', entry_cap, torch.float32) if want_pdb else None
        c_f, c_rc, c_am = (get('c_frame', cell_cap, torch.int32), get('c_rc', cell_cap, torch.int32),
                           get('c_amask', cell_cap, torch.int32))
        self._bind()
        self.check(self.lib.rsl_peak_emit(self.h, _ptr(rds), _ptr(mask), _ptr(offs.get('union_mask')),
                                          _ptr(peak_pow), int(peak_pow_group), F, A, S, C,
                                          _ptr(offs['entry_row_off']),
                                          _ptr(offs['cell_row_off']), _ptr(offs['entry_base']),
                                          _ptr(offs['cell_base']), int(entry_cap), int(cell_cap), _ptr(e_co),
                                          _ptr(e_c), _ptr(e_pdb), _ptr(c_f), _ptr(c_rc), _ptr(c_am)),
                   'rsl_peak_emit')
        return dict(e_coord=e_co, e_cell=e_c, e_pdb=e_pdb, c_frame=c_f, c_rc=c_rc, c_amask=c_am)

    # -- steering tables -------------------------------------------------------------------------
    def steering(self, steer_c128: np.ndarray):
        """Upload a [G, M] complex128 steering matrix: MFMA operand table (f32), fp64 copy, np.angle copy."""
        key = (steer_c128.shape, hash(steer_c128.tobytes()))
        hit = self._steer_cache.get(key)
        if hit is not None:
            return hit
        G, M = steer_c128.shape
        n = self.lib.rsl_steer_table_floats(G, M)
        host = np.zeros(n, dtype=np.float32)
        flat = np.ascontiguousarray(steer_c128.astype(np.complex128)).view(np.float64)
        nt, fl = c_int(), c_int()
        rc = self.lib.rsl_steer_table_build(flat.ctypes.data_as(ctypes.POINTER(c_double)), G, M,
                                            host.ctypes.data_as(ctypes.POINTER(c_float)), byref(nt), byref(fl))
        if rc != 0:
            raise ValueError(f"rsl_steer_table_build failed (G={G}, M={M})")
        torch = self.torch
        ent = dict(G=G, M=M, tab=self.to_dev(host), c128=self.to_dev(flat.copy()),
                   toeplitz=bool(fl.value & _lib.STEER_TOEPLITZ),
                   phase=self.to_dev(np.angle(steer_c128).astype(np.float64)))
        self._steer_cache[key] = ent
        return ent

    # -- a11-a16 ----------------------------------------------------------------------------------
    def doa(self, rds, c_frame, c_rc, steer, method: int, *, n: Optional[int] = None, n_dev=None,
            want_gmax: bool = False, want_spec: bool = False, out_idx=None, fast: bool = True,
            spec_gmajor: bool = False, spec_blocked: bool = False, out_spec=None):
        """Steering-scan argmax per cell.  fast=True (default) uses the Toeplitz f16-MFMA path when the
        steering matrix is a uniform linear array and either no spectrum or the cell-blocked spectrum (without
        gmax) is requested; fast=False forces the f32 [Re; Im] MFMA scan.  want_spec: the spectrum, f32 [n, G]; [G, n] (n = the capacity) with spec_gmajor;
        [ceil(n / 32), G, 32] with spec_blocked (see spectrum_rows)."""
        torch = self.torch
        _, A, S, C = rds.shape
        cap = int(c_frame.shape[0]) if n is None else int(n)
        idx = out_idx if out_idx is not None else self.empty((max(cap, 1),), torch.int32)
        gmax = self.empty((max(cap, 1),), torch.float32) if want_gmax else None
        spec = out_spec
        if want_spec and spec is None:
            G = steer['G']
            shape = ((max(cap, 1) + 31) // 32, G, 32) if spec_blocked else (G, max(cap, 1)) if spec_gmajor else \
                (max(cap, 1), G)
            spec = self.empty(shape, torch.float32)
        self._bind()
        m = int(method)
        if want_spec and spec_blocked:
            m |= _lib.DOA_SPEC_BLOCKED
        elif want_spec and spec_gmajor:
            m |= _lib.DOA_SPEC_GMAJOR
        if fast and steer['toeplitz'] and (not want_spec or (spec_blocked and not want_gmax)):
            m |= _lib.DOA_TOEPLITZ  # the f16-MFMA Toeplitz scan (argmax, or with the cell-blocked spectrum)
        self.check(self.lib.rsl_doa(self.h, _ptr(rds), A, S, C, _ptr(c_frame), _ptr(c_rc), _ptr(n_dev), cap,
                                    _ptr(steer['tab']), _ptr(steer['c128']), steer['G'], m, _ptr(idx), _ptr(gmax),
                                    _ptr(spec)), 'rsl_doa')
        return idx, gmax, spec

    def doa_extras(self, rds, c_frame, c_rc, steer, method: int, *, n: int, n_dev=None, esprit_scale: float,
                   out_idx, esprit=None, phase=None, gmax=None):
        """Fused Toeplitz DoA argmax + ESPRIT + spatial phase from one signature load (rsl_doa_extras)."""
        _, A, S, C = rds.shape
        self._bind()
        self.check(self.lib.rsl_doa_extras(self.h, _ptr(rds), A, S, C, _ptr(c_frame), _ptr(c_rc), _ptr(n_dev), int(n),
                                           _ptr(steer['tab']), _ptr(steer['c128']), steer['G'], int(method),
                                           float(esprit_scale), _ptr(out_idx), _ptr(gmax), _ptr(esprit),
                                           _ptr(phase)), 'rsl_doa_extras')
        return out_idx, esprit, phase

    def cell_extras(self, rds, c_frame, c_rc, *, n: int, n_dev=None, esprit_scale: float = 1 / math.pi,
                    want_sig=False, want_esprit=False, want_phase=False, gidx=None, az_table=None, bufs=None):
        torch = self.torch
        _, A, S, C = rds.shape
        b = bufs or {}
        cap = max(int(n), 1)
        sig = self.empty((cap, A), torch.complex64) if want_sig else None
        esp = (b.get('esprit') if b.get('esprit') is not None else self.empty((cap,), torch.float64)) if want_esprit else None
        ph = (b.get('phase') if b.get('phase') is not None else self.empty((cap,), torch.float64)) if want_phase else None
        az = None
        if az_table is not None:
            az = b.get('az') if b.get('az') is not None else self.empty((cap,), torch.float64)
        self._bind()
        self.check(self.lib.rsl_cell_extras(self.h, _ptr(rds), A, S, C, _ptr(c_frame), _ptr(c_rc), _ptr(n_dev),
                                            int(n), float(esprit_scale), _ptr(gidx), _ptr(az_table), _ptr(sig),
                                            _ptr(esp), _ptr(ph), _ptr(az)), 'rsl_cell_extras')
        return sig, esp, ph, az

    def confidence(self, rds, c_frame, c_rc, gidx, steer, n: int):
        torch = self.torch
        _, A, S, C = rds.shape
        conf = self.empty((max(n, 1),), torch.float64)
        self._bind()
        self.check(self.lib.rsl_confidence(self.h, _ptr(rds), A, S, C, _ptr(c_frame), _ptr(c_rc), int(n), _ptr(gidx),
                                           _ptr(steer['c128']), _ptr(steer['phase']), _ptr(conf)), 'rsl_confidence')
        return conf

    # -- configs[3] per-frame pattern ------------------------------------------------------------
    def peak_topk(self, entry_base, entry_cap: int, e_coord, e_pdb, *, thr_db: float, kmax: int, C: int):
        """Per cube k: the first kmax peak entries by power_db descending (stable; robust_angle_estimation.py:362-369).
        Returns (sel_entry, sel_frame, sel_rc) i32 [ncube * kmax] and sel_n i32 [ncube]."""
        torch = self.torch
        ncube = int(entry_base.shape[0]) - 1
        n = max(ncube * int(kmax), 1)
        se, sf, sr = (self.empty((n,), torch.int32) for _ in range(3))
        sn = self.empty((max(ncube, 1),), torch.int32)
        self._bind()
        self.check(self.lib.rsl_peak_topk(self.h, _ptr(entry_base), int(entry_cap), ncube, _ptr(e_coord), _ptr(e_pdb),
                                          float(thr_db), int(kmax), int(C), _ptr(se), _ptr(sf), _ptr(sr), _ptr(sn)),
                   'rsl_peak_topk')
        return se, sf, sr, sn

    def associate_nearest(self, range_m, az_rad, s0, off, *, thr: float = 5.0):
        """The analyser's association (radarscenes_complete_analysis.py:274-305) for every frame of a batch:
        range_m, az_rad f64 [N], s0 c128 [N] (first signature components), off i64 [nframes + 1] (device).
        Returns (match i32 [N] within the previous frame, -1 = none; dist f64 [N]; phase f64 [N])."""
        torch = self.torch
        nframes = int(off.shape[0]) - 1
        N = int(range_m.shape[0])
        match = self.empty((max(N, 1),), torch.int32)
        dist = self.empty((max(N, 1),), torch.float64)
        phase = self.empty((max(N, 1),), torch.float64)
        self._bind()
        self.check(self.lib.rsl_associate_nearest(self.h, _ptr(range_m), _ptr(az_rad), _ptr(s0), _ptr(off), nframes, N,
                                                  float(thr), _ptr(match), _ptr(dist), _ptr(phase)),
                   'rsl_associate_nearest')
        return match, dist, phase

    # -- a25-a29 ---------------------------------------------------------------------------------
    def velocity(self, az, y, seg, *, k: float, ridge: float = 0.0, bounds=(-50.0, 50.0, -50.0, 50.0),
                 amask=None, want_resid=False, out=None, gidx=None, az_table=None, n=None):
        """n: the per-target arrays' length (default len(y)); the segments in seg are clamped to it."""
        torch = self.torch
        F = int(seg.shape[0]) - 1
        o = out if out is not None else self.empty((max(F, 1), 8), torch.float64)
        N = int(y.shape[0]) if n is None else min(int(n), int(y.shape[0]))
        G = int(az_table.shape[0]) if az_table is not None else 0
        resid = self.empty((max(N, 1),), torch.float64) if want_resid else None
        pred = self.empty((max(N, 1),), torch.float64) if want_resid else None
        b4 = (c_double * 4)(*[float(x) for x in bounds])
        self._bind()
        self.check(self.lib.rsl_velocity(self.h, _ptr(az), _ptr(gidx), _ptr(az_table), G, _ptr(y), _ptr(amask),
                                         _ptr(seg), N, F, float(k), float(ridge), b4, _ptr(o), _ptr(resid), _ptr(pred)),
                   'rsl_velocity')
        return o, resid, pred


_ctx_lock = threading.Lock()
_ctx: Dict[int, Context] = {}


def spectrum_rows(spec_blocked, n: int):
    """Cell-major [n, G] view (a device copy) of a cell-blocked spectrum [ceil(cap / 32), G, 32]."""
    nb, G, _ = spec_blocked.shape
    return spec_blocked.permute(0, 2, 1).reshape(nb * 32, G)[:n]


def get_context(device: Optional[int] = None) -> Context:
    import torch
    if device is None:
        device = torch.cuda.current_device() if torch.cuda.is_available() else 0
    with _ctx_lock:
        c = _ctx.get(device)
        if c is None:
            c = Context(device)
            _ctx[device] = c
        return c

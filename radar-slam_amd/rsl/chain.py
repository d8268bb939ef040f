"""Batched per-frame chain on one MI355X: cube -> RDS -> peaks -> DoA (MUSIC argmax) -> ESPRIT -> velocity.

This is the throughput path (``bench.py``) and the engine under the drop-in wrappers.  A batch of F
frames is processed with a fixed sequence of asynchronous kernel launches on the current stream and no
host synchronisation: peak lists are written into capacity-sized buffers whose true sizes live on the
device (``entry_base[F]``, ``cell_base[F]``).  Per-antenna detections of one (range, doppler) cell share
one spatial signature (angle_estimation.py:83), so DoA/ESPRIT run once per unique cell and entries map
to cells (``e_cell``); the velocity LS weights each cell by its number of antenna detections, which
reproduces the reference's sums over all targets exactly.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _lib, tables
from .runtime import Context, get_context, unpack_coord

C_LIGHT = 3e8


@dataclass
class ChainConfig:
    num_antennas: int = 8
    num_chirps: int = 128
    fc: float = 77e9
    bandwidth: float = 1e9
    chirp_duration: float = 51.2e-6
    pri: float = 100e-6
    sampling_rate: float = 10e6
    window_type: str = 'hann'
    dc_removal: bool = True
    threshold_db: float = -20.0
    min_range: float = 1.0
    max_range: float = 200.0
    antenna_spacing: Optional[float] = None
    search_range: tuple = (-90, 90)
    search_resolution: float = 0.5
    method: str = 'music'
    velocity_lambda: Optional[float] = None    # VelocitySolver default: c / fc
    dt: float = 0.1
    ridge: float = 0.0
    bounds: tuple = (-50.0, 50.0, -50.0, 50.0)
    entry_frac: float = 0.20                   # capacity: peak entries per cube cell (9.4 % measured)
    cell_frac: float = 1.00                    # capacity: unique cells per (range, doppler) cell (54-76 %)
    spectrum: bool = False                     # also write the MUSIC / beamforming spectrum of every cell, f32
                                               # cell-blocked [cells / 32, G, 32] (rsl.runtime.spectrum_rows)
                                               # (angle_estimation.py:299 stores spectrum f64[G] per target)

    @property
    def S(self) -> int:
        return tables.samples_per_chirp(self.chirp_duration, self.sampling_rate)

    @property
    def lambda_c(self) -> float:
        return C_LIGHT / self.fc


GUARD_BYTES = 256 * 1024  # sentinel pad on each side of a guarded buffer (RadarChain(guard=True))
GUARD_FILL = 0xA5


class RadarChain:
    def __init__(self, cfg: ChainConfig, frames: int, ctx: Optional[Context] = None, vel_out=None,
                 guard: bool = False, spec_out=None):
        """vel_out: optional device f64 [frames, 8] view receiving the per-frame velocity rows (lets several
        chains on different streams fill consecutive slices of one buffer).
        guard: debug canary — every device buffer of the chain gets its own allocation with GUARD_BYTES of sentinel
        bytes on both sides; guard_violations() lists the buffers whose pads were written (a store that left its own
        buffer: tests/test_gpu_pipelined.py).
        spec_out: optional device f32 tensor receiving the cell-blocked spectrum (cfg.spectrum), of shape
        spectrum_shape(), or 'contiguous': the chain allocates it with Context.empty_contiguous (one physically
        contiguous allocation; the default allocator when the driver cannot provide one, spec_contiguous tells)."""
        self.cfg, self.F = cfg, int(frames)
        self.ctx = ctx or get_context()
        torch, ctx = self.ctx.torch, self.ctx
        self._guards = []
        A, C, S, F = cfg.num_antennas, cfg.num_chirps, cfg.S, self.F
        self.A, self.C, self.S = A, C, S
        tab = tables.chirp_table(cfg.fc, cfg.bandwidth, cfg.chirp_duration, cfg.sampling_rate, cfg.window_type, S)
        self.table = ctx.to_dev(tab.astype(np.complex64))
        self.i_lo, self.i_hi = tables.range_gate(cfg.bandwidth, S, cfg.min_range, cfg.max_range)
        self.thr_p = tables.power_threshold(cfg.threshold_db)
        d = cfg.antenna_spacing or cfg.lambda_c / 2
        self.grid = tables.azimuth_grid(cfg.search_range, cfg.search_resolution)
        self.steer = ctx.steering(tables.steering_matrix(self.grid, np.arange(A) * d, cfg.lambda_c))
        self.az_table = ctx.to_dev(np.radians(self.grid).astype(np.float64))
        self.esprit_scale = cfg.lambda_c / (2 * np.pi * d)
        lam_v = cfg.velocity_lambda or cfg.lambda_c
        self.k = 4 * np.pi * cfg.dt / lam_v
        self.method = _lib.METHOD_MUSIC if cfg.method == 'music' else _lib.METHOD_BEAMFORMING
        self.entry_cap = int(math.ceil(cfg.entry_frac * F * A * S * C)) + 64
        self.cell_cap = (int(math.ceil(cfg.cell_frac * F * S * C)) + 64 + 3) & ~3  # a multiple of 4 (16-B rows)
        e = self._guarded_empty if guard else ctx.empty
        W = (C + 63) // 64
        self.work = e((F, A, C, S), torch.complex64)
        self.rds = e((F, A, S, C), torch.complex64)
        self.mask = e((F, A, S, W), torch.int64)
        self.row_count = e((F, A, S), torch.int32)
        self.peak_pow = e((F, A, S, C), torch.float32)  # row-compact peak powers (detect -> emit)
        self.offs = dict(entry_row_off=e((F * A * S,), torch.int32), cell_row_off=e((F * S,), torch.int32),
                         scratch=e((F * S,), torch.int32), entry_base=e((F + 1,), torch.int64),
                         cell_base=e((F + 1,), torch.int64), frame_counts=e((2 * F,), torch.int64),
                         union_mask=e((F, S, W), torch.int64))
        ec, cc = self.entry_cap, self.cell_cap
        self.lists = dict(e_coord=e((ec,), torch.int32), e_cell=e((ec,), torch.int32), e_pdb=e((ec,), torch.float32),
                          c_frame=e((cc,), torch.int32), c_rc=e((cc,), torch.int32), c_amask=e((cc,), torch.int32))
        self.gidx = e((cc,), torch.int32)
        self.ext = dict(esprit=e((cc,), torch.float64), phase=e((cc,), torch.float64), az=e((cc,), torch.float64))
        self.vel = vel_out if vel_out is not None else e((F, 8), torch.float64)
        self.ncell_dev = self.offs['cell_base'][F:F + 1]
        # one signature gather for DoA + ESPRIT + phase when the Toeplitz path applies (uniform linear array)
        self.fused_doa = bool(self.steer['toeplitz']) and A >= 2 and not cfg.spectrum
        self.spec = None
        self.spec_contiguous = False
        if cfg.spectrum:
            shp = self.spectrum_shape()
            if isinstance(spec_out, str):
                if spec_out != 'contiguous':
                    raise ValueError("spec_out: a tensor, 'contiguous' or None")
                spec_out = ctx.empty_contiguous(shp, torch.float32)  # None: the driver could not provide it
                self.spec_contiguous = spec_out is not None
            if spec_out is not None:
                if tuple(spec_out.shape) != shp or spec_out.dtype != torch.float32 or not spec_out.is_contiguous():
                    raise ValueError(f'spec_out must be a contiguous float32 tensor of shape {shp}')
                self.spec = spec_out
            else:
                self.spec = e(shp, torch.float32)

    def spectrum_shape(self):
        """Shape of the cell-blocked spectrum buffer: [ceil(cell_cap / 32), G, 32] f32."""
        return ((self.cell_cap + 31) // 32, len(self.grid), 32)

    def _guarded_empty(self, shape, dtype):
        torch = self.ctx.torch
        n = 1
        for d in (shape if isinstance(shape, tuple) else (shape,)):
            n *= int(d)
        nbytes = n * torch.empty((), dtype=dtype).element_size()
        raw = torch.empty((2 * GUARD_BYTES + nbytes,), dtype=torch.uint8, device=self.ctx.device)
        raw.fill_(GUARD_FILL)
        self._guards.append(raw)
        return raw[GUARD_BYTES:GUARD_BYTES + nbytes].view(dtype).view(shape)

    def guard_violations(self):
        """Indices (allocation order) and byte counts of guarded buffers whose sentinel pads changed (synchronises)."""
        bad = []
        for k, raw in enumerate(self._guards):
            n = int((raw[:GUARD_BYTES] != GUARD_FILL).sum().item() + (raw[-GUARD_BYTES:] != GUARD_FILL).sum().item())
            if n:
                bad.append((k, n))
        return bad

    def run(self, cube, *, esprit: bool = True, velocity: bool = True):
        """Launch the whole chain for cube complex64 [F, A, C, S] on the current stream (asynchronous)."""
        self.run_front(cube)
        self.run_back(esprit=esprit, velocity=velocity)

    def run_front(self, cube, *, emit: bool = True, offsets: bool = True):
        """Memory-bound half: RDS + detection, offsets, peak / cell compaction (current stream). With emit=False the
        compaction is left to run_back(emit=True) (a pipelining split of the same work)."""
        ctx, cfg = self.ctx, self.cfg
        if self.F == 0:  # empty batch: only the (zeroed) bases
            ctx.offsets(self.mask, self.row_count, self.C, bufs=self.offs)
            return
        group = ctx.rds_detect(cube, self.table, self.thr_p, self.i_lo, self.i_hi, rds=self.rds, work=self.work,
                               mask=self.mask, row_count=self.row_count, peak_pow=self.peak_pow,
                               dc_removal=cfg.dc_removal)
        self._group = group
        if offsets:
            ctx.offsets(self.mask, self.row_count, self.C, bufs=self.offs)
        if emit:
            self._emit()

    def _emit(self):
        self.ctx.emit(self.rds, self.mask, self.offs, self.entry_cap, self.cell_cap, want_pdb=True, bufs=self.lists,
                      peak_pow=self.peak_pow, peak_pow_group=self._group)

    def run_back(self, *, esprit: bool = True, velocity: bool = True, emit: bool = False, offsets: bool = False):
        """Compute-bound half: DoA scan (+ ESPRIT, phase) and the velocity solve, on run_front's lists (emit=True:
        the compaction first, after run_front(emit=False))."""
        ctx, cfg = self.ctx, self.cfg
        L = self.lists
        if self.F == 0:
            return
        if offsets:
            ctx.offsets(self.mask, self.row_count, self.C, bufs=self.offs)
        if emit:
            self._emit()
        if self.fused_doa:
            ctx.doa_extras(self.rds, L['c_frame'], L['c_rc'], self.steer, self.method, n=self.cell_cap,
                           n_dev=self.ncell_dev, esprit_scale=self.esprit_scale, out_idx=self.gidx,
                           esprit=self.ext['esprit'] if esprit else None, phase=self.ext['phase'] if velocity else None)
        else:
            ctx.doa(self.rds, L['c_frame'], L['c_rc'], self.steer, self.method, n=self.cell_cap,
                    n_dev=self.ncell_dev, out_idx=self.gidx, want_spec=self.spec is not None, spec_blocked=True,
                    out_spec=self.spec)
            if esprit or velocity:
                ctx.cell_extras(self.rds, L['c_frame'], L['c_rc'], n=self.cell_cap, n_dev=self.ncell_dev,
                                esprit_scale=self.esprit_scale, want_esprit=esprit, want_phase=velocity,
                                bufs=self.ext)
        if velocity:
            ctx.velocity(None, self.ext['phase'], self.offs['cell_base'], k=self.k, ridge=cfg.ridge,
                         bounds=cfg.bounds, amask=L['c_amask'], out=self.vel, gidx=self.gidx, az_table=self.az_table,
                         n=self.cell_cap)

    def totals(self):
        eb = self.offs['entry_base'][self.F].item()
        cb = self.offs['cell_base'][self.F].item()
        return int(eb), int(cb)

    def results(self):
        """Synchronise and copy the batch results to host numpy arrays."""
        ne, nc = self.totals()
        if ne > self.entry_cap or nc > self.cell_cap:
            raise RuntimeError(f"peak capacity exceeded: entries {ne}/{self.entry_cap}, cells {nc}/{self.cell_cap}")
        L = self.lists
        h = lambda t, n: t[:n].cpu().numpy()
        return dict(entry_base=self.offs['entry_base'].cpu().numpy(), cell_base=self.offs['cell_base'].cpu().numpy(),
                    **dict(zip(('e_ant', 'e_rbin', 'e_dbin'), unpack_coord(h(L['e_coord'], ne)))),
                    e_cell=h(L['e_cell'], ne), e_pdb=h(L['e_pdb'], ne).astype(np.float64), c_frame=h(L['c_frame'], nc),
                    c_rc=h(L['c_rc'], nc), c_amask=h(L['c_amask'], nc), gidx=h(self.gidx, nc),
                    esprit=h(self.ext['esprit'], nc), phase=h(self.ext['phase'], nc),
                    az=np.radians(self.grid)[h(self.gidx, nc)],
                    velocity=self.vel.cpu().numpy(), grid=self.grid)

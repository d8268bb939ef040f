"""Device synthetic FMCW cubes: the batch-scale counterpart of
``FMCWRadarSimulator.synthesize_frame`` (reference scripts/simulate_raw.py:147-221).

``SyntheticCubes(ctx, scatterers, ...)`` computes the scatterers' fp64 [A, S] pattern once with ``rsl_synth_pattern``
and ``generate(F, frame0, seed)`` writes c64 [F, A, C, S] cubes = pattern + complex Gaussian noise with
``rsl_synth_cube`` (Philox-4x32-10, counter = global sample index: frame blocks of one seed compose exactly).
Constructor arguments follow the reference simulator (simulate_raw.py:57-80) and its scene dict keys
(range_sc, azimuth_sc, rcs, vr; simulate_raw.py:174-178).
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np


class SyntheticCubes:
    def __init__(self, ctx, scatterers: Sequence[Dict], *, fc: float = 77e9, bandwidth: float = 1e9,
                 chirp_duration: float = 40e-6, num_chirps: int = 64, num_antennas: int = 8,
                 antenna_spacing: Optional[float] = None, sampling_rate: float = 10e6, noise_power: float = 0.01):
        import torch
        from .runtime import _ptr
        self.ctx = ctx
        self.A, self.C = int(num_antennas), int(num_chirps)
        self.S = int(chirp_duration * sampling_rate)  # simulate_raw.py:75
        self.noise_power = float(noise_power)
        sc = np.array([[s.get('range_sc', 0.0), s.get('azimuth_sc', 0.0), s.get('rcs', -10.0), s.get('vr', 0.0)]
                       for s in scatterers], dtype=np.float64).reshape(-1, 4)
        self.pattern = ctx.empty((self.A, self.S), torch.complex128)
        dsc = ctx.to_dev(sc) if len(sc) else None
        ctx._bind()
        ctx.check(ctx.lib.rsl_synth_pattern(ctx.h, _ptr(dsc), len(sc), self.A, self.S, float(fc), float(bandwidth),
                                            float(chirp_duration), float(antenna_spacing or 0.0),
                                            _ptr(self.pattern)), 'rsl_synth_pattern')

    def generate(self, frames: int, *, seed: int = 0, frame0: int = 0, out=None):
        """c64 [frames, A, C, S] on the device (asynchronous on the context's stream)."""
        import torch
        from .runtime import _ptr
        c = self.ctx
        if out is None:
            out = c.empty((frames, self.A, self.C, self.S), torch.complex64)
        c._bind()
        c.check(c.lib.rsl_synth_cube(c.h, _ptr(self.pattern), int(frames), self.A, self.C, self.S, self.noise_power,
                                     int(seed) & 0xFFFFFFFFFFFFFFFF, int(frame0), _ptr(out)), 'rsl_synth_cube')
        return out

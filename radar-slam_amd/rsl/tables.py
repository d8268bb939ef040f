"""Host-side fp64 table construction (setup, not per-element work).

Everything the kernels need that depends only on the radar configuration is computed here once, in
float64 exactly as the reference computes it, and uploaded (cast to fp32 / c64 where the kernel
computes in fp32):

* ``chirp_table``   conj(reference_chirp) * window            (dechirp.py:74-83, 99-108, 139)
* ``range_gate``    index interval of linspace(0, rr*S, S) in [min_range, max_range]  (dechirp.py:241, 263)
* ``power_threshold`` 10^(thr/10) - 1e-12                      (dechirp.py:238, 252)
* ``azimuth_grid`` / ``steering_matrix``                       (angle_estimation.py:59-60, 92-107)
"""
from __future__ import annotations

import numpy as np

C_LIGHT = 3e8


def samples_per_chirp(chirp_duration: float, sampling_rate: float) -> int:
    return int(chirp_duration * sampling_rate)  # dechirp.py:63 (truncating)


def window_values(window_type: str, n: int) -> np.ndarray:
    from scipy.signal import windows  # dechirp.py:15, 99-106
    if window_type == 'hann':
        return windows.hann(n)
    if window_type == 'hamming':
        return windows.hamming(n)
    if window_type == 'blackman':
        return windows.blackman(n)
    raise ValueError(f"Unknown window type: {window_type}")


def reference_chirp(fc, bandwidth, chirp_duration, sampling_rate) -> np.ndarray:
    S = samples_per_chirp(chirp_duration, sampling_rate)
    t = np.linspace(0, chirp_duration, S)
    chirp_rate = bandwidth / chirp_duration
    return np.exp(1j * (2 * np.pi * (fc * t + 0.5 * chirp_rate * t ** 2)))


def chirp_table(fc, bandwidth, chirp_duration, sampling_rate, window_type, S) -> np.ndarray:
    """conj(ref) * window as complex128[S].  Raises the reference's broadcast ValueError when the frame's
    sample count differs from int(T_c * f_s) (dechirp.py:139)."""
    ref = reference_chirp(fc, bandwidth, chirp_duration, sampling_rate)
    if ref.shape[0] != S:
        raise ValueError(f"operands could not be broadcast together with shapes ({S},) ({ref.shape[0]},) ")
    return np.conj(ref) * window_values(window_type, S)


def range_axis(bandwidth, S):
    return np.linspace(0, (C_LIGHT / (2 * bandwidth)) * S, S)


def doppler_axis(sampling_rate, C):
    return np.linspace(-sampling_rate / 2, sampling_rate / 2, C)


def range_gate(bandwidth, S, min_range, max_range):
    r = range_axis(bandwidth, S)
    ok = np.nonzero((r >= min_range) & (r <= max_range))[0]
    if ok.size == 0:
        return 1, 0
    return int(ok[0]), int(ok[-1])


def power_threshold(threshold_db: float) -> float:
    return float(10.0 ** (threshold_db / 10.0) - 1e-12)


def azimuth_grid(search_range=(-90, 90), search_resolution=0.5):
    return np.arange(search_range[0], search_range[1] + search_resolution, search_resolution)


def steering_matrix(grid_deg, antenna_positions, lambda_c) -> np.ndarray:
    az = np.radians(np.asarray(grid_deg, dtype=np.float64))
    ph = 2 * np.pi * antenna_positions[None, :] * np.sin(az)[:, None] / lambda_c
    return np.exp(1j * ph)

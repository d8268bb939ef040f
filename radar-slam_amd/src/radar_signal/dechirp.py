"""Signal preprocessing (dechirp, window, DC removal, range-Doppler FFT, peak detection) on MI355X.

Drop-in for ``src/radar_signal/dechirp.py`` of the reference (``SignalPreprocessor`` :21-310,
``process_frame`` :313-355).  Per-element work runs in librsl.so kernels:

* ``generate_range_doppler_spectrum`` -> K1/K2 (``rsl_rds``): conj(ref)*window table (fp64 on the host),
  range FFT with the DC bin zeroed, Doppler FFT, fftshift on both axes folded into the store;
* ``extract_range_doppler_peaks``     -> K3 (``rsl_detect``/``rsl_peak_offsets``/``rsl_peak_emit``);
* ``dechirp_signal`` / ``apply_window`` / ``remove_dc`` / ``process_chirp`` -> ``rsl_preprocess_rows``.

Results come back as complex128 / float64 (upcast from the fp32 device computation).  Batched device
variants (``*_batch``) keep torch tensors on the GPU.
"""
from __future__ import annotations

import logging
from typing import Dict, Optional, Tuple

import numpy as np

from rsl import ops, tables

logger = logging.getLogger(__name__)


class SignalPreprocessor:
    """FMCW preprocessing with the reference's constructor, attributes and methods (dechirp.py:21-310)."""

    def __init__(self, fc: float = 77e9, bandwidth: float = 1e9, chirp_duration: float = 40e-6,
                 pri: float = 100e-6, num_chirps: int = 64, sampling_rate: float = 10e6,
                 window_type: str = 'hann', dc_removal: bool = True):
        self.fc = fc
        self.bandwidth = bandwidth
        self.chirp_duration = chirp_duration
        self.pri = pri
        self.num_chirps = num_chirps
        self.sampling_rate = sampling_rate
        self.window_type = window_type
        self.dc_removal = dc_removal
        self.c = 3e8
        self.lambda_c = self.c / self.fc
        self.samples_per_chirp = tables.samples_per_chirp(chirp_duration, sampling_rate)
        self.chirp_rate = self.bandwidth / self.chirp_duration
        self.range_resolution = self.c / (2 * self.bandwidth)
        self.velocity_resolution = self.lambda_c / (2 * self.num_chirps * self.pri)
        logger.info("Initialized signal preprocessor:")
        logger.info(f"  Range resolution: {self.range_resolution:.2f} m")
        logger.info(f"  Velocity resolution: {self.velocity_resolution:.2f} m/s")

    # -- host tables (fp64, as the reference) -------------------------------------------------------
    def generate_reference_chirp(self) -> np.ndarray:
        """exp(j 2 pi (fc t + k t^2 / 2)), t = linspace(0, T_c, S) (dechirp.py:74-83)."""
        return tables.reference_chirp(self.fc, self.bandwidth, self.chirp_duration, self.sampling_rate)

    def _window(self, n: int, window_type: Optional[str] = None) -> np.ndarray:
        return tables.window_values(window_type or self.window_type, n)

    def _table(self, S: int) -> np.ndarray:
        ref = self.generate_reference_chirp()
        if ref.shape[0] != S:  # the reference fails in dechirp_signal's broadcast (dechirp.py:139)
            raise ValueError(f"operands could not be broadcast together with shapes ({S},) ({ref.shape[0]},) ")
        return np.conj(ref) * self._window(S)

    # -- a3..a6: per-chirp helpers (device row kernel) ---------------------------------------------
    def apply_window(self, signal: np.ndarray, window_type: str = None) -> np.ndarray:
        sig = np.asarray(signal)
        return ops.preprocess_rows(sig, self._window(sig.shape[-1], window_type).astype(np.complex128), dc=False)

    def remove_dc(self, signal: np.ndarray) -> np.ndarray:
        sig = np.asarray(signal)
        flat = sig.reshape(1, -1)  # np.mean over every element (dechirp.py:120)
        return ops.preprocess_rows(flat, np.ones(flat.shape[-1], np.complex128), dc=True).reshape(sig.shape)

    def dechirp_signal(self, received_signal: np.ndarray, reference_chirp: Optional[np.ndarray] = None) -> np.ndarray:
        ref = self.generate_reference_chirp() if reference_chirp is None else np.asarray(reference_chirp)
        return ops.preprocess_rows(received_signal, np.conj(ref), dc=False)

    def process_chirp(self, chirp_signal: np.ndarray, reference_chirp: Optional[np.ndarray] = None) -> np.ndarray:
        """dechirp -> window -> DC removal in one row kernel (dechirp.py:143-166)."""
        ref = self.generate_reference_chirp() if reference_chirp is None else np.asarray(reference_chirp)
        sig = np.asarray(chirp_signal)
        if ref.shape[0] != sig.shape[-1]:
            raise ValueError(f"operands could not be broadcast together with shapes ({sig.shape[-1]},) "
                             f"({ref.shape[0]},) ")
        return ops.preprocess_rows(sig, np.conj(ref) * self._window(sig.shape[-1]), dc=self.dc_removal)

    # -- a7 -----------------------------------------------------------------------------------------
    def generate_range_doppler_spectrum(self, frame_signals: np.ndarray,
                                        chirp_subset: Optional[Tuple[int, int]] = None) -> np.ndarray:
        """[A, C, S] -> complex128 RDS [A, S, C], fftshift on range and Doppler (dechirp.py:168-213)."""
        fs = np.asarray(frame_signals) if not ops._is_dev(frame_signals) else frame_signals
        A, C, S = fs.shape
        chirp0, nC = 0, C
        if chirp_subset is not None:
            start, end = chirp_subset
            idx = np.arange(C)[start:end]  # python slice semantics (dechirp.py:186)
            if idx.size == 0 or np.any(np.diff(idx) != 1):
                raise ValueError(f"chirp_subset {chirp_subset} selects no contiguous chirps")
            chirp0, nC = int(idx[0]), int(idx.size)
        return ops.range_doppler(fs, self._table(S), chirp0=chirp0, num_chirps=nC, dc_removal=self.dc_removal)

    def generate_range_doppler_spectrum_batch(self, frames, chirp_subset: Optional[Tuple[int, int]] = None):
        """Device batch variant: [F, A, C, S] (numpy or torch) -> torch complex64 [F, A, S, C] on the GPU."""
        F, A, C, S = frames.shape
        chirp0, nC = (0, C) if chirp_subset is None else (chirp_subset[0], chirp_subset[1] - chirp_subset[0])
        return ops.range_doppler(frames, self._table(S), chirp0=chirp0, num_chirps=nC, dc_removal=self.dc_removal,
                                 keep_on_device=True)

    # -- a8 -----------------------------------------------------------------------------------------
    def extract_range_doppler_peaks(self, rds: np.ndarray, threshold_db: float = -20.0, min_range: float = 1.0,
                                    max_range: float = 200.0) -> Dict:
        """3x3 local maxima above threshold within the range gate (dechirp.py:215-278); same dict."""
        A, S, C = rds.shape
        range_bins_m = tables.range_axis(self.bandwidth, S)
        doppler_bins_hz = np.linspace(-self.sampling_rate / 2, self.sampling_rate / 2, C)
        i_lo, i_hi = tables.range_gate(self.bandwidth, S, min_range, max_range)
        r = ops.detect_peaks(rds, threshold_db=threshold_db, i_lo=i_lo, i_hi=i_hi, want_db=True)
        ant, ib, jb, pdb = r['antenna'], r['range_bin'], r['doppler_bin'], r['power_db']
        peaks = [{'antenna': int(a), 'range_bin': i, 'doppler_bin': j, 'range_m': range_bins_m[i],
                  'doppler_hz': doppler_bins_hz[j], 'power_db': p}
                 for a, i, j, p in zip(ant.tolist(), ib, jb, pdb)]
        return {'peaks': peaks, 'range_bins_m': range_bins_m, 'doppler_bins_hz': doppler_bins_hz,
                'power_spectrum_db': r['power_spectrum_db']}

    def visualize_rds(self, rds: np.ndarray, antenna_idx: int = 0, save_path: Optional[str] = None) -> None:
        import matplotlib.pyplot as plt
        power_db = 10 * np.log10(np.abs(rds[antenna_idx, :, :]) ** 2 + 1e-12)
        rb = np.linspace(0, self.range_resolution * rds.shape[1], rds.shape[1])
        db = np.linspace(-self.sampling_rate / 2, self.sampling_rate / 2, rds.shape[2])
        plt.figure(figsize=(10, 6))
        plt.imshow(power_db, aspect='auto', origin='lower', extent=[db[0], db[-1], rb[0], rb[-1]], cmap='jet')
        plt.colorbar(label='Power (dB)')
        plt.xlabel('Doppler Frequency (Hz)')
        plt.ylabel('Range (m)')
        plt.title(f'Range-Doppler Spectrum (Antenna {antenna_idx})')
        if save_path:
            plt.savefig(save_path, dpi=150, bbox_inches='tight')
        plt.show()


def process_frame(raw_signals_path: str, output_path: str, radar_params: Dict,
                  chirp_subset: Optional[Tuple[int, int]] = None) -> Dict:
    """File wrapper (dechirp.py:313-355): load .npy cube, RDS, peaks, save .npy + _peaks.npz."""
    raw = np.load(raw_signals_path)
    logger.info(f"Loaded raw signals: {raw.shape}")
    pre = SignalPreprocessor(**radar_params)
    rds = pre.generate_range_doppler_spectrum(raw, chirp_subset)
    logger.info(f"Generated RDS: {rds.shape}")
    peak_info = pre.extract_range_doppler_peaks(rds)
    logger.info(f"Found {len(peak_info['peaks'])} peaks")
    np.save(output_path, rds)
    np.savez(output_path.replace('.npy', '_peaks.npz'), **peak_info)
    return {'rds_shape': rds.shape, 'num_peaks': len(peak_info['peaks']), 'peak_info': peak_info}


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser(description='Process raw FMCW signals')
    ap.add_argument('--raw', required=True, help='Path to raw signals file')
    ap.add_argument('--out', required=True, help='Output path for RDS')
    ap.add_argument('--chirp-start', type=int, help='Start chirp index')
    ap.add_argument('--chirp-end', type=int, help='End chirp index')
    a = ap.parse_args()
    params = {'fc': 77e9, 'bandwidth': 1e9, 'chirp_duration': 40e-6, 'pri': 100e-6, 'num_chirps': 64,
              'sampling_rate': 10e6}
    sub = (a.chirp_start, a.chirp_end) if a.chirp_start is not None and a.chirp_end is not None else None
    print(f"Processing complete: {process_frame(a.raw, a.out, params, sub)}")

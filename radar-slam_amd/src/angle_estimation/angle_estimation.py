"""Angle-of-arrival estimation (MUSIC / ESPRIT / beamforming) on MI355X.

Drop-in for ``src/angle_estimation/angle_estimation.py`` of the reference (``AngleEstimator`` :23-365,
``extract_angles_from_rds`` :368-417).

The reference's MUSIC covariance is rank-1 (R = s s^H of one normalised snapshot, :127), so the
noise-subspace denominator is M - |a^H s|^2 exactly and MUSIC shares beamforming's steering
contraction |A^H S|^2; both run in librsl's MFMA scan kernel (``rsl_doa``).  ESPRIT's SVD of the
(M-1)x2 shift matrix reduces to a 2x2 Hermitian eigenproblem, evaluated in fp64 (``rsl_cell_extras``).
``num_sources != 1`` runs the general subspace forms in fp64 (``rsl_music_subspace`` / ``rsl_esprit_subspace``):
with a rank-1 R the reference's larger signal subspaces contain null-space vectors that LAPACK picks by round-off;
the device fixes them by a Householder completion (see rsl_subspace.hip and tests/test_gpu_dropin.py for which
outputs are reference-determined).
"""
from __future__ import annotations

import logging
from typing import Dict, List, Optional, Tuple

import numpy as np

from rsl import ops, tables
from rsl.runtime import get_context

logger = logging.getLogger(__name__)


class AngleEstimator:
    """ULA angle estimator with the reference's constructor/attributes/methods (angle_estimation.py:23-365)."""

    def __init__(self, fc: float = 77e9, antenna_spacing: float = None, num_antennas: int = 8,
                 search_range: Tuple[float, float] = (-90, 90), search_resolution: float = 0.5):
        self.fc = fc
        self.c = 3e8
        self.lambda_c = self.c / self.fc
        self.antenna_spacing = antenna_spacing or (self.lambda_c / 2)
        self.num_antennas = num_antennas
        self.search_range = search_range
        self.search_resolution = search_resolution
        self.antenna_positions = np.arange(self.num_antennas) * self.antenna_spacing
        self.azimuth_grid = tables.azimuth_grid(search_range, search_resolution)
        self._steer = tables.steering_matrix(self.azimuth_grid, self.antenna_positions, self.lambda_c)
        self._esprit_scale = self.lambda_c / (2 * np.pi * self.antenna_spacing)
        logger.info("Initialized angle estimator:")
        logger.info(f"  Antennas: {self.num_antennas}, spacing: {self.antenna_spacing * 1000:.1f} mm")
        logger.info(f"  Search range: {search_range[0]}° to {search_range[1]}°")
        logger.info(f"  Search resolution: {search_resolution}°")

    # -- a11 / a12 ------------------------------------------------------------------------------------
    def extract_spatial_signature(self, rds: np.ndarray, range_bin: int, doppler_bin: int) -> np.ndarray:
        """rds[:, r, d] normalised to unit power (angle_estimation.py:67-90), gathered on the device."""
        sig, _, _ = ops.cell_extras(rds=rds, rbins=[range_bin], dbins=[doppler_bin], want_sig=True)
        return sig[0]

    def generate_steering_vector(self, azimuth_deg: float) -> np.ndarray:
        """exp(j 2 pi x_m sin(az) / lambda) (angle_estimation.py:92-107), host fp64 table row."""
        return tables.steering_matrix([azimuth_deg], self.antenna_positions, self.lambda_c)[0]

    # -- a13 .. a16 -------------------------------------------------------------------------------------
    def music_spectrum(self, spatial_signature: np.ndarray, num_sources: int = 1) -> np.ndarray:
        """1/|a^H E_n E_n^H a| over the azimuth grid, 0 where <= 1e-12 (angle_estimation.py:109-154)."""
        if num_sources != 1:
            return ops.subspace_music(np.asarray(spatial_signature)[None], self._steer, num_sources)[0]
        _, spec = ops.doa('music', self._steer, sigs=np.asarray(spatial_signature)[None], want_spec=True)
        return spec[0]

    def estimate_angle_music(self, spatial_signature: np.ndarray, num_sources: int = 1) -> Tuple[float, np.ndarray]:
        if num_sources != 1:
            spec = self.music_spectrum(spatial_signature, num_sources)
            return self.azimuth_grid[np.argmax(spec)], spec
        idx, spec = ops.doa('music', self._steer, sigs=np.asarray(spatial_signature)[None], want_spec=True)
        return self.azimuth_grid[idx[0]], spec[0]

    def estimate_angle_esprit(self, spatial_signature: np.ndarray, num_sources: int = 1) -> float:
        """Closed-form rank-1 ESPRIT in fp64 (angle_estimation.py:178-225); 0.0 if it fails, as the reference."""
        if num_sources != 1:
            return float(ops.subspace_esprit(np.asarray(spatial_signature)[None], num_sources,
                                             self._esprit_scale)[0])
        try:
            _, esp, _ = ops.cell_extras(sigs=np.asarray(spatial_signature)[None], esprit_scale=self._esprit_scale,
                                        want_esprit=True)
            return esp[0]
        except (ValueError, RuntimeError) as e:
            logger.warning(f"ESPRIT failed: {e}")
            return 0.0

    def estimate_angle_beamforming(self, spatial_signature: np.ndarray) -> Tuple[float, np.ndarray]:
        idx, spec = ops.doa('beamforming', self._steer, sigs=np.asarray(spatial_signature)[None], want_spec=True)
        return self.azimuth_grid[idx[0]], spec[0]

    # -- a17 ------------------------------------------------------------------------------------------
    def process_targets(self, rds: np.ndarray, peak_info: Dict, method: str = 'music') -> List[Dict]:
        """All peaks in one batched device pass (angle_estimation.py:253-309); same target dicts."""
        peaks = list(peak_info['peaks'])
        if method not in ('music', 'esprit', 'beamforming'):
            for _ in peaks:  # the reference raises inside its per-target try and skips every target
                logger.warning(f"Error processing target: Unknown method: {method}")
            logger.info(f"Processed 0 targets using {method}")
            return []
        A, S, C = rds.shape
        keep = []
        for p in peaks:
            r, d = p['range_bin'], p['doppler_bin']
            if -S <= r < S and -C <= d < C:
                keep.append(p)
            else:
                logger.warning("Error processing target: index out of bounds")
        rb = np.array([p['range_bin'] % S for p in keep], dtype=np.int64)
        db = np.array([p['doppler_bin'] % C for p in keep], dtype=np.int64)
        ctx = get_context()
        d_rds = ops.as_dev_c64(ctx, rds)
        sig, esp, _ = ops.cell_extras(rds=d_rds, rbins=rb, dbins=db, esprit_scale=self._esprit_scale,
                                      want_sig=True, want_esprit=(method == 'esprit'))
        if method == 'esprit':
            angles, spec = esp, None
        else:
            idx, spec = ops.doa(method, self._steer, rds=d_rds, rbins=rb, dbins=db, want_spec=True)
            angles = self.azimuth_grid[idx]
        targets = []
        for n, p in enumerate(keep):
            ang = angles[n]
            targets.append({'range_m': p['range_m'], 'doppler_hz': p['doppler_hz'], 'power_db': p['power_db'],
                            'azimuth_deg': ang, 'azimuth_rad': np.radians(ang), 'antenna': p['antenna'],
                            'range_bin': p['range_bin'], 'doppler_bin': p['doppler_bin'],
                            'spatial_signature': sig[n], 'spectrum': None if spec is None else spec[n]})
        logger.info(f"Processed {len(targets)} targets using {method}")
        return targets

    def visualize_angle_spectrum(self, targets: List[Dict], save_path: Optional[str] = None) -> None:
        if not targets:
            logger.warning("No targets to visualize")
            return
        import matplotlib.pyplot as plt
        fig, axes = plt.subplots(2, 2, figsize=(12, 10))
        angles = [t['azimuth_deg'] for t in targets]
        ranges = [t['range_m'] for t in targets]
        powers = [t['power_db'] for t in targets]
        axes[0, 0].hist(angles, bins=20, alpha=0.7)
        axes[0, 0].set_title('Angle Distribution')
        axes[0, 1].scatter(angles, ranges, c=powers, cmap='viridis', alpha=0.7)
        axes[0, 1].set_title('Range vs Angle')
        axes[1, 0].scatter(angles, powers, alpha=0.7)
        axes[1, 0].set_title('Power vs Angle')
        if targets[0]['spectrum'] is not None:
            axes[1, 1].plot(self.azimuth_grid, 10 * np.log10(targets[0]['spectrum'] + 1e-12))
            axes[1, 1].set_title('MUSIC Spectrum')
        plt.tight_layout()
        if save_path:
            plt.savefig(save_path, dpi=150, bbox_inches='tight')
        plt.show()


def extract_angles_from_rds(rds_path: str, peak_info_path: str, output_path: str, method: str = 'music',
                            radar_params: Dict = None) -> Dict:
    """File wrapper (angle_estimation.py:368-417)."""
    rds = np.load(rds_path)
    peak_info = dict(np.load(peak_info_path, allow_pickle=True))
    logger.info(f"Loaded RDS: {rds.shape}")
    logger.info(f"Found {len(peak_info['peaks'])} peaks")
    if radar_params is None:
        radar_params = {'fc': 77e9, 'antenna_spacing': 3e8 / (2 * 77e9), 'num_antennas': 8}
    est = AngleEstimator(**radar_params)
    targets = est.process_targets(rds, peak_info, method)
    np.savez(output_path, targets=targets, radar_params=radar_params)
    logger.info(f"Saved angle estimates for {len(targets)} targets")
    return {'num_targets': len(targets), 'method': method, 'targets': targets}


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser(description='Extract angles from RDS data')
    ap.add_argument('--rds', required=True)
    ap.add_argument('--peaks', required=True)
    ap.add_argument('--out', required=True)
    ap.add_argument('--method', choices=['music', 'esprit', 'beamforming'], default='music')
    a = ap.parse_args()
    print(f"Angle extraction complete: {extract_angles_from_rds(a.rds, a.peaks, a.out, a.method)}")

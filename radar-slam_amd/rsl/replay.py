"""configs[3] per-frame call pattern on MI355X: the in-memory ego-motion run of
``CompleteRadarScenesAnalyzer.analyze_sequence_with_ego_motion``
(reference results/ground_truth_comparison/radarscenes_complete_analysis.py:97-272), batched over a whole sequence.

Per frame and sensor the reference synthesises a cube from the sensor's scatterers (:169), forms the RDS and the
-25 dB peaks (:170-171), and runs RobustAngleEstimator.process_targets_robust (:174-176; 2-degree grid, temporal window
3, confidence threshold 0.6, 50 targets, :68-76).  Per frame it then associates the frame's targets with the previous
frame's (:186, :274-305), runs AdvancedVelocityOptimizer.run_robust_optimization (:190; max velocity 30, max angular
velocity 5, two runs, :77-87) on three or more associations, and integrates a naive pose
(x += vx dt, y += vy dt, yaw += wz dt, :202-210).

Here every cube of the sequence goes through the device at once:
  1. cubes: ``rsl_synth_pattern`` + ``rsl_synth_cube`` per (frame, sensor) from its scatterer list (Philox noise:
     statistically, not bitwise, the reference's global np.random stream), or cubes the caller uploads (parity runs);
  2. ``RadarChain.run_front`` on the whole batch: RDS + 3x3 peaks at the -25 dB threshold, compacted entries;
  3. ``rsl_peak_topk``: each cube's first max_targets entries by power_db, descending, stable (:362-369);
  4. ``rsl_doa`` (beamforming, 2-degree grid) + ``rsl_confidence`` + the normalised signatures (``rsl_cell_extras``)
     for all selected entries of all cubes;
  5. host: the reference's stateful temporal smoothing keyed by target id (robust :274-330), in (frame, sensor)
     order -- sequential by definition, at most max_targets values per cube;
  6. ``rsl_associate_nearest``: every frame's association with its predecessor at once;
  7. per frame, in order (the adaptive bounds are stateful): the Advanced wrapped-phase solve on the device.
"""
from __future__ import annotations

import math
import time
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib, tables
from .chain import ChainConfig, RadarChain
from .runtime import Context, get_context, unpack_coord

C_LIGHT = 3e8

# CompleteRadarScenesAnalyzer.__init__ (radarscenes_complete_analysis.py:47-56)
ANALYZER_RADAR_PARAMS = {'fc': 77e9, 'bandwidth': 1e9, 'chirp_duration': 40e-6, 'pri': 100e-6, 'num_chirps': 32,
                         'num_antennas': 8, 'sampling_rate': 10e6, 'noise_power': 0.01}


def scatterer_array(scatterers) -> np.ndarray:
    """[N, 4] f64 (range_sc, azimuth_sc, rcs, vr) from a DataFrame / dict of columns / list of dicts / array, with the
    reference simulator's per-row defaults (simulate_raw.py:174-178)."""
    if scatterers is None:
        return np.zeros((0, 4))
    if isinstance(scatterers, np.ndarray):
        return np.asarray(scatterers, np.float64).reshape(-1, 4)
    if hasattr(scatterers, 'columns'):  # pandas DataFrame (RadarScenesLoader.convert_radar_to_scatterers)
        n = len(scatterers)
        col = lambda k, d: (scatterers[k].to_numpy(np.float64) if k in scatterers.columns else np.full(n, d))
        return np.stack([col('range_sc', 0.0), col('azimuth_sc', 0.0), col('rcs', -10.0), col('vr', 0.0)], axis=1)
    if isinstance(scatterers, dict):
        n = len(next(iter(scatterers.values()))) if scatterers else 0
        col = lambda k, d: np.asarray(scatterers.get(k, np.full(n, d)), np.float64)
        return np.stack([col('range_sc', 0.0), col('azimuth_sc', 0.0), col('rcs', -10.0), col('vr', 0.0)], axis=1)
    return np.array([[s.get('range_sc', 0.0), s.get('azimuth_sc', 0.0), s.get('rcs', -10.0), s.get('vr', 0.0)]
                     for s in scatterers], np.float64).reshape(-1, 4)


class SceneReplay:
    """Batched configs[3] pattern.  ``run(frames)`` takes the processed frames in order, each a dict with
    'timestamp' and 'scatterers' = {sensor_id: scatterers} (sensors in the reference's order; empty lists skipped as
    at :165-166), and returns per-frame targets, associations, velocity estimates and naive poses."""

    def __init__(self, ctx: Optional[Context] = None, radar_params: Optional[Dict] = None, *,
                 search_resolution: float = 2.0, temporal_window: int = 3, confidence_threshold: float = 0.6,
                 max_targets: int = 50, threshold_db: float = -25.0, max_velocity: float = 30.0,
                 max_angular_velocity: float = 5.0, regularization_weight: float = 0.01,
                 num_optimization_runs: int = 2, dt: float = 0.1, assoc_threshold: float = 5.0,
                 angle_estimator=None, velocity_optimizer=None):
        """angle_estimator / velocity_optimizer: existing drop-in RobustAngleEstimator / AdvancedVelocityOptimizer
        instances whose state the replay should carry (the analyzer's attributes); default: new ones with the
        analyser's parameters."""
        from src.algorithms.robust_angle_estimation import RobustAngleEstimator
        from src.algorithms.advanced_velocity_optimization import AdvancedVelocityOptimizer
        self.ctx = ctx or get_context()
        rp = dict(ANALYZER_RADAR_PARAMS, **(radar_params or {}))
        self.rp = rp
        self.fc = rp['fc']
        self.A, self.C = int(rp['num_antennas']), int(rp['num_chirps'])
        self.S = tables.samples_per_chirp(rp['chirp_duration'], rp['sampling_rate'])
        self.threshold_db, self.max_targets, self.dt, self.assoc_threshold = threshold_db, max_targets, dt, assoc_threshold
        d = C_LIGHT / (2 * self.fc)
        # the analyser's estimators (radarscenes_complete_analysis.py:68-87): their state (smoothing deques, adaptive
        # bounds, velocity history) carries across run() calls exactly as the reference's attributes do
        self.angle_estimator = angle_estimator or RobustAngleEstimator(
            fc=self.fc, antenna_spacing=d, num_antennas=self.A, search_resolution=search_resolution,
            temporal_window=temporal_window, confidence_threshold=confidence_threshold, max_targets=max_targets)
        self.max_targets = self.angle_estimator.max_targets
        self.velocity_optimizer = velocity_optimizer or AdvancedVelocityOptimizer(fc=self.fc, lambda_c=C_LIGHT / self.fc,
                                                            num_antennas=self.A, antenna_spacing=d,
                                                            max_velocity=max_velocity,
                                                            max_angular_velocity=max_angular_velocity,
                                                            regularization_weight=regularization_weight,
                                                            num_optimization_runs=num_optimization_runs,
                                                            use_parallel=False)
        self.cfg = ChainConfig(num_antennas=self.A, num_chirps=self.C, fc=self.fc, bandwidth=rp['bandwidth'],
                               chirp_duration=rp['chirp_duration'], pri=rp['pri'], sampling_rate=rp['sampling_rate'],
                               threshold_db=threshold_db, antenna_spacing=self.angle_estimator.antenna_spacing,
                               search_resolution=self.angle_estimator.search_resolution,
                               method='beamforming')
        self.grid = self.angle_estimator.azimuth_grid
        self.range_bins_m = tables.range_axis(rp['bandwidth'], self.S)
        self.doppler_bins_hz = tables.doppler_axis(rp['sampling_rate'], self.C)
        self.timings: Dict[str, float] = {}

    # -- 1. cubes -------------------------------------------------------------------------------
    def synthesize(self, scatterer_lists: Sequence[np.ndarray], *, seed: int = 0):
        """c64 [K, A, C, S] device cubes, one per scatterer list (rsl_synth_pattern + rsl_synth_cube)."""
        from .synth import SyntheticCubes
        torch = self.ctx.torch
        K = len(scatterer_lists)
        out = self.ctx.empty((max(K, 1), self.A, self.C, self.S), torch.complex64)
        rp = self.rp
        for k, sc in enumerate(scatterer_lists):
            rows = [dict(range_sc=r, azimuth_sc=a, rcs=c, vr=v) for r, a, c, v in np.asarray(sc).reshape(-1, 4)]
            gen = SyntheticCubes(self.ctx, rows, fc=rp['fc'], bandwidth=rp['bandwidth'],
                                 chirp_duration=rp['chirp_duration'], num_chirps=self.C, num_antennas=self.A,
                                 sampling_rate=rp['sampling_rate'], noise_power=rp['noise_power'])
            gen.generate(1, seed=seed, frame0=k, out=out[k:k + 1])
        return out[:K]

    # -- 2-4. device stages ------------------------------------------------------------------------
    def select(self, cubes):
        """RDS + peaks of every cube, the robust selection and its DoA / confidence / signatures (one batch)."""
        ctx = self.ctx
        K = int(cubes.shape[0])
        chain = RadarChain(self.cfg, K, ctx)
        chain.run_front(cubes)
        L = chain.lists
        se, sf, sr, sn = ctx.peak_topk(chain.offs['entry_base'], chain.entry_cap, L['e_coord'], L['e_pdb'],
                                       thr_db=self.threshold_db, kmax=self.max_targets, C=self.C)
        n = K * self.max_targets
        steer = chain.steer
        gidx, _, _ = ctx.doa(chain.rds, sf, sr, steer, _lib.METHOD_BEAMFORMING, n=n)
        conf = ctx.confidence(chain.rds, sf, sr, gidx, steer, n)
        sig, _, _, _ = ctx.cell_extras(chain.rds, sf, sr, n=n, want_sig=True)
        ne, _ = chain.totals()
        if ne > chain.entry_cap:
            raise RuntimeError(f"peak capacity exceeded: entries {ne}/{chain.entry_cap}")
        torch = ctx.torch
        sel_entry = se.cpu().numpy().reshape(K, self.max_targets)
        sel_n = sn[:K].cpu().numpy()
        safe = se.clamp(min=0).long()
        coord = L['e_coord'][safe].cpu().numpy().reshape(K, self.max_targets)
        pdb = L['e_pdb'][safe].cpu().numpy().astype(np.float64).reshape(K, self.max_targets)
        return dict(sel_entry=sel_entry, sel_n=sel_n, coord=coord, power_db=pdb,
                    gidx=gidx[:n].cpu().numpy().reshape(K, self.max_targets),
                    conf=conf[:n].cpu().numpy().reshape(K, self.max_targets),
                    sig=sig[:n].cpu().numpy().astype(np.complex128).reshape(K, self.max_targets, self.A),
                    entries=ne, chain=chain)

    # -- 5. host: the reference's temporal smoothing -----------------------------------------------
    def targets_of(self, sel, k: int, timestamp) -> List[Dict]:
        """process_targets_robust's outputs for cube k (robust_angle_estimation.py:371-409), in selection order."""
        est = self.angle_estimator
        out = []
        ant, rb, db = unpack_coord(sel['coord'][k])
        for r in range(int(sel['sel_n'][k])):
            tid = f"target_{int(rb[r])}_{int(db[r])}"
            ang0 = self.grid[int(sel['gidx'][k, r])]
            ang, conf = est.apply_temporal_smoothing(tid, ang0, float(sel['conf'][k, r]))
            ia = est.detect_multipath_interference(sel['sig'][k, r])
            if conf >= est.confidence_threshold and not ia['is_multipath']:
                out.append({'range_m': self.range_bins_m[int(rb[r])], 'doppler_hz': self.doppler_bins_hz[int(db[r])],
                            'power_db': sel['power_db'][k, r], 'azimuth_deg': ang, 'azimuth_rad': np.radians(ang),
                            'confidence': conf, 'is_reliable': True, 'interference_analysis': ia,
                            'antenna': int(ant[r]), 'range_bin': np.int64(rb[r]), 'doppler_bin': np.int64(db[r]),
                            'spatial_signature': sel['sig'][k, r], 'target_id': tid,
                            'timestamp': timestamp or time.time()})
        return out

    # -- 6. association --------------------------------------------------------------------------
    def associate(self, frame_targets: List[List[Dict]]):
        """Associations of every frame with its predecessor (radarscenes_complete_analysis.py:274-305), in one launch.
        Returns one list per frame (frame 0: [])."""
        ctx = self.ctx
        counts = [len(t) for t in frame_targets]
        off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        N = int(off[-1])
        if N == 0 or len(frame_targets) < 2:
            return [[] for _ in frame_targets]
        flat = [t for ts in frame_targets for t in ts]
        r = np.array([t['range_m'] for t in flat], np.float64)
        a = np.array([t['azimuth_rad'] for t in flat], np.float64)
        s0 = np.array([t['spatial_signature'][0] for t in flat], np.complex128)
        match, dist, phase = ctx.associate_nearest(ctx.to_dev(r), ctx.to_dev(a), ctx.to_dev(s0.view(np.float64)),
                                                   ctx.to_dev(off), thr=self.assoc_threshold)
        match, dist, phase = match[:N].cpu().numpy(), dist[:N].cpu().numpy(), phase[:N].cpu().numpy()
        out = [[]]
        for f in range(1, len(frame_targets)):
            prev = frame_targets[f - 1]
            lst = []
            for i in range(int(off[f]), int(off[f + 1])):
                if match[i] >= 0:
                    lst.append({'current': flat[i], 'previous': prev[int(match[i])],
                                'temporal_phase_diff': float(phase[i]), 'distance': float(dist[i])})
            out.append(lst)
        return out

    # -- the whole pattern -------------------------------------------------------------------------
    def run(self, frames: Sequence[Dict], *, cubes=None, seed: int = 0, pose0=(0.0, 0.0, 0.0)) -> Dict:
        """frames: processed frames in order; cubes: optional c64 [K, A, C, S] device cubes in (frame, sensor) order
        (default: synthesised on the device).  Returns per-frame targets, associations, optimiser results, velocity
        estimates (or None) and naive poses [x, y, yaw]."""
        t0 = time.perf_counter()
        lists, owner = [], []
        for fi, fr in enumerate(frames):
            for sid, sc in fr['scatterers'].items():
                arr = scatterer_array(sc)
                if len(arr) == 0:  # radarscenes_complete_analysis.py:165-166
                    continue
                lists.append(arr)
                owner.append(fi)
        if cubes is None:
            cubes = self.synthesize(lists, seed=seed)
        elif int(cubes.shape[0]) != len(lists):
            raise ValueError(f"expected {len(lists)} cubes (one per non-empty sensor), got {int(cubes.shape[0])}")
        t1 = time.perf_counter()
        sel = self.select(cubes) if lists else None
        t2 = time.perf_counter()
        frame_targets: List[List[Dict]] = [[] for _ in frames]
        for k, fi in enumerate(owner):
            frame_targets[fi].extend(self.targets_of(sel, k, frames[fi].get('timestamp')))
        t3 = time.perf_counter()
        assoc = self.associate(frame_targets)
        t4 = time.perf_counter()
        pose = np.array(pose0, np.float64)
        opt_results, estimates, poses = [], [], []
        for fi in range(len(frames)):
            est = None
            res = None
            if fi > 0 and len(assoc[fi]) >= 3:  # :184-188
                res = self.velocity_optimizer.run_robust_optimization(assoc[fi], dt=self.dt)
                if res['success']:
                    est = {'velocity': res['velocity'], 'angular_velocity': res['angular_velocity'],
                           'rmse': res['rmse'], 'confidence': 1.0 - min(1.0, res['rmse'] / 5.0)}
                    pose[0] += est['velocity'][0] * self.dt  # :208-210
                    pose[1] += est['velocity'][1] * self.dt
                    pose[2] += est['angular_velocity'][2] * self.dt
            opt_results.append(res)
            estimates.append(est)
            poses.append(pose.copy())
        t5 = time.perf_counter()
        self.timings = dict(synth=t1 - t0, device_select=t2 - t1, smoothing=t3 - t2, association=t4 - t3,
                            velocity=t5 - t4)
        return dict(targets=frame_targets, associations=assoc, opt_results=opt_results, velocity_estimates=estimates,
                    poses=np.array(poses).reshape(-1, 3), cube_owner=np.array(owner, np.int64),
                    selections=sel)

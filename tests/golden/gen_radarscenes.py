#!/usr/bin/env python3
"""Golden vectors for the configs[3] per-frame call pattern by running the REFERENCE
``CompleteRadarScenesAnalyzer`` (results/ground_truth_comparison/radarscenes_complete_analysis.py) in the build
container on a SYNTHETIC RadarScenes-format sequence (the dataset and h5py are absent).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_radarscenes.py

What is real and what is stood in:
- the analyzer, simulator, preprocessor, robust estimator, Advanced optimizer and the loader's pandas methods
  (extract_radar_frames, get_odometry_at_time, convert_radar_to_scatterers; radarscenes_loader.py:139-254) are the
  reference's own code;
- h5py is an empty module object (radarscenes_loader.py:11 imports it; no h5py code runs);
- ``RadarScenesLoader.__init__`` reads ``data/sensors.json`` / ``data/sequences.json`` from a temporary directory
  written here, and ``load_sequence_data`` (the HDF5 read, :55-112) is replaced by a function returning the synthetic
  radar / odometry DataFrames in the loader's column layout;
- ``simulator.synthesize_frame`` is wrapped to seed the global legacy stream with 3000 + call index before each call,
  so every cube is reproducible by the oracle (oracle.synthesize_frame, bit-identical for the same seed).

Recorded (data only, no pickles): the scene, per (frame, sensor) call the seed and robust targets, per frame the
associations (index pairs into the previous / current frame's target lists, distances, temporal phases), per
optimiser call the adaptive bounds it ran with, its DE costs and result, the naive poses, and the exception the
analyzer raises at its end (``_compute_error_metrics`` truth-tests numpy arrays, :309).  The reference does not travel.
"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import REF, OUT, _import_reference  # noqa: E402

N_FRAMES = 6
SENSORS = (1, 3)
FRAME_US = 100_000
T0_US = 1_000_000


def synthetic_sequence(seed=11):
    """Radar detections in the loader's column layout (radarscenes_loader.py:245-252 reads range_sc, azimuth_sc, rcs,
    vr, x_cc, y_cc; :162-176 buckets on timestamp and sensor_id) and an odometry table (x_seq, y_seq, yaw_seq, vx,
    yaw_rate; :215-222).  A car drives at 8 m/s past static scatterers, each seen by both sensors."""
    rs = np.random.RandomState(seed)
    n_static = 7
    base_r = rs.uniform(3.0, 14.0, n_static)
    base_az = rs.uniform(-0.9, 0.9, n_static)
    rcs = rs.uniform(8.0, 22.0, n_static)
    rows = []
    for f in range(N_FRAMES):
        for si, sid in enumerate(SENSORS):
            t = T0_US + f * FRAME_US + 5_000 + 20_000 * si
            for k in range(n_static):
                r = base_r[k] - 0.8 * f + 0.5 * si
                az = base_az[k] + 0.02 * f - 0.1 * si
                vr = -8.0 * np.cos(az)
                rows.append(dict(timestamp=np.int64(t + k), sensor_id=np.int64(sid), range_sc=r, azimuth_sc=az,
                                 rcs=rcs[k] - 2.0 * si, vr=vr, x_cc=r * np.cos(az), y_cc=r * np.sin(az)))
            # a weak far scatterer and an invalid one (range <= 0 is skipped, simulate_raw.py:181)
            rows.append(dict(timestamp=np.int64(t + 50), sensor_id=np.int64(sid), range_sc=40.0 + f, azimuth_sc=0.3,
                             rcs=-5.0, vr=1.0, x_cc=0.0, y_cc=0.0))
            rows.append(dict(timestamp=np.int64(t + 51), sensor_id=np.int64(sid), range_sc=-1.0, azimuth_sc=0.0,
                             rcs=0.0, vr=0.0, x_cc=0.0, y_cc=0.0))
    radar = pd.DataFrame(rows)
    ts = np.arange(T0_US - 200_000, T0_US + (N_FRAMES + 2) * FRAME_US, 10_000, dtype=np.int64)
    tt = (ts - T0_US) * 1e-6
    odo = pd.DataFrame(dict(timestamp=ts, x_seq=8.0 * tt, y_seq=0.1 * tt ** 2, yaw_seq=0.05 * tt,
                            vx=np.full(len(ts), 8.0), yaw_rate=np.full(len(ts), 0.05)))
    return radar, odo


def main():
    _import_reference()
    sys.path.insert(0, os.path.join(REF, 'results', 'ground_truth_comparison'))
    import src.datasets.radarscenes_loader as L
    import radarscenes_complete_analysis as RCA
    import src.algorithms.advanced_velocity_optimization as MA

    radar, odo = synthetic_sequence()
    tmp = tempfile.mkdtemp()
    os.makedirs(os.path.join(tmp, 'data'))
    for n in ('sensors.json', 'sequences.json'):
        with open(os.path.join(tmp, 'data', n), 'w') as f:
            json.dump({}, f)
    analyzer = RCA.CompleteRadarScenesAnalyzer(tmp)
    analyzer.loader.load_sequence_data = lambda sid: {'sequence_id': sid, 'radar_data': radar, 'odometry_data': odo}

    out = {}
    synth_calls, robust_calls, assoc_calls, opt_calls, de_calls = [], [], [], [], []
    orig_synth = analyzer.simulator.synthesize_frame

    def synth(scatterers, frame_idx=0):
        seed = 3000 + len(synth_calls)
        np.random.seed(seed)
        sc = scatterers[['range_sc', 'azimuth_sc', 'rcs', 'vr']].to_numpy(np.float64)
        synth_calls.append((seed, sc))
        return orig_synth(scatterers, frame_idx)
    analyzer.simulator.synthesize_frame = synth

    orig_robust = analyzer.angle_estimator.process_targets_robust

    def robust(rds, peak_info, frame_timestamp=None):
        tg = orig_robust(rds, peak_info, frame_timestamp=frame_timestamp)
        robust_calls.append((len(synth_calls) - 1, frame_timestamp, len(peak_info['peaks']), tg))
        return tg
    analyzer.angle_estimator.process_targets_robust = robust

    orig_assoc = analyzer._create_target_associations

    def assoc(cur, prev):
        a = orig_assoc(cur, prev)
        ci = {id(t): i for i, t in enumerate(cur)}
        pi = {id(t): i for i, t in enumerate(prev)}
        assoc_calls.append((len(cur), len(prev), np.array([ci[id(x['current'])] for x in a], np.int64),
                            np.array([pi[id(x['previous'])] for x in a], np.int64),
                            np.array([x['distance'] for x in a]), np.array([x['temporal_phase_diff'] for x in a])))
        return a
    analyzer._create_target_associations = assoc

    orig_de = MA.differential_evolution

    def de(*a, **k):
        r = orig_de(*a, **k)
        de_calls.append((bool(r.success), float(r.fun), np.asarray(r.x, float)))
        return r
    MA.differential_evolution = de

    opt = analyzer.velocity_optimizer
    orig_opt = opt.run_robust_optimization

    def run_opt(associations, dt, previous_motion=None):
        b = opt.adaptive_bounds
        bounds = np.array(b['velocity_bounds'] + b['angular_velocity_bounds'], np.float64)
        d0 = len(de_calls)
        t0 = time.time()
        r = orig_opt(associations, dt, previous_motion)
        print(f'  optimiser call {len(opt_calls)}: {len(associations)} associations, {time.time() - t0:.1f} s',
              flush=True)
        opt_calls.append((len(assoc_calls) - 1, bounds, r, de_calls[d0:]))
        return r
    opt.run_robust_optimization = run_opt

    t0 = time.time()
    err = ''
    try:
        analyzer.analyze_sequence_with_ego_motion('sequence_synthetic', max_frames=N_FRAMES)
    except Exception as e:  # _compute_error_metrics (:309) on numpy arrays
        err = f'{type(e).__name__}: {e}'
    print(f'reference run: {time.time() - t0:.1f} s; final exception: {err!r}')

    out['radar_params'] = np.array([77e9, 1e9, 40e-6, 100e-6, 32, 8, 10e6, 0.01])
    out['final_exception'] = np.array(err)
    out['synth_seed'] = np.array([s for s, _ in synth_calls], np.int64)
    out['synth_nsc'] = np.array([len(sc) for _, sc in synth_calls], np.int64)
    out['synth_sc'] = np.concatenate([sc for _, sc in synth_calls]) if synth_calls else np.zeros((0, 4))
    # synth call -> (frame, sensor) via the robust calls (one per synthesized cube, in order)
    out['call_ts'] = np.array([int(ts) for _, ts, _, _ in robust_calls], np.int64)
    out['call_npeaks'] = np.array([n for _, _, n, _ in robust_calls], np.int64)
    keys = ('range_m', 'doppler_hz', 'power_db', 'azimuth_deg', 'azimuth_rad', 'confidence', 'antenna', 'range_bin',
            'doppler_bin')
    ntg = []
    for k in keys:
        out['tg_' + k] = np.array([t[k] for _, _, _, tg in robust_calls for t in tg])
    for _, _, _, tg in robust_calls:
        ntg.append(len(tg))
    out['tg_sig'] = np.array([t['spatial_signature'] for _, _, _, tg in robust_calls for t in tg])
    out['tg_id'] = np.array([t['target_id'] for _, _, _, tg in robust_calls for t in tg])
    out['call_ntg'] = np.array(ntg, np.int64)
    out['as_ncur'] = np.array([a[0] for a in assoc_calls], np.int64)
    out['as_nprev'] = np.array([a[1] for a in assoc_calls], np.int64)
    out['as_n'] = np.array([len(a[2]) for a in assoc_calls], np.int64)
    for j, k in enumerate(('cur', 'prev', 'dist', 'phase')):
        out['as_' + k] = np.concatenate([a[2 + j] for a in assoc_calls]) if assoc_calls else np.zeros(0)
    out['opt_assoc_call'] = np.array([o[0] for o in opt_calls], np.int64)
    out['opt_bounds'] = np.array([o[1] for o in opt_calls])
    out['opt_success'] = np.array([bool(o[2]['success']) for o in opt_calls])
    out['opt_cost'] = np.array([o[2].get('cost', np.nan) for o in opt_calls])
    out['opt_x'] = np.array([np.concatenate([o[2]['velocity'], o[2]['angular_velocity']]) if o[2]['success']
                             else np.full(6, np.nan) for o in opt_calls])
    out['opt_rmse'] = np.array([o[2].get('rmse', np.nan) for o in opt_calls])
    out['opt_de_cost'] = np.array([[c[1] for c in o[3]] for o in opt_calls])
    out['odo'] = odo.to_numpy(np.float64)
    out['radar'] = radar[['timestamp', 'sensor_id', 'range_sc', 'azimuth_sc', 'rcs', 'vr', 'x_cc',
                          'y_cc']].to_numpy(np.float64)
    np.savez_compressed(os.path.join(OUT, 'golden_radarscenes.npz'), **out)
    print('calls:', len(synth_calls), 'targets per call:', ntg, 'associations:', out['as_n'].tolist(),
          'costs:', out['opt_cost'].tolist())


if __name__ == '__main__':
    main()

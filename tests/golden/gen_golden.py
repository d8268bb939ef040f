#!/usr/bin/env python3
"""Generate golden vectors by importing and running the REFERENCE (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

The reference tree (/root/reference, read-only) is put on sys.path; ``scripts/simulate_raw.py``
imports h5py at module top (simulate_raw.py:15) but only uses it in ``process_sequence``, so an
empty stand-in module object is placed in ``sys.modules`` before import (no h5py code runs).
Outputs are small .npz fixtures (data only) next to this script.  Nothing here runs on the GPU
box; the fixtures travel, the reference does not.
"""
import hashlib
import os
import sys
import time
import types

import numpy as np

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    sys.dont_write_bytecode = True
    sys.modules.setdefault('h5py', types.ModuleType('h5py'))
    import matplotlib
    matplotlib.use('Agg')
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, 'scripts'))
    import logging
    logging.disable(logging.CRITICAL)
    from scripts.simulate_raw import FMCWRadarSimulator
    from src.radar_signal.dechirp import SignalPreprocessor
    from src.angle_estimation.angle_estimation import AngleEstimator
    from src.velocity_solver.velocity_solver import VelocitySolver
    from src.algorithms.robust_angle_estimation import RobustAngleEstimator
    from src.algorithms.velocity_solver_improved import ImprovedVelocitySolver
    from src.pose_integration.pose_integration import PoseIntegrator
    return types.SimpleNamespace(FMCWRadarSimulator=FMCWRadarSimulator, SignalPreprocessor=SignalPreprocessor,
                                 AngleEstimator=AngleEstimator, VelocitySolver=VelocitySolver,
                                 RobustAngleEstimator=RobustAngleEstimator,
                                 ImprovedVelocitySolver=ImprovedVelocitySolver, PoseIntegrator=PoseIntegrator)


SCENE = [  # tests/test_synth_raw.py:165-190
    {'range_sc': 20.0, 'azimuth_sc': 0.0, 'rcs': -10.0, 'vr': 0.0},
    {'range_sc': 40.0, 'azimuth_sc': float(np.radians(45.0)), 'rcs': -8.0, 'vr': 5.0},
    {'range_sc': 60.0, 'azimuth_sc': float(np.radians(-30.0)), 'rcs': -12.0, 'vr': -3.0},
]

CONFIGS = {
    # name: (num_antennas, num_chirps, chirp_duration) ; f_s = 10 MHz -> S = T_c * f_s
    'tiny': (8, 16, 3.2e-6),       # S = 32
    'odd400': (8, 16, 40e-6),      # S = 400 (reference default T_c; non power of two)
    'cfg1': (8, 64, 25.6e-6),      # S = 256 (BASELINE configs[0])
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    R = _import_reference()
    import pandas as pd
    t0 = time.time()
    rs = np.random.RandomState(7)
    for name, (A, C, Tc) in (CONFIGS.items() if os.environ.get('GOLDEN_ONLY') != 'pose' else []):
        seed = 1000 + len(name)
        sim = R.FMCWRadarSimulator(fc=77e9, bandwidth=1e9, chirp_duration=Tc, pri=100e-6, num_chirps=C,
                                   num_antennas=A, sampling_rate=10e6, noise_power=0.01)
        np.random.seed(seed)
        cube = sim.synthesize_frame(pd.DataFrame(SCENE))
        pre = R.SignalPreprocessor(fc=77e9, bandwidth=1e9, chirp_duration=Tc, pri=100e-6, num_chirps=C,
                                   sampling_rate=10e6)
        rds = pre.generate_range_doppler_spectrum(cube)
        rds_sub = pre.generate_range_doppler_spectrum(cube, chirp_subset=(2, C - 3))
        pinfo = pre.extract_range_doppler_peaks(rds)
        pinfo30 = pre.extract_range_doppler_peaks(rds, threshold_db=-30.0, min_range=5.0, max_range=50.0)
        pk = pinfo['peaks']
        pa = np.array([p['antenna'] for p in pk], np.int16)
        pi = np.array([p['range_bin'] for p in pk], np.int32)
        pj = np.array([p['doppler_bin'] for p in pk], np.int32)
        pdb = np.array([p['power_db'] for p in pk], np.float64)
        est = R.AngleEstimator(fc=77e9, antenna_spacing=3e8 / (2 * 77e9), num_antennas=A)
        nsel = min(len(pk), 600)
        sel = np.sort(rs.choice(len(pk), nsel, replace=False))
        sub = {'peaks': [pk[k] for k in sel]}
        t_m = time.time()
        tm = est.process_targets(rds, sub, method='music')
        t_m = time.time() - t_m
        te = est.process_targets(rds, sub, method='esprit')
        tb = est.process_targets(rds, sub, method='beamforming')
        nspec = 48
        rds_sample_idx = np.sort(rs.choice(rds.size, min(rds.size, 4096), replace=False))
        fix = dict(
            A=A, C=C, S=rds.shape[1], chirp_duration=Tc, seed=seed,
            cube_sha=sha(cube), cube_sample_idx=rds_sample_idx, cube_sample=cube.reshape(-1)[rds_sample_idx],
            rds_sha=sha(rds), rds_sample_idx=rds_sample_idx, rds_sample=rds.reshape(-1)[rds_sample_idx],
            rds_absmax=np.abs(rds).max(), rds_sub_sha=sha(rds_sub),
            rds_sub_sample=rds_sub.reshape(-1)[rds_sample_idx[rds_sample_idx < rds_sub.size]],
            peak_a=pa, peak_i=pi, peak_j=pj, peak_db=pdb,
            range_bins_m=pinfo['range_bins_m'], doppler_bins_hz=pinfo['doppler_bins_hz'],
            power_db_sha=sha(pinfo['power_spectrum_db']),
            peak30_a=np.array([p['antenna'] for p in pinfo30['peaks']], np.int16),
            peak30_i=np.array([p['range_bin'] for p in pinfo30['peaks']], np.int32),
            peak30_j=np.array([p['doppler_bin'] for p in pinfo30['peaks']], np.int32),
            sel=sel,
            music_deg=np.array([t['azimuth_deg'] for t in tm]),
            music_spec=np.array([t['spectrum'] for t in tm[:nspec]]),
            esprit_deg=np.array([t['azimuth_deg'] for t in te]),
            bf_deg=np.array([t['azimuth_deg'] for t in tb]),
            bf_spec=np.array([t['spectrum'] for t in tb[:nspec]]),
            sig=np.array([t['spatial_signature'] for t in tm]),
        )
        if name == 'tiny':
            fix['cube'] = cube
            fix['rds'] = rds
        # Velocity solver (DE, seed 42): top-50 MUSIC targets by power, both wavelengths.
        top = np.argsort(-np.array([t['power_db'] for t in tm]), kind='stable')[:50]
        tsel = [tm[k] for k in top]
        vs = R.VelocitySolver(fc=77e9, num_antennas=A)
        r1 = vs.solve_velocity(rds, tsel, dt=0.1)
        vsb = R.VelocitySolver(fc=77e9, lambda_c=77e9 / 3e8, num_antennas=A,
                               antenna_spacing=3e8 / (2 * 77e9))      # run_ego_motion_pipeline.py:244-249
        r2 = vsb.solve_velocity(rds, tsel, dt=0.1)
        fix.update(vel_top=top, vel_v=r1['velocity'], vel_w=r1['angular_velocity'], vel_cost=r1['cost'],
                   vel_rmse=r1['rmse'], vel_maxres=r1['max_residual'], vel_res=r1['residuals'],
                   velbug_v=r2['velocity'], velbug_cost=r2['cost'], velbug_rmse=r2['rmse'],
                   velbug_maxres=r2['max_residual'])
        np.savez_compressed(os.path.join(OUT, f'golden_{name}.npz'), **fix)
        print(f'{name}: rds {rds.shape} peaks {len(pk)} music {len(tm)} ({t_m:.1f}s) '
              f'v={r1["velocity"][:2]} vbug={r2["velocity"][:2]}  t={time.time() - t0:.0f}s', flush=True)

    if os.environ.get('GOLDEN_ONLY') == 'pose':
        return pose_only(R, t0)
    # Robust estimator: stateful 3-frame sequence at 'tiny'-like size but S=64, C=32.
    A, C, Tc = 8, 32, 6.4e-6
    sim = R.FMCWRadarSimulator(fc=77e9, bandwidth=1e9, chirp_duration=Tc, pri=100e-6, num_chirps=C,
                               num_antennas=A, sampling_rate=10e6, noise_power=0.01)
    pre = R.SignalPreprocessor(fc=77e9, bandwidth=1e9, chirp_duration=Tc, pri=100e-6, num_chirps=C,
                               sampling_rate=10e6)
    rob = R.RobustAngleEstimator(fc=77e9, num_antennas=A, max_targets=40, confidence_threshold=0.55)
    seq = {}
    rows = []
    for f in range(3):
        np.random.seed(2000 + (f % 2))           # frames 0 and 2 identical -> exercises smoothing
        cube = sim.synthesize_frame(pd.DataFrame(SCENE))
        rds = pre.generate_range_doppler_spectrum(cube)
        pinfo = pre.extract_range_doppler_peaks(rds)
        tg = rob.process_targets_robust(rds, pinfo, frame_timestamp=1.0 + f)
        seq[f'rds{f}'] = rds.astype(np.complex128)
        for t in tg:
            ia = t['interference_analysis']
            rows.append([f, t['range_bin'], t['doppler_bin'], t['azimuth_deg'], t['confidence'],
                         float(ia['num_sources']), float(ia['is_multipath']), t['power_db']])
    seq['rows'] = np.array(rows)
    st = rob.get_target_statistics()
    seq['stats'] = np.array([st['total_targets_tracked'], st['active_targets'], st['average_confidence']])
    np.savez_compressed(os.path.join(OUT, 'golden_robust.npz'), **seq)
    print(f'robust: {len(rows)} reliable rows')

    pose_only(R, t0)


def pose_only(R, t0):
    # Pose integration (pose_integration.py:67-220), 24 steps.
    prs = np.random.RandomState(11)
    vel = prs.randn(24, 3)
    om = 0.3 * prs.randn(24, 3)
    ts = np.arange(24) * 0.1
    pint = R.PoseIntegrator()
    # integrate_pose raises for N >= 2: norm(omega)[N] * diff(t)[N-1] (pose_integration.py:199)
    try:
        pint.integrate_pose(vel, om, ts)
        raised = ''
    except ValueError as e:
        raised = str(e)
    pos = pint.integrate_translational_velocity(vel, ts)
    ori, rot = pint.integrate_angular_velocity(om, ts)
    pe = R.PoseIntegrator(integration_method='euler', smoothing=False)
    pos_e = pe.integrate_translational_velocity(vel, ts)
    tr1 = pint.integrate_pose(vel[:1], om[:1], ts[:1])
    np.savez_compressed(os.path.join(OUT, 'golden_pose.npz'), vel=vel, om=om, ts=ts, raised=raised,
                        positions=pos, orientations=ori, rotations=rot, positions_euler=pos_e,
                        one_total_rotation=tr1['total_rotation'], one_total_distance=tr1['total_distance'])
    print(f'done in {time.time() - t0:.0f}s')


if __name__ == '__main__':
    main()

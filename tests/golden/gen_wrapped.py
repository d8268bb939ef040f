#!/usr/bin/env python3
"""Golden vectors for the wrapped-phase solvers (rows a30, a31) by running the REFERENCE in the build container.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_wrapped.py

Two consecutive synthetic cfg1 frames (seeds 1000, 1001) -> reference RDS -> the TOPK strongest peaks ->
AngleEstimator.process_targets('music') -> ImprovedVelocitySolver.solve_velocity_with_association
(velocity_solver_improved.py:479-506) and AdvancedVelocityOptimizer.run_robust_optimization
(advanced_velocity_optimization.py:410-524, with and without a previous motion).  Data only (no pickles):
targets as arrays, association pairs, and the DE results.  The reference itself does not travel.
"""
import os
import sys
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import REF, OUT, SCENE, _import_reference  # noqa: E402

TOPK = 40


def targets_for(R, frame, Tc, C, A):
    sp = R.SignalPreprocessor(chirp_duration=Tc, num_chirps=C)
    rds = sp.generate_range_doppler_spectrum(frame)
    pk = sp.extract_range_doppler_peaks(rds)
    peaks = sorted(pk['peaks'], key=lambda p: -p['power_db'])[:TOPK]  # stable: reference order among ties
    est = R.AngleEstimator(num_antennas=A)
    return est.process_targets(rds, {'peaks': peaks}, method='music')


def pack(tg):
    return dict(range_m=np.array([t['range_m'] for t in tg]), azimuth_rad=np.array([t['azimuth_rad'] for t in tg]),
                sig=np.stack([t['spatial_signature'] for t in tg]),
                range_bin=np.array([t['range_bin'] for t in tg]), doppler_bin=np.array([t['doppler_bin'] for t in tg]))


def main():
    R = _import_reference()
    sys.path.insert(0, REF)
    from src.algorithms.advanced_velocity_optimization import AdvancedVelocityOptimizer
    A, C, Tc = 8, 64, 25.6e-6
    sim = R.FMCWRadarSimulator(chirp_duration=Tc, num_chirps=C, num_antennas=A)
    frames = []
    for s in (1000, 1001):
        np.random.seed(s)
        frames.append(sim.synthesize_frame(pd.DataFrame(SCENE)))
    t0 = time.time()
    prev_t = targets_for(R, frames[0], Tc, C, A)
    cur_t = targets_for(R, frames[1], Tc, C, A)
    out = {}
    for name, tg in (('prev', prev_t), ('cur', cur_t)):
        for k, v in pack(tg).items():
            out[f'{name}_{k}'] = v
    # record every differential_evolution call of the reference solvers (result objects are not kept: data only)
    import src.algorithms.velocity_solver_improved as MI
    import src.algorithms.advanced_velocity_optimization as MA
    calls = []

    def recording(orig):
        def de(*a, **k):
            r = orig(*a, **k)
            calls.append((bool(r.success), float(r.fun), np.asarray(r.x, float), int(r.nit), int(r.nfev)))
            return r
        return de
    MI.differential_evolution = recording(MI.differential_evolution)
    MA.differential_evolution = recording(MA.differential_evolution)
    solver = R.ImprovedVelocitySolver()
    assoc = solver.associate_targets_across_frames(cur_t, prev_t)
    cur_ids = {id(t): i for i, t in enumerate(cur_t)}
    prev_ids = {id(t): i for i, t in enumerate(prev_t)}
    out['assoc_cur'] = np.array([cur_ids[id(a['current'])] for a in assoc])
    out['assoc_prev'] = np.array([prev_ids[id(a['previous'])] for a in assoc])
    out['assoc_dist'] = np.array([a['distance'] for a in assoc])
    out['assoc_phase'] = np.array([a['temporal_phase_diff'] for a in assoc])
    def save_calls(tag, c0):
        cs = calls[c0:]
        out[f'{tag}_de_success'] = np.array([c[0] for c in cs])
        out[f'{tag}_de_fun'] = np.array([c[1] for c in cs])
        out[f'{tag}_de_x'] = np.stack([np.pad(c[2], (0, 6 - len(c[2]))) for c in cs])
        out[f'{tag}_de_dim'] = np.array([len(c[2]) for c in cs])
        out[f'{tag}_de_nit'] = np.array([c[3] for c in cs])

    res = solver.two_step_optimization(assoc, 0.1)
    print(f'improved: {time.time() - t0:.1f}s  n_assoc={len(assoc)} success={res["success"]} '
          f'cost={res.get("cost")} DE={calls}', flush=True)
    out['imp_success'] = np.asarray(res['success'])
    save_calls('imp', 0)
    if res['success']:
        for k in ('velocity', 'angular_velocity', 'cost', 'rmse', 'max_residual', 'residuals', 'predicted_phases'):
            out[f'imp_{k}'] = np.asarray(res[k])
    for tag, prevm in (('adv', None), ('advp', np.array([3.0, -1.0, 0.2, 0.05, -0.02, 0.1]))):
        t1 = time.time()
        opt = AdvancedVelocityOptimizer(use_parallel=False, num_optimization_runs=2)
        c0 = len(calls)
        r = opt.run_robust_optimization(assoc, 0.1, previous_motion=prevm)
        print(f'{tag}: {time.time() - t1:.1f}s success={r["success"]} cost={r.get("cost")}', flush=True)
        out[f'{tag}_success'] = np.asarray(r['success'])
        save_calls(tag, c0)
        if r['success']:
            for k in ('velocity', 'angular_velocity', 'cost', 'rmse', 'max_residual', 'successful_runs'):
                out[f'{tag}_{k}'] = np.asarray(r[k])
        out[f'{tag}_bounds'] = np.array(opt.adaptive_bounds['velocity_bounds'])
        if prevm is not None:
            out[f'{tag}_prev'] = prevm
    np.savez_compressed(os.path.join(OUT, 'golden_wrapped.npz'), **out)
    print('wrote golden_wrapped.npz', flush=True)


if __name__ == '__main__':
    main()

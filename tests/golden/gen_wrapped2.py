#!/usr/bin/env python3
"""More golden vectors for the wrapped-phase solvers (rows a30, a31) by running the REFERENCE in the
build container, one case per process:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_wrapped2.py CASE      (CASE in CASES, or 'all')

Each case: two consecutive synthetic cfg1 frames -> reference RDS -> the TOPK strongest peaks ->
AngleEstimator.process_targets('music') -> ImprovedVelocitySolver.solve_velocity_with_association or
AdvancedVelocityOptimizer.run_robust_optimization, with a different target count, wavelength (the pipeline's
lambda = fc / c, run_ego_motion_pipeline.py:246) or previous motion.  Every differential_evolution call is recorded
(success, best cost, x); results are data only (tests/golden/golden_wrapped_<case>.npz).
"""
import os
import subprocess
import sys
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import REF, OUT, SCENE, _import_reference  # noqa: E402

FC = 77e9
CASES = {  # name: (solver, TOPK, seeds, lambda_c or None, previous motion or None)
    'imp_n20': ('improved', 20, (2000, 2001), None, None),
    'imp_lam': ('improved', 30, (2002, 2003), FC / 3e8, None),
    'adv_n60': ('advanced', 60, (2004, 2005), None, None),
    'advp_n30': ('advanced', 30, (2006, 2007), None, (-4.0, 2.5, 0.1, 0.02, 0.01, -0.05)),
    'adv_lam': ('advanced', 30, (2008, 2009), FC / 3e8, None),
}


def targets_for(R, frame, Tc, C, A, topk):
    sp = R.SignalPreprocessor(chirp_duration=Tc, num_chirps=C)
    rds = sp.generate_range_doppler_spectrum(frame)
    pk = sp.extract_range_doppler_peaks(rds)
    peaks = sorted(pk['peaks'], key=lambda p: -p['power_db'])[:topk]  # stable: reference order among ties
    est = R.AngleEstimator(num_antennas=A)
    return est.process_targets(rds, {'peaks': peaks}, method='music')


def pack(tg):
    return dict(range_m=np.array([t['range_m'] for t in tg]), azimuth_rad=np.array([t['azimuth_rad'] for t in tg]),
                sig=np.stack([t['spatial_signature'] for t in tg]),
                range_bin=np.array([t['range_bin'] for t in tg]), doppler_bin=np.array([t['doppler_bin'] for t in tg]))


def run_case(name):
    solver_kind, topk, seeds, lam, prevm = CASES[name]
    R = _import_reference()
    sys.path.insert(0, REF)
    from src.algorithms.advanced_velocity_optimization import AdvancedVelocityOptimizer
    import src.algorithms.velocity_solver_improved as MI
    import src.algorithms.advanced_velocity_optimization as MA
    A, C, Tc = 8, 64, 25.6e-6
    sim = R.FMCWRadarSimulator(chirp_duration=Tc, num_chirps=C, num_antennas=A)
    frames = []
    for s in seeds:
        np.random.seed(s)
        frames.append(sim.synthesize_frame(pd.DataFrame(SCENE)))
    prev_t = targets_for(R, frames[0], Tc, C, A, topk)
    cur_t = targets_for(R, frames[1], Tc, C, A, topk)
    out = {'case': np.array(name), 'solver': np.array(solver_kind), 'lambda_c': np.array(lam if lam else 3e8 / FC),
           'seeds': np.array(seeds)}
    for tag, tg in (('prev', prev_t), ('cur', cur_t)):
        for k, v in pack(tg).items():
            out[f'{tag}_{k}'] = v
    calls = []

    def recording(orig):
        def de(*a, **k):
            r = orig(*a, **k)
            calls.append((bool(r.success), float(r.fun), np.asarray(r.x, float)))
            return r
        return de
    MI.differential_evolution = recording(MI.differential_evolution)
    MA.differential_evolution = recording(MA.differential_evolution)
    imp = R.ImprovedVelocitySolver(lambda_c=lam) if lam else R.ImprovedVelocitySolver()
    assoc = imp.associate_targets_across_frames(cur_t, prev_t)
    ci = {id(t): i for i, t in enumerate(cur_t)}
    pi = {id(t): i for i, t in enumerate(prev_t)}
    out['assoc_cur'] = np.array([ci[id(a['current'])] for a in assoc])
    out['assoc_prev'] = np.array([pi[id(a['previous'])] for a in assoc])
    out['assoc_phase'] = np.array([a['temporal_phase_diff'] for a in assoc])
    t0 = time.time()
    if solver_kind == 'improved':
        res = imp.two_step_optimization(assoc, 0.1)
    else:
        kw = {'lambda_c': lam} if lam else {}
        opt = AdvancedVelocityOptimizer(use_parallel=False, num_optimization_runs=2, **kw)
        res = opt.run_robust_optimization(assoc, 0.1, previous_motion=None if prevm is None else np.array(prevm))
        out['bounds_after'] = np.array(opt.adaptive_bounds['velocity_bounds'])
        if prevm is not None:
            out['prev_motion'] = np.array(prevm)
    out['success'] = np.asarray(res['success'])
    out['message'] = np.array(str(res.get('message', '')))
    if res['success']:
        out['cost'] = np.asarray(res['cost'])
        out['x'] = np.concatenate([res['velocity'], res['angular_velocity']])
    out['de_success'] = np.array([c[0] for c in calls])
    out['de_fun'] = np.array([c[1] for c in calls])
    out['de_x'] = np.stack([np.pad(c[2], (0, 6 - len(c[2]))) for c in calls])
    out['de_dim'] = np.array([len(c[2]) for c in calls])
    np.savez_compressed(os.path.join(OUT, f'golden_wrapped_{name}.npz'), **out)
    print(f'{name}: {time.time() - t0:.1f}s n_assoc={len(assoc)} success={res["success"]} '
          f'cost={res.get("cost")} DE={[c[:2] for c in calls]}', flush=True)


if __name__ == '__main__':
    which = sys.argv[1] if len(sys.argv) > 1 else 'all'
    if which == 'all':
        procs = [subprocess.Popen([sys.executable, __file__, c]) for c in CASES]
        sys.exit(max(p.wait() for p in procs))
    run_case(which)

#!/usr/bin/env python3
"""Golden vectors for the velocity error statistics: imports the REFERENCE's
evaluation/compute_velocity_error.py (numpy / pandas / matplotlib only; build container only) and records
VelocityErrorEvaluator.compute_velocity_errors / analyze_error_trends / generate_error_report on synthetic
velocity tracks.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_velocity_error.py

Writes tests/golden/golden_velocity_error.npz (data only: inputs and outputs).
"""
import os
import sys

import numpy as np

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))


def tracks():
    rs = np.random.RandomState(211)
    cases = {}
    n = 900
    t = np.arange(n) * 0.1
    gt = np.column_stack([8 + np.sin(t / 7), 0.3 * np.cos(t / 5), 0.05 * rs.randn(n),
                          0.01 * rs.randn(n), 0.01 * rs.randn(n), 0.1 * np.sin(t / 11)])
    est = gt + 0.05 * rs.randn(n, 6) + np.array([0.02, -0.01, 0, 0, 0.001, 0]) + 1e-3 * t[:, None]
    cases['drive'] = (est, gt, t, 10)
    n = 7   # shorter than the window; no timestamps (index axis)
    gt = rs.randn(n, 6)
    cases['short'] = (gt + 0.2 * rs.randn(n, 6), gt, None, 10)
    n = 250  # odd window
    gt = rs.randn(n, 6)
    cases['odd'] = (gt + rs.standard_t(3, (n, 6)), gt, np.cumsum(rs.uniform(0.05, 0.15, n)), 7)
    return cases


def main():
    sys.dont_write_bytecode = True
    import matplotlib
    matplotlib.use('Agg')
    import logging
    logging.disable(logging.CRITICAL)
    sys.path.insert(0, REF)
    from evaluation.compute_velocity_error import VelocityErrorEvaluator
    out = {}
    for name, (est, gt, ts, w) in tracks().items():
        ev = VelocityErrorEvaluator()
        out[f'{name}_est'], out[f'{name}_gt'], out[f'{name}_window'] = est, gt, np.int64(w)
        if ts is not None:
            out[f'{name}_ts'] = ts
        res = ev.compute_velocity_errors(est, gt, ts)
        for c, m in res['component_metrics'].items():
            for k, v in m.items():
                out[f'{name}_c_{c}_{k}'] = np.float64(v)
        for k, v in res['overall_metrics'].items():
            out[f'{name}_o_{k}'] = np.float64(v)
        tr = ev.analyze_error_trends(res, window_size=w)
        for k in ('moving_avg_errors', 'drift_coefficients', 'error_variance'):
            out[f'{name}_t_{k}'] = tr[k]
        out[f'{name}_report'] = np.array(ev.generate_error_report(res, tr))
    np.savez_compressed(os.path.join(OUT, 'golden_velocity_error.npz'), **out)
    print('wrote', len(out), 'arrays')


if __name__ == '__main__':
    main()

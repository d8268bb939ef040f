"""Velocity error statistics (drop-in evaluation.compute_velocity_error, host-side numpy by design: an [N, 6]
reduction) against golden vectors recorded from the reference's
evaluation/compute_velocity_error.py:46-251 by tests/golden/gen_velocity_error.py."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'golden_velocity_error.npz')


@pytest.mark.parametrize('case', ['drive', 'short', 'odd'])
def test_velocity_errors_match_reference(case):
    from evaluation.compute_velocity_error import VelocityErrorEvaluator
    g = np.load(GOLD)
    ts = g[f'{case}_ts'] if f'{case}_ts' in g.files else None
    ev = VelocityErrorEvaluator()
    res = ev.compute_velocity_errors(g[f'{case}_est'], g[f'{case}_gt'], ts)
    for c, m in res['component_metrics'].items():
        for k, v in m.items():
            np.testing.assert_allclose(v, g[f'{case}_c_{c}_{k}'], rtol=1e-12, atol=1e-15, err_msg=(c, k))
    for k, v in res['overall_metrics'].items():
        np.testing.assert_allclose(v, g[f'{case}_o_{k}'], rtol=1e-12, atol=1e-15, err_msg=k)
    tr = ev.analyze_error_trends(res, window_size=int(g[f'{case}_window']))
    # the moving average runs through a prefix sum: f64 rounding differs from a per-window mean by ~1e-15
    np.testing.assert_allclose(tr['moving_avg_errors'], g[f'{case}_t_moving_avg_errors'], rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(tr['drift_coefficients'], g[f'{case}_t_drift_coefficients'], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(tr['error_variance'], g[f'{case}_t_error_variance'], rtol=1e-12, atol=1e-15)
    assert ev.generate_error_report(res, tr) == str(g[f'{case}_report'])


def test_velocity_errors_shape_checks():
    from evaluation.compute_velocity_error import VelocityErrorEvaluator
    ev = VelocityErrorEvaluator()
    with pytest.raises(ValueError):
        ev.compute_velocity_errors(np.zeros((4, 6)), np.zeros((5, 6)))
    with pytest.raises(ValueError):
        ev.compute_velocity_errors(np.zeros((4, 5)), np.zeros((4, 5)))


def test_evaluate_velocity_errors_files(tmp_path):
    import matplotlib
    matplotlib.use('Agg')
    from evaluation.compute_velocity_error import evaluate_velocity_errors
    rs = np.random.RandomState(3)
    gt_v, gt_w = rs.randn(40, 3), rs.randn(40, 3)
    np.savez(tmp_path / 'gt.npz', velocity=gt_v, angular_velocity=gt_w)
    np.savez(tmp_path / 'est.npz', velocity=gt_v + 0.1 + 0.01 * rs.randn(40, 3), angular_velocity=gt_w)
    np.save(tmp_path / 'ts.npy', np.arange(40) * 0.1)
    res = evaluate_velocity_errors(str(tmp_path / 'est.npz'), str(tmp_path / 'gt.npz'), str(tmp_path / 'out.npz'),
                                   str(tmp_path / 'ts.npy'))
    np.testing.assert_allclose(res['component_metrics']['vx']['bias'], 0.1, atol=0.01)
    for suffix in ('_report.md', '_errors.png', '_comparison.png', '.npz'):
        assert (tmp_path / f'out{suffix}').exists()

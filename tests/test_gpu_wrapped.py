"""GPU parity of rows a30/a31: cross-frame association and the wrapped-phase solvers (librsl rsl_associate /
rsl_wrapped_solve through the drop-in classes) against the reference's own results in golden_wrapped.npz.

Parity contract: the association is exact; the wrapped cost is multimodal (one basin per
0.0195 m/s), so the solvers must reach a cost <= the reference's differential-evolution cost on the same
associations, and the reported cost must equal the oracle's restatement of the reference cost at the
reported motion (1e-9 relative).  The reference's Improved step 1 DE stops at maxiter without converging on
this data (scipy success=False -> the reference returns 'Step 1 failed'); its best cost is still recorded and
is the bound used here.
"""
import numpy as np
import pytest

import radar_oracle as O

pytestmark = pytest.mark.gpu

K = 4 * np.pi * 0.1 / (3e8 / 77e9)
TOL = 1e-9


def _targets(z, p):
    return [{'range_m': float(r), 'azimuth_rad': float(a), 'spatial_signature': s, 'range_bin': int(rb),
             'doppler_bin': int(db)}
            for r, a, s, rb, db in zip(z[f'{p}_range_m'], z[f'{p}_azimuth_rad'], z[f'{p}_sig'], z[f'{p}_range_bin'],
                                       z[f'{p}_doppler_bin'])]


def _geometry(z):
    r = z['cur_range_m'][z['assoc_cur']]
    az = z['cur_azimuth_rad'][z['assoc_cur']]
    pos = np.stack([r * np.cos(az), r * np.sin(az), np.zeros_like(r)], axis=1)
    return pos, np.stack([az, np.zeros_like(az)], axis=1), z['assoc_phase']


def test_association_exact(ctx, golden):
    from src.algorithms.velocity_solver_improved import ImprovedVelocitySolver
    z = golden('wrapped')
    cur, prev = _targets(z, 'cur'), _targets(z, 'prev')
    assoc = ImprovedVelocitySolver().associate_targets_across_frames(cur, prev)
    ci = [cur.index(a['current']) for a in assoc]
    pi = [prev.index(a['previous']) for a in assoc]
    assert ci == z['assoc_cur'].tolist() and pi == z['assoc_prev'].tolist()
    assert np.abs(np.array([a['distance'] for a in assoc]) - z['assoc_dist']).max() <= 1e-12
    assert np.abs(np.array([a['temporal_phase_diff'] for a in assoc]) - z['assoc_phase']).max() <= 1e-15


def test_association_edge_cases(ctx):
    from rsl import ops
    m, d = ops.associate(np.zeros((0, 2)), np.ones((3, 2)), 5.0)
    assert m.size == 0
    m, d = ops.associate(np.array([[0.0, 0.0], [0.1, 0.0]]), np.zeros((0, 2)), 5.0)
    assert (m == -1).all()
    # equal distances: the lowest previous index wins; a used target is not reused
    m, d = ops.associate(np.array([[0.0, 0.0], [0.0, 0.0]]), np.array([[1.0, 0.0], [-1.0, 0.0], [9.0, 0.0]]), 5.0)
    assert m.tolist() == [0, 1] and d.tolist() == [1.0, 1.0]
    # strict threshold
    m, _ = ops.associate(np.array([[0.0, 0.0]]), np.array([[5.0, 0.0]]), 5.0)
    assert m.tolist() == [-1]
    rs = np.random.RandomState(3)
    cur, prev = rs.uniform(-20, 20, (300, 2)), rs.uniform(-20, 20, (280, 2))
    m, d = ops.associate(cur, prev, 2.0)
    mo, do = O.associate_greedy(cur, prev, 2.0)
    assert (m == mo).all() and np.allclose(d[m >= 0], do[mo >= 0], rtol=0, atol=1e-12)


def test_improved_solver_beats_reference_de(ctx, golden):
    from src.algorithms.velocity_solver_improved import ImprovedVelocitySolver
    z = golden('wrapped')
    solver = ImprovedVelocitySolver()
    res = solver.solve_velocity_with_association(_targets(z, 'cur'), _targets(z, 'prev'), dt=0.1)
    assert res['success'] and res['num_associations'] == len(z['assoc_cur'])
    pos, ang, y = _geometry(z)
    x = np.concatenate([res['velocity'], res['angular_velocity']])
    assert abs(O.improved_cost(x, pos, ang, y, K) - res['cost']) <= TOL * res['cost']
    ref = float(z['imp_de_fun'][0])  # reference step-1 DE best (3-D, w = 0)
    assert res['step1_result'].fun <= ref * (1 + TOL), (res['step1_result'].fun, ref)
    assert res['cost'] <= ref * (1 + TOL)
    assert np.all(np.abs(res['velocity'][:2]) <= 50) and abs(res['velocity'][2]) <= 10
    r = y - O.phase_pred(x, pos, ang, K)
    assert np.abs(np.arctan2(np.sin(r), np.cos(r)) - res['residuals']).max() < 1e-9


@pytest.mark.parametrize('tag', ['adv', 'advp'])
def test_advanced_optimizer_beats_reference_de(ctx, golden, tag):
    from src.algorithms.advanced_velocity_optimization import AdvancedVelocityOptimizer
    from src.algorithms.velocity_solver_improved import ImprovedVelocitySolver
    z = golden('wrapped')
    prev = z['advp_prev'] if tag == 'advp' else None
    assoc = ImprovedVelocitySolver().associate_targets_across_frames(_targets(z, 'cur'), _targets(z, 'prev'))
    opt = AdvancedVelocityOptimizer(use_parallel=False, num_optimization_runs=2)
    res = opt.run_robust_optimization(assoc, 0.1, previous_motion=prev)
    assert res['success'] and res['successful_runs'] == 2
    pos, ang, y = _geometry(z)
    x = np.concatenate([res['velocity'], res['angular_velocity']])
    assert abs(O.advanced_cost(x, pos, ang, y, K, prev) - res['cost']) <= TOL * res['cost']
    assert res['cost'] <= float(z[f'{tag}_cost']) * (1 + TOL), (res['cost'], float(z[f'{tag}_cost']))
    assert np.array_equal(np.array(opt.adaptive_bounds['velocity_bounds']), z[f'{tag}_bounds'])
    assert len(opt.velocity_history) == 1


def test_advanced_adaptive_bounds_update(ctx):
    """Second solve: bounds follow update_adaptive_bounds (advanced_velocity_optimization.py:94-151)."""
    from src.algorithms.advanced_velocity_optimization import AdvancedVelocityOptimizer
    opt = AdvancedVelocityOptimizer()
    opt.update_adaptive_bounds(np.array([10.0, -4.0, 0.0]), np.zeros(3))
    opt.update_adaptive_bounds(np.array([12.0, -5.0, 1.0]), np.array([0.0, 0.0, 0.5]))
    vb = opt.adaptive_bounds['velocity_bounds']
    assert vb[0] == (-50.0, min(50.0, 12.0 + min(10.0, np.linalg.norm([12, -5, 1]) * 0.5)))
    assert vb[1] == (max(-50.0, -5.0 - min(10.0, np.linalg.norm([12, -5, 1]) * 0.5)), 50.0)
    assert opt.adaptive_bounds['acceleration_bounds'][0] == (-40.0, 40.0)


# More reference DE runs (tests/golden/gen_wrapped2.py): other target counts, the pipeline's
# lambda = fc / c (run_ego_motion_pipeline.py:246), previous motion.  Where the reference's DE does not converge it
# returns success False ('Step 1 failed', velocity_solver_improved.py:398-400; 'All optimization runs failed',
# advanced_velocity_optimization.py) while the build reports its basin-resolved minimum with success True
# (INTEGRATION.md); the contract is the cost: never above the reference's best DE cost on the same associations.
WIDE = ['imp_n20', 'imp_lam', 'adv_n60', 'advp_n30', 'adv_lam']


@pytest.mark.parametrize('case', WIDE)
def test_wrapped_solvers_vs_reference_de_wide(ctx, golden, case):
    from src.algorithms.advanced_velocity_optimization import AdvancedVelocityOptimizer
    from src.algorithms.velocity_solver_improved import ImprovedVelocitySolver
    z = golden(f'wrapped_{case}')
    lam = float(z['lambda_c'])
    k = 4 * np.pi * 0.1 / lam
    imp = ImprovedVelocitySolver(lambda_c=lam)
    cur, prev = _targets(z, 'cur'), _targets(z, 'prev')
    assoc = imp.associate_targets_across_frames(cur, prev)
    assert [cur.index(a['current']) for a in assoc] == z['assoc_cur'].tolist()
    assert [prev.index(a['previous']) for a in assoc] == z['assoc_prev'].tolist()
    assert np.abs(np.array([a['temporal_phase_diff'] for a in assoc]) - z['assoc_phase']).max() <= 1e-15
    pos, ang, y = _geometry(z)
    de = z['de_fun']
    if str(z['solver']) == 'improved':
        res = imp.two_step_optimization(assoc, 0.1)
        assert res['success']
        x = np.concatenate([res['velocity'], res['angular_velocity']])
        assert abs(O.improved_cost(x, pos, ang, y, k) - res['cost']) <= TOL * res['cost']
        assert res['step1_result'].fun <= float(de[0]) * (1 + TOL), (res['step1_result'].fun, float(de[0]))
        if bool(z['success']):  # the reference's 6-D step 2 converged: its final cost bounds ours
            assert res['cost'] <= float(z['cost']) * (1 + TOL), (res['cost'], float(z['cost']))
    else:
        pm = z['prev_motion'] if 'prev_motion' in z else None
        opt = AdvancedVelocityOptimizer(use_parallel=False, num_optimization_runs=2, lambda_c=lam)
        res = opt.run_robust_optimization(assoc, 0.1, previous_motion=pm)
        assert res['success'] and res['successful_runs'] == 2
        x = np.concatenate([res['velocity'], res['angular_velocity']])
        assert abs(O.advanced_cost(x, pos, ang, y, k, pm) - res['cost']) <= TOL * res['cost']
        assert res['cost'] <= float(de.min()) * (1 + TOL), (res['cost'], float(de.min()))
        if bool(z['success']):  # bounds follow the reference's update after a converged run
            assert np.array_equal(np.array(opt.adaptive_bounds['velocity_bounds']), z['bounds_after'])


@pytest.mark.parametrize('case', ['adv_n60', 'imp_n20'])
def test_wrapped_search_latency(ctx, golden, case, record_property):
    """the stage-1 grid of rsl_wrapped_search at the reference's own scale (+-50 m/s box, 77 GHz, dt 0.1:
    spacing 0.5 x 2 pi / k = 9.7 mm/s, ~10^4 points per axis, ~10^8 starts) — its per-call latency is measured and
    printed (DESIGN.md §3 records it), and bounded here so a regression in the start count cannot go unnoticed."""
    import math
    import time
    import torch
    from rsl import ops
    z = golden(f'wrapped_{case}')
    k = 4 * np.pi * 0.1 / float(z['lambda_c'])
    pos, ang, y = _geometry(z)
    lo = [-50.0, -50.0, -10.0, -10.0, -10.0, -10.0]
    hi = [50.0, 50.0, 10.0, 10.0, 10.0, 10.0]
    ops.wrapped_search(pos, ang, y, k, mode=0, lo=lo, hi=hi, nv=3, ctx=ctx)  # warm-up (code objects, scratch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x, cost = ops.wrapped_search(pos, ang, y, k, mode=0, lo=lo, hi=hi, nv=3, ctx=ctx)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    g = min(32768, math.ceil(100.0 / (0.5 * 2 * math.pi / k)))
    print(f'wrapped_search {case}: n={len(y)} targets, grid {g} x {g} = {g * g:.3g} starts, '
          f'{dt * 1e3:.1f} ms per call, cost {cost:.4f}')
    record_property('wrapped_search_ms', dt * 1e3)
    assert np.isfinite(cost) and dt < 5.0

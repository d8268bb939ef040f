"""GPU: the reference-compatible classes (src.*) against the golden vectors of the reference itself and
against the oracle, through the C ABI (librsl.so).  Tolerances: tests/parity.py."""
import numpy as np
import pytest

import parity as P
import radar_oracle as O

pytestmark = pytest.mark.gpu

NAMES = ['tiny', 'odd400', 'cfg1']


@pytest.fixture(scope='module')
def data(golden, ctx):
    out = {}
    for n in NAMES:
        z = golden(n)
        np.random.seed(int(z['seed']))
        cube = O.synthesize_frame(O.TEST_SCENE, chirp_duration=float(z['chirp_duration']), num_chirps=int(z['C']),
                                  num_antennas=int(z['A']))
        out[n] = (z, cube, O.range_doppler_spectrum(cube, chirp_duration=float(z['chirp_duration'])))
    return out


def pre_for(z):
    from src.radar_signal.dechirp import SignalPreprocessor
    return SignalPreprocessor(fc=77e9, bandwidth=1e9, chirp_duration=float(z['chirp_duration']), pri=100e-6,
                              num_chirps=int(z['C']), sampling_rate=10e6)


@pytest.mark.parametrize('name', NAMES)
def test_rds_vs_golden(data, name):
    z, cube, ref = data[name]
    pre = pre_for(z)
    rds = pre.generate_range_doppler_spectrum(cube)
    assert rds.dtype == np.complex128 and rds.shape == ref.shape
    amax = float(z['rds_absmax'])
    err = np.abs(rds.reshape(-1)[z['rds_sample_idx']] - z['rds_sample']).max() / amax
    assert err <= P.RDS_ATOL_REL
    assert P.rds_error(rds, ref) <= P.RDS_ATOL_REL
    C = int(z['C'])
    sub = pre.generate_range_doppler_spectrum(cube, chirp_subset=(2, C - 3))
    idx = z['rds_sample_idx'][z['rds_sample_idx'] < sub.size]
    assert np.abs(sub.reshape(-1)[idx] - z['rds_sub_sample']).max() / amax <= P.RDS_ATOL_REL
    if name == 'tiny':
        assert P.rds_error(rds, z['rds']) <= P.RDS_ATOL_REL


@pytest.mark.parametrize('name', NAMES)
def test_peaks_vs_golden(data, name):
    z, cube, ref = data[name]
    pre = pre_for(z)
    info = pre.extract_range_doppler_peaks(ref)
    pk = info['peaks']
    ga = np.array([p['antenna'] for p in pk])
    gi = np.array([p['range_bin'] for p in pk])
    gj = np.array([p['doppler_bin'] for p in pk])
    key = lambda a, i, j: set(zip(a.tolist(), i.tolist(), j.tolist()))
    got, want = key(ga, gi, gj), key(z['peak_a'], z['peak_i'], z['peak_j'])
    diff = got ^ want
    A, S, C = ref.shape
    m = np.zeros(ref.shape, bool)
    m[ga, gi, gj] = True
    from rsl import tables
    ng, nr, nd, nu = P.peak_diff(m, ref, gate=tables.range_gate(1e9, S, 1.0, 200.0))
    assert nu == 0 and len(diff) == nd
    assert nd <= max(2, 1e-4 * nr)
    if nd == 0:  # same order as the reference
        assert (ga == z['peak_a']).all() and (gi == z['peak_i']).all() and (gj == z['peak_j']).all()
        pdb = np.array([p['power_db'] for p in pk])
        assert np.abs(pdb - z['peak_db']).max() < 1e-4
    assert type(pk[0]['antenna']) is int and isinstance(pk[0]['range_bin'], np.integer)
    assert set(pk[0]) == {'antenna', 'range_bin', 'doppler_bin', 'range_m', 'doppler_hz', 'power_db'}
    assert np.abs(info['power_spectrum_db'] - 10 * np.log10(np.abs(ref) ** 2 + 1e-12)).max() < 1e-3
    assert np.array_equal(info['range_bins_m'], z['range_bins_m'])
    # other threshold / gate
    i30 = pre.extract_range_doppler_peaks(ref, threshold_db=-30.0, min_range=5.0, max_range=50.0)['peaks']
    got30 = key(np.array([p['antenna'] for p in i30]), np.array([p['range_bin'] for p in i30]),
                np.array([p['doppler_bin'] for p in i30]))
    assert len(got30 ^ key(z['peak30_a'], z['peak30_i'], z['peak30_j'])) <= 2


@pytest.mark.parametrize('name', NAMES)
def test_process_targets_vs_golden(data, name):
    from src.angle_estimation.angle_estimation import AngleEstimator
    z, cube, ref = data[name]
    est = AngleEstimator(fc=77e9, antenna_spacing=3e8 / (2 * 77e9), num_antennas=int(z['A']))
    sel = z['sel']
    peaks = [{'antenna': int(z['peak_a'][k]), 'range_bin': z['peak_i'][k], 'doppler_bin': z['peak_j'][k],
              'range_m': z['range_bins_m'][z['peak_i'][k]], 'doppler_hz': 0.0, 'power_db': z['peak_db'][k]}
             for k in sel]
    tm = est.process_targets(ref, {'peaks': peaks}, 'music')
    assert len(tm) == len(sel)
    st = O.steering_matrix(O.azimuth_grid(), int(z['A']))
    idx = np.array([np.argmin(np.abs(est.azimuth_grid - t['azimuth_deg'])) for t in tm])
    nm, nu, _ = P.doa_diff(idx, z['sig'], st, 'music')
    assert nu == 0 and nm <= P.doa_flip_budget(len(sel)), (nm, nu)
    assert np.abs(np.array([t['spatial_signature'] for t in tm]) - z['sig']).max() < 1e-5
    spec = np.array([t['spectrum'] for t in tm[:len(z['music_spec'])]])
    rs = z['music_spec']
    ok = rs > 0
    assert np.abs(spec[ok] - rs[ok]).max() / rs[ok].max() < 1e-4
    te = est.process_targets(ref, {'peaks': peaks}, 'esprit')
    emax, nnan = P.esprit_diff(np.array([t['azimuth_deg'] for t in te]), z['esprit_deg'])
    assert nnan == 0 and emax <= P.ESPRIT_TOL_DEG
    tb = est.process_targets(ref, {'peaks': peaks}, 'beamforming')
    idx = np.array([np.argmin(np.abs(est.azimuth_grid - t['azimuth_deg'])) for t in tb])
    nm, nu, _ = P.doa_diff(idx, z['sig'], st, 'beamforming')
    assert nu == 0 and nm <= P.doa_flip_budget(len(sel)), (nm, nu)
    bs = np.array([t['spectrum'] for t in tb[:len(z['bf_spec'])]])
    assert np.abs(bs - z['bf_spec']).max() < 1e-4
    assert est.process_targets(ref, {'peaks': peaks[:3]}, 'capon') == []
    assert set(tm[0]) == {'range_m', 'doppler_hz', 'power_db', 'azimuth_deg', 'azimuth_rad', 'antenna', 'range_bin',
                          'doppler_bin', 'spatial_signature', 'spectrum'}


def test_single_signature_methods(golden):
    from src.angle_estimation.angle_estimation import AngleEstimator
    z = golden('cfg1')
    est = AngleEstimator()
    for k in range(4):
        s = z['sig'][k]
        a, spec = est.estimate_angle_music(s)
        assert a == z['music_deg'][k] and spec.shape == (361,)
        assert np.abs(est.music_spectrum(s) - z['music_spec'][k]).max() / z['music_spec'][k].max() < 1e-4
        assert abs(est.estimate_angle_esprit(s) - z['esprit_deg'][k]) < P.ESPRIT_TOL_DEG
        b, bspec = est.estimate_angle_beamforming(s)
        assert b == z['bf_deg'][k]
    # num_sources != 1 runs (general subspace forms: test_music_num_sources_general / test_esprit_num_sources_general)
    assert est.music_spectrum(z['sig'][0], num_sources=2).shape == (len(est.azimuth_grid),)


@pytest.mark.parametrize('name', NAMES)
def test_velocity_solver_vs_golden(data, name):
    from src.angle_estimation.angle_estimation import AngleEstimator
    from src.velocity_solver.velocity_solver import VelocitySolver
    z, cube, ref = data[name]
    top = z['vel_top']
    targets = [{'range_m': 10.0 + k, 'azimuth_rad': np.radians(z['music_deg'][k]),
                'spatial_signature': z['sig'][k]} for k in top]
    vs = VelocitySolver(fc=77e9, num_antennas=int(z['A']))
    r = vs.solve_velocity(ref, targets, dt=0.1)
    assert r['success'] and r['num_targets'] == len(top)
    assert abs(r['cost'] - float(z['vel_cost'])) <= P.VEL_COST_RTOL * float(z['vel_cost'])
    assert abs(r['velocity'][0] - z['vel_v'][0]) < P.VEL_ATOL and abs(r['velocity'][1] - z['vel_v'][1]) < P.VEL_ATOL
    assert abs(r['rmse'] - float(z['vel_rmse'])) < 1e-6 and abs(r['max_residual'] - float(z['vel_maxres'])) < 1e-3
    # DE stops ~1e-7 m/s from the optimum; residuals scale by k = 4 pi dt / lambda = 322 rad per m/s
    assert np.abs(r['residuals'] - z['vel_res']).max() < 4 * np.pi * 0.1 / vs.lambda_c * P.VEL_ATOL
    for key in ('velocity', 'angular_velocity', 'cost', 'rmse', 'max_residual', 'residuals', 'predicted_phases',
                'observed_phases', 'num_targets', 'step1_result', 'step2_result'):
        assert key in r
    # the drop-in pipeline's wavelength bug (run_ego_motion_pipeline.py:246)
    vb = VelocitySolver(fc=77e9, lambda_c=77e9 / 3e8, num_antennas=8, antenna_spacing=3e8 / (2 * 77e9))
    rb = vb.solve_velocity(ref, targets, dt=0.1)
    assert abs(rb['cost'] - float(z['velbug_cost'])) <= P.VEL_COST_RTOL * float(z['velbug_cost'])
    assert abs(rb['velocity'][0] - z['velbug_v'][0]) < 0.05 and abs(rb['velocity'][1] - z['velbug_v'][1]) < 0.05
    assert vs.solve_velocity(ref, targets[:2])['success'] is False


def test_velocity_general_6dof_vs_scipy():
    """General (non-degenerate) positions/elevations: the device BVLS equals scipy's bounded LS."""
    from scipy.optimize import lsq_linear
    from src.velocity_solver.velocity_solver import VelocitySolver
    rs = np.random.RandomState(3)
    N = 40
    pos = rs.randn(N, 3) * 20
    ang = np.stack([rs.uniform(-1.5, 1.5, N), rs.uniform(-0.3, 0.3, N)], axis=1)
    vs = VelocitySolver()
    k = 4 * np.pi * 0.1 / vs.lambda_c
    ce = np.cos(ang[:, 1])
    d = np.stack([ce * np.cos(ang[:, 0]), ce * np.sin(ang[:, 0]), np.sin(ang[:, 1])], axis=1)
    J = k * np.concatenate([d, np.cross(pos, d)], axis=1)
    xt = np.array([3.0, -2.0, 0.5, 0.05, -0.02, 0.1])
    for scale in (1.0, 1e-3):
        y = J @ xt * scale + 0.01 * rs.randn(N)
        r = vs.two_step_optimization(pos, ang, y, 0.1)
        lo = [-50, -50, -10, -10, -10, -10]
        hi = [50, 50, 10, 10, 10, 10]
        ref = lsq_linear(J, y, bounds=(lo, hi), method='bvls', tol=1e-14)
        x = np.concatenate([r['velocity'], r['angular_velocity']])
        assert np.abs(x - ref.x).max() < 1e-6
        assert abs(r['cost'] - 2 * ref.cost) < 1e-8 * max(1.0, 2 * ref.cost)
        assert abs(vs.cost_function(x, pos, ang, y, 0.1) - r['cost']) < 1e-9 * max(1, r['cost'])
        pm = vs.compute_phase_difference_model(pos, ang, x[:3], x[3:], 0.1)
        assert np.abs(pm - J @ x).max() < 1e-9
    # heavily bounded case: target far outside the box
    y = J @ np.array([400.0, -300.0, 40.0, 30.0, -30.0, 20.0])
    r = vs.two_step_optimization(pos, ang, y, 0.1)
    ref = lsq_linear(J, y, bounds=([-50, -50, -10, -10, -10, -10], [50, 50, 10, 10, 10, 10]), method='bvls')
    x = np.concatenate([r['velocity'], r['angular_velocity']])
    assert abs(r['cost'] - 2 * ref.cost) <= 1e-7 * 2 * ref.cost


def test_preprocess_helpers():
    from src.radar_signal.dechirp import SignalPreprocessor
    pre = SignalPreprocessor(chirp_duration=25.6e-6)
    rs = np.random.RandomState(1)
    x = rs.randn(256) + 1j * rs.randn(256)
    ref = O.reference_chirp(77e9, 1e9, 25.6e-6, 10e6)
    w = O.window('hann', 256)
    exp = (x * np.conj(ref)) * w
    exp = exp - np.mean(exp)
    got = pre.process_chirp(x, ref)
    assert np.abs(got - exp).max() < 1e-5 * np.abs(exp).max()
    assert np.abs(pre.dechirp_signal(x) - x * np.conj(ref)).max() < 1e-5 * np.abs(x).max()
    assert np.abs(pre.apply_window(x) - x * w).max() < 1e-5 * np.abs(x).max()
    assert np.abs(pre.remove_dc(x) - (x - x.mean())).max() < 1e-5 * np.abs(x).max()
    with pytest.raises(ValueError):
        pre.apply_window(x, 'kaiser')
    with pytest.raises(ValueError):  # frame sample count != int(T_c f_s): reference broadcast error
        SignalPreprocessor(chirp_duration=40e-6).generate_range_doppler_spectrum(np.zeros((8, 16, 256), complex))


def test_robust_sequence_vs_golden(golden):
    from src.algorithms.robust_angle_estimation import RobustAngleEstimator
    from src.robust_angle_estimation import RobustAngleEstimator as R2
    assert R2 is RobustAngleEstimator
    z = golden('robust')
    rob = RobustAngleEstimator(fc=77e9, num_antennas=8, max_targets=40, confidence_threshold=0.55)
    rows = []
    for f in range(3):
        rds = z[f'rds{f}']
        tg = rob.process_targets_robust(rds, O.extract_peaks(rds), frame_timestamp=1.0 + f)
        for t in tg:
            ia = t['interference_analysis']
            rows.append([f, t['range_bin'], t['doppler_bin'], t['azimuth_deg'], t['confidence'],
                         float(ia['num_sources']), float(ia['is_multipath']), t['power_db']])
    rows = np.array(rows)
    ref = z['rows']
    assert rows.shape == ref.shape
    assert np.array_equal(rows[:, :3], ref[:, :3])
    assert np.abs(rows[:, 3] - ref[:, 3]).max() < 1e-6
    assert np.abs(rows[:, 4] - ref[:, 4]).max() < 1e-5
    assert np.array_equal(rows[:, 5:7], ref[:, 5:7])
    st = rob.get_target_statistics()
    assert st['total_targets_tracked'] == int(z['stats'][0]) and st['active_targets'] == int(z['stats'][1])
    assert abs(st['average_confidence'] - z['stats'][2]) < 1e-5


def _householder_den(s, a, K):
    """numpy restatement of rsl_subspace.hip's basis: V = [s/|s|, Householder completion], den = sum_{noise j}
    |(P a)_j|^2 (test side; the reference's null-space columns for 2 <= K < M are LAPACK round-off, parity unpinned)."""
    M = len(s)
    lo = (K if K < M else M) if K >= 0 else max(M + K, 0)
    nx = np.linalg.norm(s)
    if nx == 0:
        return sum(abs(a[M - 1 - j]) ** 2 for j in range(lo, M))
    ph = s[0] / abs(s[0]) if abs(s[0]) > 0 else 1.0
    w = s.astype(complex).copy()
    w[0] -= -ph * nx
    pa = a - 2 * w * (np.vdot(w, a) / np.vdot(w, w).real)
    return float(np.sum(np.abs(pa[lo:]) ** 2))


def test_music_num_sources_general(ctx):
    """num_sources != 1 (angle_estimation.py:109-176): K = 1 through the general path equals the closed form; K >= M
    (no noise subspace) and zero signatures equal the reference's eigh outputs exactly (spectrum 0 / den = M - K);
    K = 0 equals 1 / |a|^2; 2 <= K < M follows the Householder-basis definition and never lowers the spectrum
    below K = 1's (den_K <= den_1)."""
    from src.angle_estimation.angle_estimation import AngleEstimator
    from rsl import ops
    est = AngleEstimator()
    grid, steer = est.azimuth_grid, est._steer
    rs = np.random.RandomState(7)
    sigs = rs.randn(6, 8) + 1j * rs.randn(6, 8)
    sigs /= np.linalg.norm(sigs, axis=1, keepdims=True)
    sigs[4] = steer[100] / np.sqrt(8)        # a pure steering vector: den -> 0 at grid point 100
    sigs[5] = 0                               # zero power
    closed = O.music_spectrum_closed(sigs[:5], steer)
    g1 = ops.subspace_music(sigs[:5], steer, 1)
    d1, dc = 1 / np.where(g1 > 0, g1, np.inf), 1 / np.where(closed > 0, closed, np.inf)
    assert np.abs(d1 - dc).max() < 1e-12
    for K in (8, 11):
        assert (ops.subspace_music(sigs, steer, K) == 0).all()
        ang, sp = est.estimate_angle_music(sigs[0], num_sources=K)
        ref = O.music_spectrum_eigh(sigs[0], grid, num_sources=K)
        assert ang == grid[np.argmax(ref)] == -90.0 and (sp == ref).all()
    for K in (0, 2, 3, 7, -1, -3):
        got = ops.subspace_music(sigs, steer, K)
        zr = O.music_spectrum_eigh(sigs[5], grid, num_sources=K)  # zero signature: reference-determined
        assert np.abs(got[5] - zr).max() < 1e-12, K
        for n in range(5):
            want = np.array([_householder_den(sigs[n], steer[g], K) for g in range(len(grid))])
            live = want > 1e-9
            assert (got[n][~live] == 0).all() or K <= 0, (K, n)  # den <= 1e-12 -> 0 (:149-152)
            dg = 1 / got[n][live]
            assert np.abs(dg - want[live]).max() < 1e-11 or K == 0, (K, n)
            if K == 0:  # den = |a|^2 = M for every grid point (the reference's argmax is round-off)
                assert np.abs(got[n] - 1 / 8).max() < 1e-12
            if K >= 2:
                assert (got[n] >= g1[min(n, 4)] * (1 - 1e-9)).all() if n < 5 else True


def test_esprit_num_sources_general(ctx):
    """ESPRIT num_sources != 1 (angle_estimation.py:178-225): K = 0 -> 0.0 (the reference's eigvals(empty)[0]
    IndexError, caught); K = 1 equals the closed form; K = 2: the angle of one of the two eigenvalues of the
    reference's Phi (which of the two is LAPACK's order: unpinned); K >= 3 runs (null-space columns: unpinned)."""
    from src.angle_estimation.angle_estimation import AngleEstimator
    from scipy.linalg import svd
    est = AngleEstimator()
    rs = np.random.RandomState(3)
    lam = 3e8 / 77e9
    for n in range(8):
        s = np.exp(1j * np.arange(8) * rs.uniform(-2, 2)) + 0.3 * (rs.randn(8) + 1j * rs.randn(8))
        s /= np.linalg.norm(s)
        assert est.estimate_angle_esprit(s, num_sources=0) == 0.0 == O.esprit_svd(s, num_sources=0)
        assert abs(est.estimate_angle_esprit(s, num_sources=1) - O.esprit_closed(s[None])[0]) < 1e-5  # fp32 path
        U, _, _ = svd(np.column_stack([s[:-1], s[1:]]))
        Phi = np.linalg.pinv(U[:-1, :2]) @ U[1:, :2]
        cands = np.degrees(np.arcsin(np.angle(np.linalg.eigvals(Phi)) * lam / (2 * np.pi * (lam / 2))))
        got = est.estimate_angle_esprit(s, num_sources=2)
        assert np.min(np.abs(cands - got)) < 1e-7, (got, cands)
        for K in (3, 5, 7, 9, -2):
            v = est.estimate_angle_esprit(s, num_sources=K)
            assert isinstance(v, float)

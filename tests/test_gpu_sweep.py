"""Randomised parity sweep of the batched chain (librsl via rsl.RadarChain) against the oracle.

test_gpu_chain.py checks fixed shapes on the reference's own test scene (tests/test_synth_raw.py:165-190).  Here each
case draws its own scene (3-12 scatterers: range, azimuth, RCS, radial velocity), noise power, frame shape, detection
threshold, range gate, window (hann / hamming / blackman, dechirp.py:99-106), DC removal, grid resolution, DoA method
(MUSIC / beamforming, angle_estimation.py:109-154 / :227-251) and ridge, from a fixed seed, and checks RDS, peak
masks and entry order, DoA argmax (the same relative-gap rule and flip budget as test_gpu_chain), ESPRIT, spatial
phase and the velocity solve on 2 frames; every third case also writes the spectrum of every cell (MUSIC 1/den or
beamforming P, angle_estimation.py:143-154, :299) and checks it against the oracle's fp64 spectrum.
"""
import numpy as np
import pytest

import parity as P
import radar_oracle as O

pytestmark = pytest.mark.gpu

SHAPES = [(8, 16, 3.2e-6), (8, 16, 40e-6), (8, 64, 25.6e-6), (4, 32, 12.8e-6), (16, 32, 12.8e-6), (2, 64, 6.4e-6),
          (8, 128, 51.2e-6), (6, 48, 9.6e-6)]
NCASES = 24


def _case(k):
    rs = np.random.RandomState(9000 + k)
    A, C, Tc = SHAPES[k % len(SHAPES)]
    scene = [{'range_sc': float(rs.uniform(3.0, 70.0)), 'azimuth_sc': float(np.radians(rs.uniform(-70, 70))),
              'rcs': float(rs.uniform(-20.0, 0.0)), 'vr': float(rs.uniform(-15.0, 15.0))}
             for _ in range(rs.randint(3, 13))]
    kw = dict(threshold_db=float(rs.choice([-30.0, -20.0, -12.0])), min_range=float(rs.choice([0.0, 1.0, 5.0])),
              max_range=float(rs.choice([50.0, 200.0])), search_resolution=float(rs.choice([0.5, 1.0, 0.25])),
              method=str(rs.choice(['music', 'beamforming'])), ridge=float(rs.choice([0.0, 0.01])),
              window_type=str(rs.choice(['hann', 'hamming', 'blackman'])), dc_removal=bool(rs.rand() < 0.75))
    return A, C, Tc, scene, float(10 ** rs.uniform(-3, -1)), kw


def _mask_bool(words, C):
    A, S, W = words.shape
    bits = np.unpackbits(words.view(np.uint8).reshape(A, S, W, 8), axis=-1, bitorder='little')
    return bits.reshape(A, S, W * 64)[:, :, :C].astype(bool)


@pytest.mark.parametrize('k', range(NCASES))
def test_random_scene_parity(ctx, k):
    import rsl
    A, C, Tc, scene, noise, kw = _case(k)
    F = 2
    frames = []
    for f in range(F):
        np.random.seed(7000 + 31 * k + f)
        frames.append(O.synthesize_frame(scene, chirp_duration=Tc, num_chirps=C, num_antennas=A, noise_power=noise))
    frames = np.stack(frames)
    spectrum = k % 3 == 0  # every third case also writes the spectrum of every cell (K5'', angle_estimation.py:299)
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc, spectrum=spectrum, **kw)
    ch = rsl.RadarChain(cfg, F, ctx)
    ch.run(ctx.to_dev(frames.astype(np.complex64)))
    r = ch.results()
    rds, words = ch.rds.cpu().numpy(), ch.mask.cpu().numpy()
    if spectrum:
        from rsl.runtime import spectrum_rows
        spec = spectrum_rows(ch.spec, int(r['cell_base'][F])).cpu().numpy()
    grid_deg = O.azimuth_grid(cfg.search_range, cfg.search_resolution)
    steer = O.steering_matrix(grid_deg, A)
    lam = 3e8 / cfg.fc
    cb, eb = r['cell_base'], r['entry_base']
    tot_m = tot_n = 0
    stats = {}
    for f in range(F):
        ref = O.range_doppler_spectrum(frames[f], chirp_duration=Tc, window_type=cfg.window_type,
                                       dc_removal=cfg.dc_removal)
        assert P.rds_error(rds[f], ref) <= P.RDS_ATOL_REL, (k, f)
        ng, nr, nd, nu = P.peak_diff(_mask_bool(words[f], C), ref, threshold_db=cfg.threshold_db,
                                     gate=(ch.i_lo, ch.i_hi))
        assert nu == 0 and nd <= max(2, 1e-4 * nr), (k, f, ng, nr, nd, nu)
        if nd == 0:
            a, i, j, db = O.peak_arrays(ref, threshold_db=cfg.threshold_db, min_range=cfg.min_range,
                                          max_range=cfg.max_range)
            g = (i >= ch.i_lo) & (i <= ch.i_hi)
            a, i, j, db = a[g], i[g], j[g], db[g]
            sl = slice(eb[f], eb[f + 1])
            assert (r['e_ant'][sl] == a).all() and (r['e_rbin'][sl] == i).all() and (r['e_dbin'][sl] == j).all()
            assert len(db) == 0 or np.abs(r['e_pdb'][sl] - db).max() < 1e-4
        cs = slice(cb[f], cb[f + 1])
        rc = r['c_rc'][cs]
        if len(rc) == 0:
            continue
        ii, jj = rc // C, rc % C
        sigs = np.stack([O.spatial_signature(ref, i_, j_) for i_, j_ in zip(ii, jj)])
        nm, nun, _ = P.doa_diff(r['gidx'][cs], sigs, steer, cfg.method, stats=stats)
        assert nun == 0, (k, f, nm, nun, stats)
        ns, sgap = P.scan_flips(r['gidx'][cs], rds[f][:, ii, jj].T, steer, cfg.method)
        assert ns == 0, (k, f, 'scan-caused flips', ns, sgap)
        tot_m += nm
        tot_n += len(rc)
        if spectrum:  # den = 1/spectrum against the oracle's fp64 M - |a^H s|^2 (MUSIC), P itself (beamforming)
            got = spec[cs]
            n = np.arange(len(rc))
            assert P.spectrum_argmax_consistent(got.astype(np.float64), r['gidx'][cs], cfg.method), k
            if cfg.method == 'music':
                want = O.music_spectrum_closed(sigs, steer)
                assert ((got > 0) == (want > 0)).all(), k
                dg = np.where(got > 0, 1.0 / np.where(got > 0, got, 1.0), 0.0)
                dw = np.where(want > 0, 1.0 / np.where(want > 0, want, 1.0), 0.0)
                err = np.abs(dg - dw).max()
            else:
                err = np.abs(got - O.beamforming_spectrum(sigs, steer)).max()
            assert err < 2e-5, (k, f, err)
        if A >= 2:
            emax, nnan = P.esprit_diff(r['esprit'][cs], O.esprit_closed(sigs))
            assert nnan == 0 and emax <= P.ESPRIT_TOL_DEG, (k, f, emax, nnan)
            # spatial phase angle(s1 conj s0) (velocity_solver.py:136): against the same expression on the GPU's own
            # fp32 RDS values (the kernel's arithmetic), and against the oracle within the phase shift that the
            # cell's measured RDS error can cause (|ds| / |s| per element: weak cells next to strong ones move most)
            g = rds[f][:, ii, jj].T.astype(np.complex128)
            dg = np.angle(np.exp(1j * (r['phase'][cs] - O.observed_phase(g))))
            assert np.abs(dg).max() < 2e-5, (k, f, np.abs(dg).max())
            e = np.abs(g - ref[:, ii, jj].T)
            rr = np.abs(ref[:, ii, jj].T)
            bound = 2 * (e[:, 0] / np.maximum(rr[:, 0], 1e-300) + e[:, 1] / np.maximum(rr[:, 1], 1e-300)) + 2e-5
            dph = np.angle(np.exp(1j * (r['phase'][cs] - O.observed_phase(sigs))))
            assert (np.abs(dph) <= bound).all(), (k, f, np.abs(dph).max())
        w = np.array([bin(int(m) & 0xffffffff).count('1') for m in r['c_amask'][cs]])
        az = np.repeat(np.radians(grid_deg[r['gidx'][cs]]), w)
        y = np.repeat(r['phase'][cs], w)
        vx, vy, cost = O.velocity_ls(az, y, lambda_c=lam, ridge=cfg.ridge)
        v = r['velocity'][f]
        assert abs(v[2] - cost) <= P.VEL_COST_RTOL * max(cost, 1e-300) + 1e-12, (k, f, v[2], cost)
        assert abs(v[0] - vx) < P.VEL_ATOL and abs(v[1] - vy) < P.VEL_ATOL, (k, f, v[:2], vx, vy)
        assert int(v[5]) == len(y)
    print(f'\ncase {k} A{A} C{C} S{cfg.S} {kw}: {len(scene)} scatterers, noise {noise:.2e}, '
          f'DoA flips {tot_m} of {tot_n}')
    assert tot_m <= P.doa_flip_budget(tot_n, A, cfg.search_resolution), (k, tot_m, tot_n, stats)

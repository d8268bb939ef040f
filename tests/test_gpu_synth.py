"""Device synthetic cube generator (rsl_synth_pattern / rsl_synth_cube) against the oracle restatement of
simulate_raw.synthesize_frame (scripts/simulate_raw.py:147-221; bit-identical to the reference, pinned in
test_oracle_golden.py) for the deterministic part, and against the numpy Philox mirror (philox_ref.py) for the
noise.  Tolerances: cube 1e-6 of max|signal| (c64 rounding of fp64 values), fp64 pattern 1e-8 of it; noise 2e-5
absolute on unit-variance samples (fp32 logf / sincospif against fp64)."""
import numpy as np
import pytest

import philox_ref as PR
import radar_oracle as O

pytestmark = pytest.mark.gpu

SHAPES = {'cfg1': (8, 64, 25.6e-6), 'cfg2': (8, 128, 51.2e-6), 'cfg5': (16, 256, 102.4e-6)}


@pytest.mark.parametrize('name', list(SHAPES))
def test_pattern_matches_oracle(ctx, name):
    from rsl.synth import SyntheticCubes
    A, C, Tc = SHAPES[name]
    gen = SyntheticCubes(ctx, O.TEST_SCENE, chirp_duration=Tc, num_chirps=C, num_antennas=A, noise_power=0.0)
    cube = gen.generate(2).cpu().numpy()
    ref = O.synthesize_frame(O.TEST_SCENE, chirp_duration=Tc, num_chirps=C, num_antennas=A, noise_power=0.0,
                             rng=np.random.RandomState(0))
    scale = np.abs(ref).max()
    assert scale > 0
    for f in range(2):
        assert np.abs(cube[f] - ref).max() <= 1e-6 * scale
    # fp64 pattern: the chirp phase reaches 2.5e7 rad, whose fp64 representation alone is uncertain to ~3e-9 rad
    # (device sincos vs numpy exp differ by an ulp of the reduced argument)
    pat = gen.pattern.cpu().numpy()
    assert np.abs(pat - ref[:, 0, :]).max() <= 1e-8 * scale


def test_scatterer_edge_cases(ctx):
    from rsl.synth import SyntheticCubes
    scene = [{'range_sc': -5.0}, {'range_sc': float('nan')}, {'range_sc': 1e5, 'rcs': 0.0},
             {'range_sc': 30.0, 'azimuth_sc': 0.3, 'rcs': -5.0, 'vr': 2.0}]
    gen = SyntheticCubes(ctx, scene, chirp_duration=25.6e-6, num_chirps=4, num_antennas=4, noise_power=0.0)
    cube = gen.generate(1).cpu().numpy()[0]
    ref = O.synthesize_frame(scene, chirp_duration=25.6e-6, num_chirps=4, num_antennas=4, noise_power=0.0,
                             rng=np.random.RandomState(0))
    assert np.abs(cube - ref).max() <= 1e-6 * np.abs(ref).max()
    empty = SyntheticCubes(ctx, [], chirp_duration=25.6e-6, num_chirps=4, num_antennas=4, noise_power=0.0)
    assert not np.any(empty.generate(1).cpu().numpy())


def test_noise_matches_philox_mirror(ctx):
    from rsl.synth import SyntheticCubes
    gen = SyntheticCubes(ctx, [], chirp_duration=25.6e-6, num_chirps=8, num_antennas=4, noise_power=1.0)
    seed = 0x1234_5678_9ABC_DEF0
    got = gen.generate(3, seed=seed, frame0=5).cpu().numpy()
    ref = PR.noise(got.shape, seed, frame0=5)
    assert np.abs(got - ref).max() < 2e-5


def test_frame_blocks_compose_and_statistics(ctx):
    from rsl.synth import SyntheticCubes
    gen = SyntheticCubes(ctx, O.TEST_SCENE, chirp_duration=25.6e-6, num_chirps=64, num_antennas=8, noise_power=0.01)
    whole = gen.generate(6, seed=7).cpu().numpy()
    parts = np.concatenate([gen.generate(2, seed=7, frame0=f0).cpu().numpy() for f0 in (0, 2, 4)])
    assert np.array_equal(whole, parts)
    assert not np.array_equal(whole, gen.generate(6, seed=8).cpu().numpy())
    n = whole - gen.pattern.cpu().numpy()[None, :, None, :]
    # simulate_raw.py:216-218: sqrt(noise_power) (randn + j randn): each component has variance noise_power
    assert abs(n.real.var() - 0.01) < 3e-4 and abs(n.imag.var() - 0.01) < 3e-4
    assert abs(n.real.mean()) < 1e-3 and abs(n.imag.mean()) < 1e-3
    x = n.reshape(-1)
    assert abs(np.mean(x.real * x.imag)) < 3e-4                  # components uncorrelated
    assert abs(np.mean(x[:-1].real * x[1:].real)) < 3e-4         # neighbouring samples uncorrelated


def test_chain_on_synthetic_cubes(ctx):
    """Frames from the device generator run through the chain with the same decisions as the oracle."""
    import rsl
    import parity as P
    from rsl.synth import SyntheticCubes
    A, C, Tc = SHAPES['cfg1']
    gen = SyntheticCubes(ctx, O.TEST_SCENE, chirp_duration=Tc, num_chirps=C, num_antennas=A)
    cube = gen.generate(2, seed=3)
    ch = rsl.RadarChain(rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc), 2, ctx)
    ch.run(cube)
    res = ch.results()
    frames = cube.cpu().numpy().astype(np.complex128)
    for f in range(2):
        ref = O.range_doppler_spectrum(frames[f], chirp_duration=Tc)
        assert P.rds_error(ch.rds[f].cpu().numpy(), ref) <= P.RDS_ATOL_REL
        a, i, j, db = O.peak_arrays(ref)
        eb = res['entry_base']
        assert abs(int(eb[f + 1] - eb[f]) - len(a)) <= max(2, 1e-4 * len(a))

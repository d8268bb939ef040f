"""Batched MUSIC / beamforming spectrum (configs[1]: "range-Doppler FFT + MUSIC spectrum"): RadarChain with
spectrum=True writes f32 cell-blocked [cells / 32, G, 32] (RSL_DOA_SPEC_BLOCKED) from the Toeplitz f16-MFMA scan
(k_doa_toep with SPEC, uniform linear arrays); the f32-MFMA steering scan (k_doa_scan) writes every layout and is
the general path.
The reference stores spectrum f64[G] per target (angle_estimation.py:143-154, :299).

Tolerance: MUSIC values are 1/den with den = M - |a^H s|^2 (rank-1 closed form); fp32 |a^H s|^2 from
the fp32 RDS is good to ~1e-6 absolute, so the test compares den = 1/spectrum to the oracle's fp64 den within
DEN_ATOL = 2e-5 (exact zeros where den <= 1e-12, which fp32 cannot reach for noise cells)."""
import numpy as np
import pytest

import parity as P
import radar_oracle as O

pytestmark = pytest.mark.gpu
DEN_ATOL = 2e-5


def _frames(A, C, Tc, F, seed0=1000):
    out = []
    for f in range(F):
        np.random.seed(seed0 + f)
        out.append(O.synthesize_frame(O.TEST_SCENE, chirp_duration=Tc, num_chirps=C, num_antennas=A))
    return np.stack(out)


@pytest.mark.parametrize('name,A,C,Tc,method', [('cfg1', 8, 64, 25.6e-6, 'music'), ('cfg2', 8, 128, 51.2e-6, 'music'),
                                               ('cfg1_bf', 8, 64, 25.6e-6, 'beamforming'),
                                               ('a4', 4, 64, 25.6e-6, 'music'),
                                               ('a16', 16, 32, 12.8e-6, 'music'),       # MA = 16 (K = 32) spectrum scan
                                               ('a16_bf', 16, 32, 12.8e-6, 'beamforming')])
def test_batched_spectrum_vs_oracle(ctx, name, A, C, Tc, method):
    import rsl
    F = 2
    frames = _frames(A, C, Tc, F)
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc, spectrum=True,
                          cell_frac=0.7 if A <= 8 else 1.0, method=method)  # 16-antenna unions are denser
    ch = rsl.RadarChain(cfg, F, ctx)
    ch.run(ctx.to_dev(frames.astype(np.complex64)), esprit=False, velocity=False)
    res = ch.results()
    nc = len(res['c_rc'])
    from rsl.runtime import spectrum_rows
    spec = spectrum_rows(ch.spec, nc).cpu().numpy()  # [cells, G]
    grid = O.azimuth_grid()
    steer = O.steering_matrix(grid, A)
    cb = res['cell_base']
    rs = np.random.RandomState(0)
    for f in range(F):
        ref = O.range_doppler_spectrum(frames[f], chirp_duration=Tc)
        sl = np.arange(cb[f], cb[f + 1])
        pick = sl if len(sl) <= 4000 else np.sort(rs.choice(sl, 4000, replace=False))
        rc = res['c_rc'][pick]
        sigs = np.stack([O.spatial_signature(ref, r // C, r % C) for r in rc])
        got = spec[pick]
        # the grid index is a maximum of the written spectrum up to the scan's precision (tests/parity.py)
        assert P.spectrum_argmax_consistent(got.astype(np.float64), res['gidx'][pick], method)
        if method == 'music':
            want = O.music_spectrum_closed(sigs, steer)
            assert ((got > 0) == (want > 0)).all()
            dg = np.where(got > 0, 1.0 / np.where(got > 0, got, 1.0), 0.0)
            dw = np.where(want > 0, 1.0 / np.where(want > 0, want, 1.0), 0.0)
            err = np.abs(dg - dw).max()
        else:
            want = O.beamforming_spectrum(sigs, steer)
            err = np.abs(got - want).max()
        print(f'{name} frame {f}: {len(pick)} cells, max |den - den_ref| = {err:.2e}')
        assert err < DEN_ATOL, (name, f, err)


def test_spectrum_layouts_agree(ctx):
    """Grid-major (RSL_DOA_SPEC_GMAJOR), cell-blocked (RSL_DOA_SPEC_BLOCKED) and cell-major spectra of the same cells
    are bit-identical."""
    import rsl
    import torch
    frames = _frames(8, 64, 25.6e-6, 1)
    cfg = rsl.ChainConfig(num_antennas=8, num_chirps=64, chirp_duration=25.6e-6)
    ch = rsl.RadarChain(cfg, 1, ctx)
    ch.run(ctx.to_dev(frames.astype(np.complex64)))
    nc = ch.totals()[1]
    L = ch.lists
    _, _, s_cm = ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=nc, want_spec=True, fast=False)
    _, _, s_gm = ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=nc, want_spec=True,
                         spec_gmajor=True, fast=False)
    _, _, s_bl = ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=nc, want_spec=True,
                         spec_blocked=True, fast=False)
    from rsl.runtime import spectrum_rows
    torch.cuda.synchronize()
    assert torch.equal(s_cm, s_gm.t())
    assert torch.equal(s_cm, spectrum_rows(s_bl, nc))
    # grid-major with a leading dimension of 1, 2 or 3 cells: the layout is a flag of its own, so ld = 1 is not taken
    # for the cell-blocked layout (which would write G * 32 floats into a [G][1] buffer)
    for n in (1, 2, 3):
        _, _, s1 = ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=n, want_spec=True,
                           spec_gmajor=True, fast=False)
        torch.cuda.synchronize()
        assert tuple(s1.shape) == (len(ch.grid), n)
        assert torch.equal(s_cm[:n], s1.t())


@pytest.mark.parametrize('method', ['music', 'beamforming'])
def test_toeplitz_spectrum_matches_f32_scan(ctx, method):
    """The Toeplitz spectrum (f16 hi/lo products) against the f32-MFMA scan's spectrum of the same cells: MUSIC den
    within DEN_ATOL, beamforming |a^H s|^2 within 2e-5, same argmax wherever the f32 scan's top-2 gap is clear, and
    the argmax is a maximum of the written spectrum."""
    import rsl
    import torch
    from rsl.runtime import spectrum_rows
    frames = _frames(8, 128, 51.2e-6, 2)
    cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6, method=method)
    ch = rsl.RadarChain(cfg, 2, ctx)
    ch.run(ctx.to_dev(frames.astype(np.complex64)), esprit=False, velocity=False)
    nc = ch.totals()[1]
    L = ch.lists
    i_t, _, s_t = ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=nc, want_spec=True,
                          spec_blocked=True)
    i_f, _, s_f = ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=nc, want_spec=True,
                          spec_blocked=True, fast=False)
    torch.cuda.synchronize()
    st = spectrum_rows(s_t, nc).cpu().numpy().astype(np.float64)
    sf = spectrum_rows(s_f, nc).cpu().numpy().astype(np.float64)
    it, jf = i_t[:nc].cpu().numpy(), i_f[:nc].cpu().numpy()
    n = np.arange(nc)
    assert P.spectrum_argmax_consistent(st, it, method)
    if method == 'music':
        assert ((st > 0) == (sf > 0)).all()
        dt = np.where(st > 0, 1.0 / np.where(st > 0, st, 1.0), 0.0)
        df = np.where(sf > 0, 1.0 / np.where(sf > 0, sf, 1.0), 0.0)
        err = np.abs(dt - df).max()
        key = 8.0 - df
    else:
        err = np.abs(st - sf).max()
        key = sf
    srt = np.sort(key, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 1e-6 * np.abs(srt[:, -1])  # the parity rule's 1e-6 (tests/parity.py)
    print(f'{method}: {nc} cells, max diff {err:.2e}, argmax differs at {(it != jf).sum()} cells '
          f'({(it != jf)[clear].sum()} with a clear gap)')
    assert err < DEN_ATOL
    assert (it == jf)[clear].all()


def test_spectrum_contiguous_allocation(ctx):
    """RadarChain(spec_out='contiguous') (the bench's configs[1] buffer): the spectrum lands in its own
    physically contiguous allocation (Context.empty_contiguous) and is bit-identical to the default allocation's; a
    spec_out tensor of the wrong shape is refused; the block is freed with the chain (allocated again at once)."""
    import rsl
    import torch
    A, C, Tc = 8, 64, 25.6e-6
    frames = _frames(A, C, Tc, 2)
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc, spectrum=True, cell_frac=0.7)
    cube = ctx.to_dev(frames.astype(np.complex64))
    ref = rsl.RadarChain(cfg, 2, ctx)
    ref.run(cube, esprit=False, velocity=False)
    for _ in range(2):
        ch = rsl.RadarChain(cfg, 2, ctx, spec_out='contiguous')
        assert ch.spec_contiguous and tuple(ch.spec.shape) == ch.spectrum_shape()
        ch.run(cube, esprit=False, velocity=False)
        torch.cuda.synchronize()
        nc = ch.totals()[1]
        assert nc == ref.totals()[1]
        from rsl.runtime import spectrum_rows
        assert torch.equal(spectrum_rows(ch.spec, nc).view(torch.int32), spectrum_rows(ref.spec, nc).view(torch.int32))
        del ch
    with pytest.raises(ValueError):
        rsl.RadarChain(cfg, 2, ctx, spec_out=torch.empty((3, 361, 32), device='cuda'))

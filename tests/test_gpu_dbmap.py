"""The fused RDS + detection launch's optional dB map (rsl_rds_detect db_map: the detection map of dechirp.py:243,
10 log10(|X|^2 + 1e-12)) on all three K2 bodies: the c64 LDS kernel (cfg1 shape) and the packed register-form kernels
(cfg2: k_doppler_detect_r128, configs[4] shape: k_doppler_detect_r256).  Requesting the map must not change the RDS,
the masks or the row counts, and the map must equal the expression on the launch's own RDS."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = {  # name: (F, A, C, T_c)
    'cfg1': (3, 8, 64, 25.6e-6),
    'cfg2': (3, 8, 128, 51.2e-6),
    'cfg5': (1, 16, 256, 102.4e-6),
}


@pytest.mark.parametrize('name', list(SHAPES))
def test_db_map(ctx, name):
    import rsl
    F, A, C, Tc = SHAPES[name]
    ch = rsl.RadarChain(rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc), F, ctx)
    S = ch.rds.shape[2]
    g = torch.Generator(device='cuda').manual_seed(5)
    cube = torch.complex(torch.randn(F, A, C, S, device='cuda', generator=g),
                         torch.randn(F, A, C, S, device='cuda', generator=g)) * 0.1

    def run(db):
        ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                       row_count=ch.row_count, peak_pow=ch.peak_pow, db_map=db, dc_removal=True)
        torch.cuda.synchronize()
        return ch.rds.clone(), ch.mask.clone(), ch.row_count.clone()

    ref = run(None)
    db = torch.full((F, A, S, C), float('nan'), dtype=torch.float32, device='cuda')
    got = run(db)
    bits = lambda t: t.view(torch.float32).view(torch.int32) if t.is_complex() else t
    for a, b, w in zip(ref, got, ('rds', 'mask', 'row_count')):
        assert torch.equal(bits(a), bits(b)), f'{name}: {w} changed with the dB map'
    assert int(ref[2].sum()) > 0
    want = 10.0 * torch.log10(got[0].abs().double() ** 2 + 1e-12)
    assert not torch.isnan(db).any(), f'{name}: dB map not fully written'
    err = (db.double() - want).abs().max().item()
    assert err < 2e-4, f'{name}: dB map off by {err} dB'

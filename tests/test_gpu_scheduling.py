"""K1 tile scheduling: the per-XCD dequeue (default, rsl_fft.hip `k_range_fft_p<..., DYN = true>`) against the static
persistent walk (RSL_RF_DYN=0), on the same device cubes. Scheduling must not change a single bit of the range
spectra, RDS, peak masks or peak powers: grids below 8 workgroups (static fallback), tile counts that do not divide
over the 8 XCDs, and batches far larger than the resident grid; then 20 more launches on the default path, so every
queue slot (8, round-robin) has been reused after its self-reset.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = {  # name: (F, A, C, T_c)  -> K1 tiles = F * A * ceil(C / 8) at S = 512
    'below8': (1, 1, 16, 51.2e-6),       # 2 tiles: grid < 8, static walk
    'ragged': (3, 3, 24, 51.2e-6),       # 27 tiles over 8 XCDs (3 or 4 each)
    'cfg1': (5, 8, 64, 25.6e-6),         # S = 256
    'cfg2': (40, 8, 128, 51.2e-6),       # 5120 tiles: 6.7 per resident workgroup
    'cfg2_pack': (40, 8, 128, 51.2e-6),  # the same with packed `work` rows (RSL_WORK_PACK=1)
}


def _run(ctx, ch, cube, dyn, pack=False):
    old = os.environ.get('RSL_RF_DYN')
    os.environ['RSL_RF_DYN'] = dyn
    old_pack = os.environ.get('RSL_WORK_PACK')
    os.environ['RSL_WORK_PACK'] = '1' if pack else '0'
    try:
        ch.work.zero_()
        ch.rds.zero_()
        ch.peak_pow.zero_()
        ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                       row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop('RSL_RF_DYN', None)
        else:
            os.environ['RSL_RF_DYN'] = old
        if old_pack is None:
            os.environ.pop('RSL_WORK_PACK', None)
        else:
            os.environ['RSL_WORK_PACK'] = old_pack
    return [t.clone() for t in (ch.work, ch.rds, ch.mask, ch.row_count, ch.peak_pow)]


def _bits(t):
    # bitwise: packed `work` rows (24-bit mantissas) reinterpreted as c64 include NaN patterns
    if t.is_complex():
        t = t.view(torch.float32)
    return t.view(torch.int32) if t.dtype == torch.float32 else t


@pytest.mark.parametrize('name', list(SHAPES))
def test_dequeue_matches_static_walk(ctx, name):
    import rsl
    F, A, C, Tc = SHAPES[name]
    ch = rsl.RadarChain(rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc), F, ctx)
    S = ch.rds.shape[2]
    g = torch.Generator(device='cuda').manual_seed(7)
    cube = torch.complex(torch.randn(F, A, C, S, device='cuda', generator=g),
                         torch.randn(F, A, C, S, device='cuda', generator=g)) * 0.1
    pack = name.endswith('_pack')
    ref = _run(ctx, ch, cube, '0', pack)
    assert ref[1].abs().amax().item() > 0
    for rep in range(21):
        got = _run(ctx, ch, cube, '1', pack)
        for a, b, what in zip(ref, got, ('work', 'rds', 'mask', 'row_count', 'peak_pow')):
            assert torch.equal(_bits(a), _bits(b)), f'{name}: {what} differs on launch {rep}'

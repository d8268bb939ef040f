"""The one-launch RDS path (k_rds_ring: range FFT and Doppler FFT + detection in one persistent launch, `work` kept
as a per-XCD ring of slabs in L2) against the two-kernel path (K1 + K2) on the same cubes: RDS, detection masks,
row counts and the tile-compact peak powers must be bit-identical (same FFT arithmetic, only the hand-off of the
range spectra differs), at batches that reuse every ring slot many times and at ring sizes / leads that force waits
on both hand-offs.  The oracle parity of the path itself is test_gpu_chain.py's cfg2_ring case.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(ctx, cube, F, env):
    import rsl
    import torch
    cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
    ch = rsl.RadarChain(cfg, F, ctx)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        grp = ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                             row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)
        torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    rc = ch.row_count.cpu().numpy()
    pk = ch.peak_pow.cpu().numpy()
    # tile-compact peak powers: each run of `grp` rows holds its rows' peaks packed from the run's first slot
    F_, A, S, C = pk.shape
    runs = pk.reshape(F_, A, S // grp, grp * C)
    cnt = rc.reshape(F_, A, S // grp, grp).sum(-1)
    valid = np.arange(grp * C)[None, None, None, :] < cnt[..., None]
    out = dict(rds=ch.rds.cpu().numpy(), mask=ch.mask.cpu().numpy(), rc=rc, pk=np.where(valid, runs, 0), grp=grp)
    del ch
    return out


@pytest.fixture(scope='module')
def cubes(ctx):
    import rsl  # noqa: F401
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import make_cubes
    return {F: make_cubes(ctx, 1, F, 8, 128, 51.2e-6, 7)[0] for F in (3, 48)}


@pytest.mark.parametrize('F,env', [
    (3, {}),                                            # 24 slabs < 8 R: own slab addresses
    (48, {}),                                           # 384 slabs: every ring slot reused ~12 times
    (48, {'RSL_RING_R': '2', 'RSL_RING_L': '1'}),       # two slots per XCD: range tiles wait for their slot
    (48, {'RSL_RING_R': '3', 'RSL_RING_L': '2'}),
    (48, {'RSL_RING_R': '8', 'RSL_RING_L': '7'}),
    (48, {'RSL_RING_BPC': '1'}),                        # one workgroup per CU
])
def test_ring_matches_two_kernel_path(ctx, cubes, F, env):
    # the two-kernel reference with c64 `work` rows (the ring hands over unpacked range spectra)
    ref = _run(ctx, cubes[F], F, {'RSL_RING': '0', 'RSL_WORK_PACK': '0'})
    got = _run(ctx, cubes[F], F, dict(env, RSL_RING='1'))
    assert ctx.lib.rsl_ring_faults(ctx.h) == 0
    assert got['grp'] == ref['grp']
    for k in ('rds', 'mask', 'rc', 'pk'):
        assert np.array_equal(got[k].view(np.uint8), ref[k].view(np.uint8)), k
    assert ctx.lib.rsl_ring_faults(ctx.h) == 0

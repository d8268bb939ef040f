"""The product library is environment-independent: every run-time switch that rounds 1-2 read
(variant selectors, cache policies, ablations) is set to a non-default value, and the whole chain must give
bit-identical outputs to a run with none of them set.  The switches were removed from librsl.so; the ablations
survive only in the development build (librsl_dev.so), which the runtime never loads by default."""
import os

import numpy as np
import pytest
import torch

import radar_oracle as O

pytestmark = pytest.mark.gpu

OLD_SWITCHES = {
    'RSL_RING': '1', 'RSL_RING_R': '2', 'RSL_RING_L': '1', 'RSL_FUSED': '1', 'RSL_WORK_PACK': '1', 'RSL_RF_DYN': '0',
    'RSL_RF_CB': '16', 'RSL_RF_BPC': '1', 'RSL_RF_PD': '2', 'RSL_RF_NP': '1', 'RSL_RF_CP': '0', 'RSL_RF_DBG': '1',
    'RSL_DD_CP': '0', 'RSL_DD_KB': '32', 'RSL_DD_XCD': '0', 'RSL_DD_LDS': '65536', 'RSL_DD_PAD': '0',
    'RSL_DD_PERSIST': '1', 'RSL_DD_DBG': '2', 'RSL_DOA_SKEW': '0', 'RSL_DOA_PPW': '0', 'RSL_DOA_FULL': '1',
    'RSL_DOA_BPC': '1', 'RSL_DOA_UNROLL': '0', 'RSL_DOA_DBG': '1', 'RSL_EMIT_CELLS': '0', 'RSL_EMIT_WPE': '0',
    'RSL_OFF_NT': '1024', 'RSL_WORK_C64': '1', 'RSL_R128_KB': '32', 'RSL_R128_TPW': '2',
}


def _run(ctx, cube, cfg, F):
    import rsl
    ch = rsl.RadarChain(cfg, F, ctx)
    ch.run(cube)
    res = ch.results()
    torch.cuda.synchronize()
    return res, ch.rds.cpu().numpy()


def test_switches_change_nothing(ctx):
    import rsl
    A, C, Tc, F = 8, 128, 51.2e-6, 2
    frames = []
    for f in range(F):
        np.random.seed(1000 + f)
        frames.append(O.synthesize_frame(O.TEST_SCENE, chirp_duration=Tc, num_chirps=C, num_antennas=A))
    cube = ctx.to_dev(np.stack(frames).astype(np.complex64))
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc)
    saved = {k: os.environ.pop(k) for k in list(os.environ) if k.startswith('RSL_') and k != 'RSL_LIBRARY'}
    try:
        ref, ref_rds = _run(ctx, cube, cfg, F)
        os.environ.update(OLD_SWITCHES)
        got, got_rds = _run(ctx, cube, cfg, F)
    finally:
        for k in OLD_SWITCHES:
            os.environ.pop(k, None)
        os.environ.update(saved)
    assert np.array_equal(ref_rds.view(np.uint32), got_rds.view(np.uint32))
    for k in ('entry_base', 'cell_base', 'e_ant', 'e_rbin', 'e_dbin', 'e_cell', 'e_pdb', 'c_rc', 'c_amask', 'gidx',
              'esprit', 'phase', 'velocity'):
        a, b = np.asarray(ref[k]), np.asarray(got[k])
        assert a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8)), k

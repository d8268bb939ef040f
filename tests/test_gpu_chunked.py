"""ChainConfig.front_chunk: RDS + detection in frame chunks through one chunk-sized `work` buffer (K1 -> K2 of each
chunk back to back, so that the packed range spectra of a chunk can be read from the Infinity Cache) must give the
same RDS, masks, row counts, peak powers, lists, angles and velocities as one launch pair over the whole batch:
bit-identical, since the same kernels do the same arithmetic per frame (a small launch only drops the nt store hint of
the packed `work`, rsl_fft.hip launch_k1)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('A,C,TC,F,chunk', [(8, 128, 51.2e-6, 7, 3), (8, 64, 25.6e-6, 5, 2)])
def test_front_chunk_matches_one_launch(ctx, A, C, TC, F, chunk):
    import rsl
    g = torch.Generator(device='cuda').manual_seed(5)
    S = int(round(TC * 10e6))
    cube = torch.complex(torch.randn(F, A, C, S, device='cuda', generator=g),
                         torch.randn(F, A, C, S, device='cuda', generator=g)) * 0.1
    out = []
    for fc in (0, chunk):
        cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC, front_chunk=fc)
        ch = rsl.RadarChain(cfg, F, ctx)
        assert ch.chunk == (chunk if fc else F)
        ch.run(cube)
        torch.cuda.synchronize()
        out.append(dict(rds=ch.rds.clone(), mask=ch.mask.clone(), row_count=ch.row_count.clone(), res=ch.results()))
    a, b = out
    assert torch.equal(a['rds'], b['rds']) and torch.equal(a['mask'], b['mask'])
    assert torch.equal(a['row_count'], b['row_count'])
    for key, w in a['res'].items():
        assert np.array_equal(w, b['res'][key], equal_nan=True), key

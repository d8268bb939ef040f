"""The bench's pipelined chain (bench.py `step_pipelined`): two RadarChain buffers alternate, batch i's front half on
stream A overlaps batch i-1's back half on stream B, with the compaction (emit) and optionally the offsets moved to
the back stream (RSL_BENCH_EMIT_BACK 1 / 2). Every placement must give the same lists, angles, ESPRIT, phases and
velocities as one serial `run` of each batch: bit-identical, since only the stream a kernel runs on changes.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

A, C, TC, F, NB = 8, 64, 25.6e-6, 3, 4  # cfg1 frame shape, 4 batches of 3 frames


def _cubes():
    g = torch.Generator(device='cuda').manual_seed(11)
    S = int(round(TC * 10e6))
    return [torch.complex(torch.randn(F, A, C, S, device='cuda', generator=g),
                          torch.randn(F, A, C, S, device='cuda', generator=g)) * 0.1 for _ in range(NB)]


@pytest.mark.parametrize('placement', [0, 1, 2])
def test_pipelined_matches_serial(ctx, placement):
    import rsl
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
    cubes = _cubes()
    ser = rsl.RadarChain(cfg, F, ctx)
    want = []
    for cube in cubes:
        ser.run(cube)
        want.append(ser.results())
    chains = [rsl.RadarChain(cfg, F, ctx) for _ in range(2)]
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    evA = [torch.cuda.Event() for _ in range(2)]
    evB = [torch.cuda.Event() for _ in range(2)]
    used = [False, False]
    got = [None] * NB
    main = torch.cuda.current_stream()
    for i, cube in enumerate(cubes):
        k = i % 2
        ch = chains[k]
        if used[k]:  # buffer reuse: batch i-2's results are read before its buffers are overwritten
            evB[k].synchronize()
            got[i - 2] = ch.results()
        sA.wait_stream(main)
        with torch.cuda.stream(sA):
            ch.run_front(cube, emit=placement == 0, offsets=placement < 2)
            evA[k].record(sA)
        with torch.cuda.stream(sB):
            sB.wait_event(evA[k])
            ch.run_back(emit=placement > 0, offsets=placement == 2)
            evB[k].record(sB)
        used[k] = True
    torch.cuda.synchronize()
    for i in (NB - 2, NB - 1):
        got[i] = chains[i % 2].results()
    for i in range(NB):
        assert want[i]['c_rc'].size > 0
        for key, w in want[i].items():
            assert np.array_equal(w, got[i][key], equal_nan=True), f'batch {i}: {key} differs (placement {placement})'

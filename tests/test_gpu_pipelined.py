"""The bench's pipelined chain (bench.py `step_pipelined`): two RadarChain buffers alternate, batch i's front half on
stream A overlaps batch i-1's back half on stream B, with the compaction (emit) and optionally the offsets moved to
the back stream (RSL_BENCH_EMIT_BACK 1 / 2). Every placement must give the same lists, angles, ESPRIT, phases and
velocities as one serial `run` of each batch: bit-identical, since only the stream a kernel runs on changes.

Canary: the pipelined chains are guarded (RadarChain(guard=True): every device buffer has its own
allocation with 256 KiB sentinel pads on both sides), and after each batch the test checks, in pipeline order, the
range spectra (`work`, K1's output), the RDS (K2), the peak masks / row counts and then the lists, and that no
guard pad of either chain was written.  A failure names the first stage that differs, so a K1 fault, a K2 fault and
a foreign store into a buffer are told apart.
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


def _written(ch, name, t):
    """The part of a chain buffer the front half writes: packed `work` (S, C = 256, 64 / 512, 128 / 1024, 256) fills
    the first 6 of every 8 bytes' worth of the c64 buffer (tiles from the start); the rest is never written."""
    if name == 'work' and (ch.rds.shape[2], ch.rds.shape[3]) in ((256, 64), (512, 128), (1024, 256)):
        raw = t.reshape(-1).view(torch.uint8)
        return raw[:raw.numel() * 6 // 8]
    return t


def first_stage_diff(ch, w):
    """First pipeline stage whose device buffer differs from the serial run: work (K1), rds (K2), mask / row_count
    (K2 detection); None if all equal."""
    for name in ('work', 'rds', 'mask', 'row_count'):
        a, b = _written(ch, name, getattr(ch, name)), _written(ch, name, w[name])
        if not torch.equal(a, b):
            d = (a != b).nonzero()
            return f"{name} ({d.shape[0]} values differ, first {d[:4].tolist()})"
    return None


def run_pipelined(ctx, cfg, cubes, placement, want, guard=True):
    """The bench's two-stream schedule over `cubes`; returns a list of error strings (empty: bit-identical)."""
    import rsl
    chains = [rsl.RadarChain(cfg, F, ctx, guard=guard) for _ in range(2)]
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    evA = [torch.cuda.Event() for _ in range(2)]
    evB = [torch.cuda.Event() for _ in range(2)]
    used = [False, False]
    errs = []
    main = torch.cuda.current_stream()

    def check(i, ch):
        st = first_stage_diff(ch, want[i])
        if st:
            errs.append(f'batch {i}: first differing stage {st}')
        for k, c in enumerate(chains):
            bad = c.guard_violations()
            if bad:
                errs.append(f'batch {i}: guard pads of chain {k} written (buffer index, bytes): {bad}')
        res = ch.results()
        for key, w in want[i]['res'].items():
            if not np.array_equal(w, res[key], equal_nan=True):
                errs.append(f'batch {i}: {key} differs')
                break

    for i, cube in enumerate(cubes):
        k = i % 2
        ch = chains[k]
        if used[k]:  # buffer reuse: batch i-2's results are read before its buffers are overwritten
            evB[k].synchronize()
            check(i - 2, ch)
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
        check(i, chains[i % 2])
    return errs


def serial_reference(ctx, cfg, cubes):
    import rsl
    ser = rsl.RadarChain(cfg, F, ctx)
    want = []
    for cube in cubes:
        ser.run(cube)
        torch.cuda.synchronize()
        want.append(dict(work=ser.work.clone(), rds=ser.rds.clone(), mask=ser.mask.clone(),
                         row_count=ser.row_count.clone(), res=ser.results()))
        assert want[-1]['res']['c_rc'].size > 0
    return want


@pytest.fixture(scope='module')
def serial(ctx):
    import rsl
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
    cubes = _cubes()
    return cfg, cubes, serial_reference(ctx, cfg, cubes)


@pytest.mark.parametrize('placement', [0, 1, 2])
def test_pipelined_matches_serial(ctx, serial, placement):
    cfg, cubes, want = serial
    errs = run_pipelined(ctx, cfg, cubes, placement, want)
    assert not errs, f'placement {placement}: ' + '; '.join(errs)


def test_guard_canary_detects_foreign_store(ctx):
    """The canary itself: a store one element past a guarded buffer is reported."""
    import rsl
    cfg = rsl.ChainConfig(num_antennas=2, num_chirps=16, chirp_duration=3.2e-6)
    ch = rsl.RadarChain(cfg, 1, ctx, guard=True)
    assert ch.guard_violations() == []
    r = ch.rds.view(-1)
    r.as_strided((1,), (1,), r.storage_offset() + r.numel()).fill_(1.0 + 1.0j)  # the 8 bytes right after the RDS
    bad = ch.guard_violations()
    assert len(bad) == 1 and bad[0][1] > 0

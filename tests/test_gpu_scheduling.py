"""K1 tile scheduling (rsl_fft.hip `k_range_fft_p`): the per-XCD dequeue of grids with >= 8 workgroups and the static
walk of smaller grids must not change a single bit of the range spectra, RDS, peak masks or peak powers.

Each case runs the same device cubes as one batch and as one launch per frame (a different grid, a different tile ->
workgroup assignment and different dequeue heads), then 20 more batch launches, so the stream's queue slot has been
reused after its self-reset: grids below 8 workgroups (the static walk), tile counts that do not divide over
the 8 XCDs, and batches far larger than the resident grid.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = {  # name: (F, A, C, T_c)  -> K1 tiles = F * A * ceil(C / 8) at S = 512
    'below8': (3, 1, 16, 51.2e-6),       # 2 tiles per frame: the per-frame grids are below 8 (static walk)
    'ragged': (3, 3, 24, 51.2e-6),       # 27 tiles over 8 XCDs (3 or 4 each); 9 per frame
    'cfg1': (5, 8, 64, 25.6e-6),         # S = 256, packed: k_range_fft_r256, 8 class tiles per (frame, antenna)
    'cfg2': (40, 8, 128, 51.2e-6),       # 5120 tiles: 6.7 per resident workgroup
    'cfg5': (6, 16, 256, 102.4e-6),      # S = 1024, packed: k_range_fft_r1024, 32 class tiles per (frame, antenna)
}


def _run(ctx, ch, cube, frames=None):
    """K1 + K2/K3 over cube[frames] (all frames when None) into the chain's buffers; returns clones of the frames'
    slices of work, rds, mask, row_count and peak_pow."""
    sl = slice(None) if frames is None else frames
    bufs = [t[sl] for t in (ch.work, ch.rds, ch.mask, ch.row_count, ch.peak_pow)]
    for t in bufs:
        t.zero_()
    ctx.rds_detect(cube[sl], ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=bufs[1], work=bufs[0], mask=bufs[2],
                   row_count=bufs[3], peak_pow=bufs[4], dc_removal=True)
    torch.cuda.synchronize()
    return [t.clone() for t in bufs]


def _bits(t):
    if t.is_complex():
        t = t.view(torch.float32)
    return t.view(torch.int32) if t.dtype == torch.float32 else t


@pytest.mark.parametrize('name', list(SHAPES))
def test_scheduling_invariance(ctx, name):
    import rsl
    F, A, C, Tc = SHAPES[name]
    ch = rsl.RadarChain(rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc), F, ctx)
    S = ch.rds.shape[2]
    g = torch.Generator(device='cuda').manual_seed(7)
    cube = torch.complex(torch.randn(F, A, C, S, device='cuda', generator=g),
                         torch.randn(F, A, C, S, device='cuda', generator=g)) * 0.1
    ref = _run(ctx, ch, cube)
    assert ref[1].abs().amax().item() > 0
    what = ('work', 'rds', 'mask', 'row_count', 'peak_pow')
    # packed `work` (S = 512, C = 128; S = 1024, C = 256; S = 256, C = 64) holds 6 B per value of tiles from the buffer
    # start, so a frame's c64-sized slice is laid out differently in a one-frame launch: compare the outputs there, the
    # whole buffer on repeated launches
    packed = (S, C) in ((512, 128), (1024, 256), (256, 64))
    for f in range(F):  # one launch per frame: other grids, other tile -> workgroup maps
        got = _run(ctx, ch, cube, slice(f, f + 1))
        for a, b, w in zip(ref, got, what):
            if w == 'work' and packed:
                continue
            assert torch.equal(_bits(a[f:f + 1]), _bits(b)), f'{name}: {w} of frame {f} differs (per-frame launch)'
    for rep in range(20):
        got = _run(ctx, ch, cube)
        for a, b, w in zip(ref, got, what):
            assert torch.equal(_bits(a), _bits(b)), f'{name}: {w} differs on launch {rep}'


def test_concurrent_streams(ctx):
    """K1 launches in flight on several streams at once: each stream owns its dequeue slot (rsl_fft.hip
    rf_slot), so chains of two shapes on three streams, 8 launches each, all enqueued before any completes, give the
    serial results bit for bit."""
    import rsl
    shapes = [(6, 8, 128, 51.2e-6), (6, 8, 128, 51.2e-6), (2, 16, 256, 102.4e-6)]
    chains, cubes, refs = [], [], []
    g = torch.Generator(device='cuda').manual_seed(11)
    for F, A, C, Tc in shapes:
        ch = rsl.RadarChain(rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc), F, ctx)
        S = ch.rds.shape[2]
        cube = torch.complex(torch.randn(F, A, C, S, device='cuda', generator=g),
                             torch.randn(F, A, C, S, device='cuda', generator=g)) * 0.1
        chains.append(ch)
        cubes.append(cube)
        refs.append(_run(ctx, ch, cube))
    streams = [torch.cuda.Stream() for _ in shapes]
    outs = [[] for _ in shapes]
    torch.cuda.synchronize()
    for rep in range(8):
        for k, (ch, cube, st) in enumerate(zip(chains, cubes, streams)):
            with torch.cuda.stream(st):
                ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                               row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)
                outs[k].append([t.clone() for t in (ch.rds, ch.mask, ch.row_count)])
    torch.cuda.synchronize()
    for k in range(len(shapes)):
        for rep, got in enumerate(outs[k]):
            for a, b, w in zip((refs[k][1], refs[k][2], refs[k][3]), got, ('rds', 'mask', 'row_count')):
                assert torch.equal(_bits(a), _bits(b)), f'stream {k}: {w} differs on launch {rep}'


def test_many_streams(ctx):
    """More streams than round 5's first design had queue slots (64): each stream gets its own K1 dequeue queue
    (rsl_fft.hip rf_queue), so 72 streams with a launch each in flight at once give the serial results bit for bit."""
    import rsl
    F, A, C, Tc = 2, 8, 128, 51.2e-6
    g = torch.Generator(device='cuda').manual_seed(5)
    ch0 = rsl.RadarChain(rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc), F, ctx)
    S = ch0.rds.shape[2]
    cube = torch.complex(torch.randn(F, A, C, S, device='cuda', generator=g),
                         torch.randn(F, A, C, S, device='cuda', generator=g)) * 0.1
    ref = _run(ctx, ch0, cube)
    chains = [rsl.RadarChain(rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc), F, ctx)
              for _ in range(72)]
    streams = [torch.cuda.Stream() for _ in chains]
    torch.cuda.synchronize()
    for ch, st in zip(chains, streams):
        with torch.cuda.stream(st):
            ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                           row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)
    torch.cuda.synchronize()
    for k, ch in enumerate(chains):
        for a, b, w in zip((ref[1], ref[2], ref[3]), (ch.rds, ch.mask, ch.row_count), ('rds', 'mask', 'row_count')):
            assert torch.equal(_bits(a), _bits(b)), f'stream {k}: {w} differs'


@pytest.mark.parametrize('name', ['cfg1', 'cfg2', 'cfg5'])
def test_chirp_window_packed(ctx, name):
    """A chirp window (chirp0 > 0 inside a longer cube) on the packed paths: K1 reads its class rows at the window's
    offset; the outputs equal those of the window copied out as its own contiguous cube."""
    import rsl
    F, A, C, Tc = {'cfg1': (2, 8, 64, 25.6e-6), 'cfg2': (2, 8, 128, 51.2e-6), 'cfg5': (1, 16, 256, 102.4e-6)}[name]
    ch = rsl.RadarChain(rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc), F, ctx)
    S = ch.rds.shape[2]
    c0, Ct = 5, C + 9
    g = torch.Generator(device='cuda').manual_seed(3)
    big = torch.complex(torch.randn(F, A, Ct, S, device='cuda', generator=g),
                        torch.randn(F, A, Ct, S, device='cuda', generator=g)) * 0.1
    ref = _run(ctx, ch, big[:, :, c0:c0 + C].contiguous())
    bufs = [t.zero_() for t in (ch.work, ch.rds, ch.mask, ch.row_count, ch.peak_pow)]
    ctx.rds_detect(big, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                   row_count=ch.row_count, peak_pow=ch.peak_pow, chirp0=c0, num_chirps=C, dc_removal=True)
    torch.cuda.synchronize()
    for a, b, w in zip(ref, bufs, ('work', 'rds', 'mask', 'row_count', 'peak_pow')):
        assert torch.equal(_bits(a), _bits(b)), f'{name}: {w} differs for the chirp window'


def test_two_handles_share_no_queue(ctx):
    """K1's tile queues belong to the handle (rsl_context::rfq) and are keyed by stream inside it.
    Two handles on device 0, both launching on the null stream (handle 0, what torch reports for a default stream,
    the key every device's default stream shared in round 5's process-global map) and on one extra stream each, all
    launches enqueued before any completes, give the serial results bit for bit; a handle destroyed and re-created
    (its queues freed, new ones allocated at the same stream keys) still does."""
    import rsl
    F, A, C, Tc = 6, 8, 128, 51.2e-6
    g = torch.Generator(device='cuda').manual_seed(17)
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc)
    ch0 = rsl.RadarChain(cfg, F, ctx)
    S = ch0.rds.shape[2]
    cube = torch.complex(torch.randn(F, A, C, S, device='cuda', generator=g),
                         torch.randn(F, A, C, S, device='cuda', generator=g)) * 0.1
    ref = _run(ctx, ch0, cube)
    for life in range(2):
        hs = [rsl.Context(0), rsl.Context(0)]
        null = torch.cuda.default_stream()  # cuda_stream == 0: the null stream
        extra = [torch.cuda.Stream(), torch.cuda.Stream()]
        jobs = [(h, st, rsl.RadarChain(cfg, F, h)) for h in hs for st in (null, extra[hs.index(h)])]
        torch.cuda.synchronize()
        for rep in range(4):
            for h, st, ch in jobs:
                with torch.cuda.stream(st):
                    h.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                                 row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)
        torch.cuda.synchronize()
        for k, (h, st, ch) in enumerate(jobs):
            for a, b, w in zip((ref[1], ref[2], ref[3]), (ch.rds, ch.mask, ch.row_count), ('rds', 'mask', 'row_count')):
                assert torch.equal(_bits(a), _bits(b)), f'life {life}, job {k}: {w} differs'
        del jobs
        for h in hs:
            h.lib.rsl_destroy(h.h)
            h.h = None


def test_k1_graph_capture(ctx):
    """rsl.h's graph-capture rule: a handle's first K1 launch on a stream allocates that stream's tile queue, which a
    capture forbids, so inside a capture it fails loudly (RuntimeError naming the capture) instead of invalidating the
    capture; after one uncaptured launch on the stream, a captured K1 + K2 replays with the serial results bit for
    bit."""
    import rsl
    F, A, C, Tc = 2, 8, 128, 51.2e-6
    h = rsl.Context(0)  # a fresh handle: no queues yet
    ch = rsl.RadarChain(rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc), F, h)
    S = ch.rds.shape[2]
    g = torch.Generator(device='cuda').manual_seed(23)
    cube = torch.complex(torch.randn(F, A, C, S, device='cuda', generator=g),
                         torch.randn(F, A, C, S, device='cuda', generator=g)) * 0.1
    ref = _run(h, ch, cube)  # default stream: the handle's twiddle tables and that stream's queue

    def launch():
        h.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                     row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)
    st = torch.cuda.Stream()
    with pytest.raises(RuntimeError, match='captur'):
        with torch.cuda.graph(torch.cuda.CUDAGraph(), stream=st):
            launch()
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        launch()  # uncaptured: the queue of st
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=st):
        launch()
    for t in (ch.work, ch.rds, ch.mask, ch.row_count, ch.peak_pow):
        t.zero_()
    torch.cuda.synchronize()
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    for a, b, w in zip(ref, (ch.work, ch.rds, ch.mask, ch.row_count, ch.peak_pow),
                       ('work', 'rds', 'mask', 'row_count', 'peak_pow')):
        assert torch.equal(_bits(a), _bits(b)), f'{w} differs after graph replay'
    h.lib.rsl_destroy(h.h)
    h.h = None

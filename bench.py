#!/usr/bin/env python3
"""Throughput benchmark: radar frames/s end-to-end on 8ch x 128chirp x 512 cubes (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W --frames-per-step F]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One step = one pass of the full per-frame chain (configs[2]: RDS + peak detection + MUSIC DoA argmax +
ESPRIT + least-squares velocity + trajectory integration) over a batch of F synthetic frames already
resident in HBM.  Frames shard across ranks (one process per GPU, weak scaling, no data-path collective);
the only exchange is the trajectory reduction of the north star: each rank scans its block's poses on the
device, the ranks all-gather 16-double block summaries over RCCL/xGMI and the per-frame poses are gathered to rank 0,
which smooths them across block edges.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'radar-slam_amd'))

METRIC = "radar frames/sec end-to-end, 8ch×128chirp×512 cube; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense f16/bf16 MFMA (no 2:1 sparsity)
DIST = False  # a torch.distributed process group is up (set in main)
PROFILE = os.path.join(ROOT, 'profiles', 'r6p_pmc.json')  # rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh)


PROFILE_CONFIG = 'cfg2'  # the workload the committed profile was collected on
CFG5_PROFILE = os.path.join(ROOT, 'profiles', 'r6p_cfg5_pmc.json')  # the configs[4] frame shape (tools/profile_cfg5.sh)
STANDALONE_RUNS = 6  # unpipelined chain runs after the timed region (kernel_ms_standalone, fft_stage_standalone)
TRAFFIC_SOURCE = ('PMC FETCH_SIZE x 2 + WRITE_SIZE per launch from ' + os.path.relpath(PROFILE, ROOT) +
                  ' (tools/profile.sh, collected on the same kernels), scaled to this launch\'s frames')


def pmc_traffic(kernel_prefix, frames_per_launch, config='cfg2'):
    """HBM bytes per launch of a kernel from the committed PMC profile (FETCH_SIZE x 2 + WRITE_SIZE, per
    MI355X_MICROARCH.md), scaled to this launch's frame count; None when no profile is present, the profile was
    collected on another workload or holds no kernel of that name (a kernel renamed or replaced since: the profile is
    stale for it, and its bytes are not reported)."""
    path = {PROFILE_CONFIG: PROFILE, 'cfg5': CFG5_PROFILE}.get(config)
    if path is None:
        return None
    try:
        prof = json.load(open(path))
    except (OSError, ValueError):
        return None
    for name, e in prof.get('kernels', {}).items():
        if name.startswith('rsl::' + kernel_prefix) and 'hbm_bytes' in e:
            return e['hbm_bytes'] * frames_per_launch / prof.get('frames_per_launch', 1000)
    return None
SCENE = [  # tests/test_synth_raw.py:165-190 (reference): range m, azimuth rad, rcs dBsm, radial velocity m/s
    dict(range_sc=20.0, azimuth_sc=0.0, rcs=-10.0, vr=0.0),
    dict(range_sc=40.0, azimuth_sc=math.radians(45.0), rcs=-8.0, vr=5.0),
    dict(range_sc=60.0, azimuth_sc=math.radians(-30.0), rcs=-12.0, vr=-3.0)]


def make_cubes(ctx, nb, F, A, C, Tc, rank):
    """nb batches of F synthetic frames from the device generator (rsl_synth_*: the reference simulator's scene
    model, simulate_raw.py:102-221, plus Philox complex Gaussian noise of power 0.01); frame blocks differ by rank."""
    import rsl
    gen = rsl.SyntheticCubes(ctx, SCENE, chirp_duration=Tc, num_chirps=C, num_antennas=A, noise_power=0.01)
    return [gen.generate(F, seed=1234, frame0=(rank * nb + i) * F) for i in range(nb)]


def _cpu_frame(args):
    """Work item of cpu_baseline's process pool, on one host core: one whole cfg2 frame (seed ``seed``) through the
    oracle, each stage timed on this core (perf_counter; the frame's synthesis is the input, not timed).
    mode 'loop' = the loop-faithful restatement: per-chirp RDS (dechirp.py:196-211), peak dicts (dechirp.py:215-278),
    then per-peak eigh MUSIC over the 361-point grid (angle_estimation.py:109-176) + SVD ESPRIT (:178-225) for the
    frame's first ``kmax`` peaks (the bounded sample; every peak when kmax <= 0); mode 'vector' = the vectorised
    restatement (fft2, closed-form MUSIC / ESPRIT over all peaks).  Returns (azimuths rad, phases of the processed
    peaks, N_p, {stage: seconds}, peaks processed)."""
    seed, mode, kmax = args
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import radar_oracle as O
    np.random.seed(1000 + seed)
    Tc = 51.2e-6
    frame = O.synthesize_frame(O.TEST_SCENE, chirp_duration=Tc, num_chirps=128, num_antennas=8)
    grid = O.azimuth_grid()
    t = {}
    t0 = time.perf_counter()
    if mode == 'loop':
        rds = O.range_doppler_spectrum_loop(frame, chirp_duration=Tc)
        t1 = time.perf_counter()
        peaks = O.extract_peaks(rds)['peaks']
        t2 = time.perf_counter()
        mine = peaks if kmax <= 0 else peaks[:kmax]
        az, sig = np.empty(len(mine)), np.empty((len(mine), 8), complex)
        for n, p in enumerate(mine):
            s = O.spatial_signature(rds, p['range_bin'], p['doppler_bin'])
            az[n] = grid[np.argmax(O.music_spectrum_eigh(s, grid))]
            O.esprit_svd(s)
            sig[n] = s
        t3 = time.perf_counter()
        Np = len(peaks)
    else:
        rds = O.range_doppler_spectrum(frame, chirp_duration=Tc)
        t1 = time.perf_counter()
        a, i, j, _ = O.peak_arrays(rds)
        t2 = time.perf_counter()
        sig = rds[:, i, j].T
        sig = sig / np.sqrt(np.sum(np.abs(sig) ** 2, axis=1, keepdims=True))
        steer = O.steering_matrix(grid, 8)
        az = np.concatenate([grid[np.argmax(O.music_spectrum_closed(sig[k:k + 8192], steer), axis=1)]
                             for k in range(0, len(sig), 8192)])
        O.esprit_closed(sig)
        t3 = time.perf_counter()
        Np = len(a)
    t.update(rds=t1 - t0, peaks=t2 - t1, doa=t3 - t2)
    return np.radians(az), O.observed_phase(sig), Np, t, len(sig)


def _cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def host_cores():
    """(cores this process may use, CPUs in its affinity mask, cgroup CPU quota in cores or None).  A GPU box grants a
    share of the host (a cgroup cpu.max quota) while the affinity mask and os.cpu_count() show the whole machine."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    for path in ('/sys/fs/cgroup/cpu.max', '/sys/fs/cgroup/cpu/cpu.cfs_quota_us'):
        try:
            txt = open(path).read().split()
        except OSError:
            continue
        if path.endswith('cpu.max') and txt and txt[0] != 'max':
            quota = int(txt[0]) / int(txt[1])
        elif path.endswith('quota_us') and txt and int(txt[0]) > 0:
            quota = int(txt[0]) / int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
        break
    use = aff if quota is None else max(1, min(aff, int(quota)))
    return use, aff, quota


def cpu_baseline(procs=0, kmax=3000, vec_frames=2, ridge=0.01):
    """Oracle ('port') chain on cfg2 frames, SURVEY §8(d)(ii), on all the host cores this process may use (``procs``
    = 0; host_cores) as single-threaded worker processes (BLAS threads = 1), one whole frame per worker at least.

    Loop-faithful line: P frames, one per worker, each through the per-chirp RDS, the peak dicts and per-peak eigh
    MUSIC + SVD ESPRIT for its first ``kmax`` peaks (a frame has ~49 k peaks at ~2.6 ms each, 130 core-s: the bounded
    sample keeps the run near 10 s), then the LS velocity of each frame in the parent.  Every stage is timed on its
    core while all P workers run together; a frame's seconds = RDS + peaks + (DoA per peak) x N_p + velocity per peak
    x N_p, and value = P / that (P frames in flight on P cores).  Vectorised line: ``vec_frames`` whole frames per
    worker, every peak, timed the same way (no extrapolation)."""
    import multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import radar_oracle as O
    for v in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
        os.environ[v] = '1'  # inherited by the spawned workers before they import numpy
    use, aff, quota = host_cores()
    P = use if procs <= 0 else max(1, min(procs, aff))
    lam = 3e8 / 77e9
    ctx = mp.get_context('spawn')

    def stage_means(res):
        tv0 = time.perf_counter()
        for r in res:
            O.velocity_ls(r[0], r[1], lambda_c=lam, ridge=ridge)
        tvel = (time.perf_counter() - tv0) / max(1, sum(r[4] for r in res))  # LS seconds per processed peak
        m = {k: float(np.mean([r[3][k] for r in res])) for k in ('rds', 'peaks', 'doa')}
        m['doa_per_peak'] = float(np.mean([r[3]['doa'] / max(r[4], 1) for r in res]))
        m['velocity_per_peak'] = tvel
        m['peaks_per_frame'] = float(np.mean([r[2] for r in res]))
        return m

    with ctx.Pool(P) as pool:
        pool.map(_cpu_frame, [(0, 'vector', 0)] * P, chunksize=1)  # worker start-up and imports outside the timing
        t0 = time.perf_counter()
        res = pool.map(_cpu_frame, [(f, 'loop', kmax) for f in range(P)], chunksize=1)
        wall_loop = time.perf_counter() - t0
        t0 = time.perf_counter()
        vres = pool.map(_cpu_frame, [(f, 'vector', 0) for f in range(P * vec_frames)], chunksize=1)
        wall_vec = time.perf_counter() - t0
    m = stage_means(res)
    npk = m['peaks_per_frame']
    frame_s = m['rds'] + m['peaks'] + (m['doa_per_peak'] + m['velocity_per_peak']) * npk
    mv = stage_means(vres)
    vframe_s = mv['rds'] + mv['peaks'] + mv['doa'] + mv['velocity_per_peak'] * mv['peaks_per_frame']
    nproc = [r[4] for r in res]
    return dict(value=P / frame_s, unit="frames/s", cores=P, kind="port", cpu=_cpu_model(), nproc=os.cpu_count(),
                cores_available=use, affinity_cpus=aff, cgroup_cpu_quota=quota,
                seconds_per_frame_per_core={"range_doppler": m['rds'], "peak_extraction": m['peaks'],
                                            "doa_music_esprit": m['doa_per_peak'] * npk,
                                            "velocity_ls": m['velocity_per_peak'] * npk, "total": frame_s},
                sample=(f"{P} whole cfg2 frames (8x128x512), one per worker process x 1 thread, all {P} together "
                        f"({wall_loop:.1f} s wall): loop-faithful oracle, per-chirp RDS and peak dicts of every "
                        f"frame timed in full, per-peak eigh MUSIC + SVD ESPRIT and LS velocity timed on the first "
                        f"{min(nproc)}-{max(nproc)} of the frame's {npk:.0f} peaks and scaled to all of them"),
                vectorised={"value": P / vframe_s, "unit": "frames/s", "cores": P,
                            "seconds_per_frame_per_core": {"range_doppler": mv['rds'], "peak_extraction": mv['peaks'],
                                                           "doa_music_esprit": mv['doa'],
                                                           "velocity_ls": mv['velocity_per_peak'] * mv['peaks_per_frame'],
                                                           "total": vframe_s},
                            "wall_frames_per_s": P * vec_frames / wall_vec,
                            "sample": f"{P * vec_frames} whole cfg2 frames, {vec_frames} per worker, every peak: "
                                      f"vectorised oracle (fft2, closed-form MUSIC / ESPRIT, LS velocity); "
                                      f"{wall_vec:.1f} s wall"})


SPEC_PROFILE = os.path.join(ROOT, 'profiles', 'r6m_spectrum_pmc.json')  # tools/profile_spectrum.sh


def spectrum_traffic(frames):
    """HBM bytes per launch of the spectrum scan (k_doa_toep with SPEC) from the committed configs[1] PMC profile."""
    try:
        prof = json.load(open(SPEC_PROFILE))
    except (OSError, ValueError):
        return None
    for name, e in prof.get('kernels', {}).items():
        if name.startswith('rsl::k_doa_toep') and 'hbm_bytes' in e:
            return e['hbm_bytes'] * frames / prof.get('frames_per_launch', 1000)
    return None


def pcie_inclusive(ctx, dev, F=500, steps=8):
    """The metric's rate when every frame's c64 cube [A, C, S] (4 MiB at cfg2) first crosses PCIe from pinned host
    memory (SURVEY §8(d) "Timed region": reported beside `value`, never as it).  Host-to-device copies of batch i + 1
    run on a copy stream while the chain processes batch i; each batch's per-frame velocities come back to pinned host
    memory.  Also the raw pinned H2D bandwidth and the same loop with the cubes resident."""
    import torch
    import rsl
    A, C, Tc = 8, 128, 51.2e-6
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc)
    gen = rsl.SyntheticCubes(ctx, SCENE, chirp_duration=Tc, num_chirps=C, num_antennas=A, noise_power=0.01)
    host = []
    for i in range(2):  # two distinct pinned host batches, generated on the device and copied out once
        d = gen.generate(F, seed=4321, frame0=i * F)
        torch.cuda.synchronize()
        h = torch.empty(d.shape, dtype=d.dtype, pin_memory=True)
        h.copy_(d)
        host.append(h)
        del d
    dbuf = [torch.empty(host[0].shape, dtype=host[0].dtype, device=dev) for _ in range(2)]
    vel_d = [torch.empty((F, 8), dtype=torch.float64, device=dev) for _ in range(2)]
    vel_h = [torch.empty((F, 8), dtype=torch.float64, pin_memory=True) for _ in range(2)]
    chains = [rsl.RadarChain(cfg, F, ctx, vel_out=vel_d[k]) for k in range(2)]
    nbytes = host[0].numel() * host[0].element_size()
    cs, ks = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    with torch.cuda.stream(cs):
        dbuf[0].copy_(host[0], non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(cs):
        for i in range(4):
            dbuf[i % 2].copy_(host[i % 2], non_blocking=True)
    torch.cuda.synchronize()
    h2d = 4 * nbytes / (time.perf_counter() - t0)
    ev_copy = [torch.cuda.Event() for _ in range(2)]
    ev_done = [torch.cuda.Event() for _ in range(2)]
    used = [False, False]

    def step(i):
        k = i % 2
        with torch.cuda.stream(cs):
            if used[k]:
                cs.wait_event(ev_done[k])  # batch i - 2 is done with dbuf[k] and vel_d[k]
                vel_h[k].copy_(vel_d[k], non_blocking=True)
            dbuf[k].copy_(host[k], non_blocking=True)
            ev_copy[k].record(cs)
        with torch.cuda.stream(ks):
            ks.wait_event(ev_copy[k])
            chains[k].run(dbuf[k])
            ev_done[k].record(ks)
        used[k] = True

    for i in range(2):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    fps = steps * F / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    with torch.cuda.stream(ks):
        for i in range(steps):
            chains[i % 2].run(dbuf[i % 2])
    torch.cuda.synchronize()
    fps_res = steps * F / (time.perf_counter() - t0)
    return {"value": fps, "unit": "frames/s", "frames_per_batch": F, "steps": steps,
            "bytes_per_frame": nbytes // F, "h2d_pinned_GBps": h2d / 1e9,
            "pcie_bound_frames_per_s": h2d / (nbytes / F), "device_resident_same_loop_frames_per_s": fps_res,
            "what": "cfg2 chain, c64 cubes copied host -> device per batch (pinned memory, copy stream overlapped "
                    "with the previous batch's chain), velocities copied back; one compute stream"}


def cu_masked_stream(dev, ncu, side, total=256):
    """A HIP stream restricted to ncu of the device's CUs (hipExtStreamCreateWithCUMask), wrapped for torch.  The
    CUs are taken in groups of 8 consecutive mask bits spread evenly over the mask (side 0 from the low groups' end of
    each spread, side 1 from the other), so that both sides keep CUs on every XCD."""
    import ctypes
    import torch
    hip = ctypes.CDLL('libamdhip64.so')
    ng = total // 8
    take = max(1, min(ng, round(ncu / 8)))
    groups = [g for g in range(ng) if (g * take) // ng != ((g + 1) * take) // ng]
    if side:
        groups = [ng - 1 - g for g in groups]
    words = [0] * (total // 32)
    for g in groups:
        for b in range(8 * g, 8 * g + 8):
            words[b // 32] |= 1 << (b % 32)
    arr = (ctypes.c_uint32 * len(words))(*words)
    st = ctypes.c_void_p()
    torch.cuda.set_device(dev)
    if hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(len(words)), arr) != 0:
        raise RuntimeError('hipExtStreamCreateWithCUMask failed')
    return torch.cuda.ExternalStream(st.value, device=dev)


def _sync_max(elapsed, dev):
    """The max over ranks of a host-timed interval (barrier + synchronize on both sides are the caller's)."""
    if not DIST:
        return elapsed
    import torch
    import torch.distributed as dist
    tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


SPEC_BUFFERS = 3  # configs[1]: spectrum output buffers the steps rotate through (placement-dependent rate)


def measure_spectrum(ctx, dev, F, steps, warmup, rank, world, timing=True, collective=True, nbuf=SPEC_BUFFERS):
    """configs[1]: 8ch x 128chirp x 512 cube, F frames per step, range-Doppler FFT + peaks + the MUSIC spectrum of every
    unique cell (f32, cell-blocked [cells / 32, 361, 32]; the reference keeps spectrum f64[G] per target,
    angle_estimation.py:299).  One chain, no pipelining; the spectrum store dominates (51 MB per frame).  Step i writes
    its spectrum to output buffer i mod nbuf (nbuf separate 57 GB allocations, all held): the store rate depends on
    where the driver places a buffer physically (DRAM write-credit stalls), so the line averages over
    nbuf placements instead of depending on one.  Returns a dict: frames/s, per-step time, the spectrum scan's HBM
    roofline and the FFT stage's, and the scan's ms per output buffer."""
    import torch
    import torch.distributed as dist
    import rsl
    A, C, S, Tc = 8, 128, 512, 51.2e-6
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc, spectrum=True, cell_frac=0.6)
    ch = rsl.RadarChain(cfg, F, ctx)
    specs = [ch.spec] + [torch.empty_like(ch.spec) for _ in range(max(1, nbuf) - 1)]
    cubes = make_cubes(ctx, 2, F, A, C, Tc, rank)

    def step(i):
        ch.spec = specs[i % len(specs)]
        ch.run(cubes[i % 2], esprit=False, velocity=False)
    for i in range(max(warmup, len(specs))):  # every output buffer written once before the timed steps
        step(i)
    torch.cuda.synchronize()
    ne, nc = ch.totals()
    if ne > ch.entry_cap or nc > ch.cell_cap:
        raise RuntimeError('peak capacity exceeded')
    if timing:
        ctx.timing(True)
        ctx.timing_reset()
    if DIST and collective:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    if DIST and collective:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if collective:
        elapsed = _sync_max(elapsed, dev)
    kt = ctx.timing_read() if timing else {}
    spans = ctx.timing_spans() if timing else {}
    ctx.timing(False)
    G = len(ch.grid)
    out = {"value": F * steps * (world if collective else 1) / elapsed, "unit": "frames/s",
           "ms_per_step": elapsed / steps * 1e3, "steps": steps, "warmup": warmup, "frames_per_step": F,
           "peaks_per_frame": ne / F, "cells_per_frame": nc / F, "doa_grid": G, "spectrum_buffers": len(specs)}
    if spans.get('doa_scan'):
        per_buf = {}
        for i, (a, b) in enumerate(spans['doa_scan']):
            per_buf.setdefault(i % len(specs), []).append(round(b - a, 3))
        out["scan_ms_per_buffer"] = {str(k): v for k, v in per_buf.items()}
    if kt:
        per = lambda k: kt[k][0] / max(kt[k][1], 1)
        sbytes = nc * G * 4 + nc * A * 8  # spectrum store + signature gather
        t = per('doa_scan') * 1e-3
        out["roofline"] = {"bound": "hbm", "kernel": "k_doa_toep (spectrum, Toeplitz f16 MFMA)",
                           "achieved": sbytes / t / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": sbytes / t / 1e9 / HBM_PEAK_GBS, "traffic": spectrum_traffic(F),
                           "traffic_source": 'PMC FETCH_SIZE x 2 + WRITE_SIZE from ' + os.path.relpath(SPEC_PROFILE, ROOT),
                           "avg_launch_ms": per('doa_scan'), "algorithmic_bytes_per_launch": sbytes}
        fb = 2 * A * C * S * 8 * F
        tf = (per('range_fft') + per('doppler_fft')) * 1e-3
        out["fft_stage"] = {"bound": "hbm", "achieved": fb / tf / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": fb / tf / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": fb}
        out["kernel_ms_per_step"] = {k: v[0] / max(v[1], 1) for k, v in kt.items() if v[1]}
    del ch, cubes, specs
    torch.cuda.empty_cache()
    return out


def run_spectrum(args, world, rank, local, dev):
    """`--config spectrum`: configs[1] as its own JSON line (measure_spectrum)."""
    import rsl
    ctx = rsl.get_context(local)
    F = args.frames_per_step or 1000
    r = measure_spectrum(ctx, dev, F, args.steps, args.warmup, rank, world, timing=not args.no_timing)
    if rank != 0:
        return
    line = {"metric": "radar frames/sec, range-Doppler FFT + MUSIC spectrum (configs[1]), 8ch x 128chirp x 512",
            "value": r.pop("value"), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": r.pop("ms_per_step"), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "configs[1]: 8ch x 128chirp x 512 synthetic cube, RDS + peaks + MUSIC spectrum of "
                                   "every unique cell (f32, cell-blocked [cells/32, 361, 32])", "frames_per_step": F,
                       "doa_grid": r["doa_grid"], "parallelism": f"frame-sharded x{world}"}}
    line.update({k: v for k, v in r.items() if k not in ("steps", "warmup", "frames_per_step", "unit")})
    print(json.dumps(line), flush=True)


def kernel_bytes_k1k2(A, C, S, F):
    """Design bytes per launch of K1 / K2 (the work round trip included: kernel efficiencies, not the stage roofline).
    Packed `work` at cfg2 (rsl_fft.hip pk_pack16: 6 B per value, the bin's exponent inside its 48-B unit):
      K1 k_range_fft_r512: read the c64 cube (8 B per value) + write the packed range spectra (6 B)  = A C S 14 B/frame
      K2 k_doppler_detect_r128: read the packed spectra of 16 + 2 halo range bins per 16-bin tile + write the c64 RDS
         (masks / peak powers, ~1 %, not counted)                                     = A C S (6 x 18 / 16 + 8) B/frame
    c64 `work` at other shapes (k_range_fft_p / k_doppler_detect): 2 A C S 8 B per frame each."""
    if (C, S) in ((128, 512), (256, 1024)):  # packed (cfg2; cfg5: k_range_fft_r1024 / k_doppler_detect_r256, the same)
        return {'range_fft': A * C * S * 14.0 * F, 'doppler_fft': A * C * S * (6.0 * 18 / 16 + 8) * F}
    if (C, S) == (64, 256):  # packed, 32-bin K2 tiles (k_doppler_detect_r64)
        return {'range_fft': A * C * S * 14.0 * F, 'doppler_fft': A * C * S * (6.0 * 34 / 32 + 8) * F}
    return {'range_fft': 2 * A * C * S * 8 * F, 'doppler_fft': 2 * A * C * S * 8 * F}


def chain_traffic_per_frame():
    """Whole-chain HBM bytes per frame from the committed PMC profile (every rsl:: kernel of the timed chain: K1, K2,
    offsets, compaction, DoA, velocity, trajectory; the synthesis is not in the timed region), or None."""
    try:
        prof = json.load(open(PROFILE))
    except (OSError, ValueError):
        return None
    tot = sum(e.get('hbm_bytes', 0.0) for name, e in prof.get('kernels', {}).items()
              if name.startswith('rsl::') and not name.startswith('rsl::k_synth'))
    return tot / prof.get('frames_per_launch', 1000)


def measure_chain(ctx, dev, A, C, Tc, F, steps, warmup, rank, world, *, ridge=0.01, pipeline=True, streams=1,
                  timing=True, standalone=True, collective=True):
    """The full chain (RDS + peaks + MUSIC argmax + ESPRIT + LS velocity + trajectory) on batches of F frames already
    resident in HBM: `steps` timed steps after `warmup`, bracketed by barrier + synchronize (max over ranks when
    `collective`).  Returns elapsed seconds, per-kernel timings (live and standalone), totals and the chain."""
    import torch
    import torch.distributed as dist
    import rsl
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc, ridge=ridge)
    NS = max(1, streams)
    if F % NS:
        raise SystemExit('--frames-per-step must be a multiple of --streams')
    nb = 2
    cubes = make_cubes(ctx, nb, F, A, C, cfg.chirp_duration, rank)
    # trajectory reduction: device prefix scan of this rank's frame block, all-gather of the
    # 16-double block summaries and of the per-frame poses over RCCL/xGMI (rsl/traj.py)
    reducer = rsl.TrajectoryReducer(ctx, F, dt=cfg.dt, collective=collective)
    main = torch.cuda.current_stream(dev)
    if pipeline:
        NS = 1
        # RSL_BENCH_NBUF: chain buffers in flight (2: batch i + 1's front half waits for batch i - 1's back half)
        NBUF = max(2, int(os.environ.get('RSL_BENCH_NBUF', '2')))
        vel2 = torch.empty((NBUF, F, 8), dtype=torch.float64, device=dev)
        chains = [rsl.RadarChain(cfg, F, ctx, vel_out=vel2[k]) for k in range(NBUF)]
        # RSL_BENCH_PRIO: stream priorities (front:back, torch's convention: lower = higher priority; 0:0 = equal)
        pf, pb = (int(x) for x in os.environ.get('RSL_BENCH_PRIO', '0:0').split(':'))
        sA, sB = torch.cuda.Stream(dev, priority=pf), torch.cuda.Stream(dev, priority=pb)
        cum = os.environ.get('RSL_BENCH_CUMASK')  # "front:back" CU counts: the two halves on CU-masked streams
        if cum:
            nf, nbk = (int(x) for x in cum.split(':'))
            sA, sB = cu_masked_stream(dev, nf, 0), cu_masked_stream(dev, nbk, 1)
        evA = [torch.cuda.Event() for _ in range(NBUF)]
        evB = [torch.cuda.Event() for _ in range(NBUF)]
        # the trajectory (scan, RCCL summary all-gather, pose gather to rank 0, smoothing) on a third stream, so the
        # collectives' latency stays off the back stream: batch i + 1's DoA does not wait for batch i's gather
        sC = torch.cuda.Stream(dev) if os.environ.get('RSL_BENCH_TRAJ_STREAM', '1') != '0' else None
        evC = [torch.cuda.Event() for _ in range(NBUF)]
        used = [False] * NBUF
    else:
        vel = torch.empty((F, 8), dtype=torch.float64, device=dev)
        chains = [rsl.RadarChain(cfg, F // NS, ctx, vel_out=vel[k * (F // NS):(k + 1) * (F // NS)]) for k in range(NS)]
        streams = [torch.cuda.Stream(dev) for _ in range(NS)]
    # 0: offsets + compaction on the front stream; 1: compaction on the back stream; 2: both on the back stream
    # default 0 since round 6: 215.7-216.6 k vs 211.4-213.5 k frames/s with the compaction on the back stream (5 rounds
    # alternating in one call, gpurun_out/r6ab_*): on the back stream it co-ran with the next K1 at 3 ms live
    # instead of 0.7 and sat on the back half's critical path
    EMIT_BACK = int(os.environ.get('RSL_BENCH_EMIT_BACK', '0'))

    def step_pipelined(i):
        k = i % len(chains)
        ch = chains[k]
        sA.wait_stream(main)
        with torch.cuda.stream(sA):
            if used[k]:
                sA.wait_event(evB[k])  # batch i-2's back half is done with these buffers
            ch.run_front(cubes[i % nb], emit=EMIT_BACK == 0, offsets=EMIT_BACK < 2)
            evA[k].record(sA)
        with torch.cuda.stream(sB):
            sB.wait_event(evA[k])
            if sC is not None and used[k]:
                sB.wait_event(evC[k])  # batch i-2's trajectory step has read chain k's velocities
            ch.run_back(emit=EMIT_BACK > 0, offsets=EMIT_BACK == 2)
            if sC is None:
                reducer.step(ch.vel, vstride=ch.vel.shape[1], nv=2)
            evB[k].record(sB)
        if sC is not None:
            with torch.cuda.stream(sC):
                sC.wait_event(evB[k])
                reducer.step(ch.vel, vstride=ch.vel.shape[1], nv=2)
                evC[k].record(sC)
        used[k] = True

    def step(i):
        if pipeline:
            return step_pipelined(i)
        cube = cubes[i % nb]
        for k, (ch, st) in enumerate(zip(chains, streams)):  # independent frame slices, concurrent streams
            st.wait_stream(main)
            with torch.cuda.stream(st):
                ch.run(cube[k * (F // NS):(k + 1) * (F // NS)])
        for st in streams:
            main.wait_stream(st)
        reducer.step(vel, vstride=vel.shape[1], nv=2)

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    for ch in (chains[:min(warmup, len(chains))] if pipeline else chains):  # the chains that ran (pipelined: one per step)
        ne, nc = ch.totals()
        if ne > ch.entry_cap or nc > ch.cell_cap:
            raise RuntimeError('peak capacity exceeded')
    if timing:
        ctx.timing(True)
        ctx.timing_reset()
    if DIST and collective:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    if DIST and collective:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if collective:
        elapsed = _sync_max(elapsed, dev)
    kt = ctx.timing_read() if timing else {}
    spans = ctx.timing_spans() if timing else {}  # per launch [start, end] on one device clock (the live timeline)
    ks = {}  # standalone kernel times: the pipelined timed region overlaps the two halves of consecutive batches
    if kt and pipeline and standalone:
        ctx.timing_reset()
        for i in range(STANDALONE_RUNS):  # one chain at a time on one stream; per-kernel means over these runs
            chains[0].run(cubes[i % nb])
        torch.cuda.synchronize()
        ks = ctx.timing_read()
    ctx.timing(False)
    counted = chains[:1] if pipeline else chains  # pipelined: both buffers hold a full batch
    ne = sum(ch.totals()[0] for ch in counted)
    nc = sum(ch.totals()[1] for ch in counted)
    return dict(elapsed=elapsed, kt=kt, ks=ks, spans=spans, ne=ne, nc=nc, NS=NS, G=len(chains[0].grid), cubes=cubes,
                chains=chains, reducer=reducer)


def live_timeline(spans, steps):
    """The unprofiled live timeline from the per-launch hipEvent spans of the timed steps (rsl_timing_spans): for each
    scope its per-launch durations (median and range), and one step (the middle one) laid out against the start of
    that step's range FFT, so the two streams' overlap can be read off (events time a scope from the later of its
    stream's previous command and the cross-stream wait in front of it, to the end of its last kernel)."""
    if not spans or 'range_fft' not in spans:
        return None
    out = {"what": "hipEvent spans of the timed steps (per launch): the unprofiled schedule", "scopes": {}}
    for k, v in spans.items():
        d = sorted(b - a for a, b in v)
        out["scopes"][k] = {"launches": len(d), "median_ms": d[len(d) // 2], "min_ms": d[0], "max_ms": d[-1]}
    i = len(spans['range_fft']) // 2
    t0 = spans['range_fft'][i][0]
    step = {}
    for k, v in spans.items():
        near = [(a - t0, b - t0) for a, b in v if -12.0 < a - t0 < 12.0]
        if near:
            step[k] = [[round(a, 3), round(b, 3)] for a, b in near]
    out["step_ms_relative_to_range_fft_start"] = step
    out["spans_ms"] = {k: [[round(a, 3), round(b, 3)] for a, b in v] for k, v in spans.items()}
    return out


def chain_rooflines(r, A, C, S, F, config):
    """roofline (FFT stage, live), fft_stage_standalone, roofline_doa, kernel_rooflines_standalone and the per-kernel
    ms of one measure_chain result."""
    kt, ks, NS, G = r['kt'], r['ks'], r['NS'], r['G']
    tsrc = TRAFFIC_SOURCE if config != 'cfg5' else TRAFFIC_SOURCE.replace(os.path.relpath(PROFILE, ROOT),
                                                                          os.path.relpath(CFG5_PROFILE, ROOT))
    out = {}
    if not kt:
        return out
    per = lambda name: kt[name][0] / max(kt[name][1], 1)  # ms per launch
    Fl = F // NS
    ncl = r['nc'] / NS  # unique cells per launch
    # Algorithmic work per launch:
    #  FFT stage (K1 + K2): read the c64 cube + write the c64 RDS, counted once: 2 A C S 8 B per frame
    #  K5 k_doa_toep: one real dot product of length 2M-1 per (cell, grid point) (Toeplitz form of |a^H s|^2),
    #     evaluated as three f16 MFMA products for fp32 accuracy (hi/lo split) -> 3 * 2 * (2M - 1) flops
    src_std = ks if ks else kt
    fft_names = {(128, 512): {'range_fft': 'k_range_fft_r512', 'doppler_fft': 'k_doppler_detect_r128'},
                 (256, 1024): {'range_fft': 'k_range_fft_r1024', 'doppler_fft': 'k_doppler_detect_r256'},
                 (64, 256): {'range_fft': 'k_range_fft_r256', 'doppler_fft': 'k_doppler_detect_r64'}}.get(
        (C, S), {'range_fft': 'k_range_fft_p', 'doppler_fft': 'k_doppler_detect'})
    per_std = lambda name: src_std[name][0] / max(src_std[name][1], 1)
    flops = 3 * 2 * (2 * A - 1) * ncl * G
    Ff = Fl  # frames per K1 / K2 launch
    kbytes = kernel_bytes_k1k2(A, C, S, Ff)

    def entry(name, ms):
        if name == 'doa_scan':
            ach = flops / (ms * 1e-3) / 1e12
            # the scope holds K5 and k_doa_fixup (the exact fp64 re-scan of its marked near-ties, launched right
            # after on the same stream): the rate is charged for both
            return {"bound": "mfma", "kernel": "k_doa_toep + k_doa_fixup", "achieved": ach, "peak": F16_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": ach / F16_MFMA_PEAK_TFLOPS,
                    "traffic": pmc_traffic('k_doa_toep', Fl, config), "traffic_source": tsrc,
                    "avg_launch_ms": ms, "algorithmic_flops_per_launch": flops,
                    "reference_equivalent_flops_per_launch": ncl * G * (8 * A + 5)}
        kern = fft_names[name]
        ach = kbytes[name] / (ms * 1e-3) / 1e9
        return {"bound": "hbm", "kernel": kern, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": ach / HBM_PEAK_GBS, "traffic": pmc_traffic(kern, Ff, config),
                "traffic_source": tsrc, "avg_launch_ms": ms, "design_bytes_per_launch": kbytes[name],
                "note": "per-kernel design bytes (cube or work in, work or RDS out): the work round trip counts "
                        "here, so these fractions are kernel efficiencies, not the stage's algorithmic roofline"}

    # Headline roofline = the FFT stage: its algorithmic bytes counted ONCE per frame over the summed
    # average launch durations of the kernels that implement it (K1 range FFT + K2 Doppler FFT / fftshift / detection),
    # measured live by hipEvents on their stream over the timed region; traffic = the same kernels' PMC HBM bytes per
    # launch.  The `work` intermediate between K1 and K2 is NOT algorithmic: it shows up as traffic above the
    # algorithmic bytes.
    big = ('range_fft', 'doppler_fft', 'doa_scan')
    fft_k = [k for k in ('range_fft', 'doppler_fft') if k in kt and kt[k][1]]
    fft_bytes = 2 * A * C * S * 8 * Ff

    def stage(src, timed):
        t = sum(src[k][0] / max(src[k][1], 1) for k in fft_k) * 1e-3
        tr = [pmc_traffic(fft_names[k], Ff, config) for k in fft_k]
        return {"bound": "hbm", "kernels": [fft_names[k] for k in fft_k],
                "achieved": fft_bytes / t / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": fft_bytes / t / 1e9 / HBM_PEAK_GBS,
                "traffic": None if any(x is None for x in tr) else sum(tr), "traffic_source": tsrc,
                "avg_launch_ms": t * 1e3, "algorithmic_bytes_per_launch": fft_bytes, "timed": timed}

    out["roofline"] = stage(kt, "hipEvents over the timed region (pipelined: the stage co-runs with the previous "
                                "batch's DoA scan)" if ks else "hipEvents over the timed region")
    if ks:
        out["fft_stage_standalone"] = stage(ks, f"mean of {STANDALONE_RUNS} standalone launches after the timed region")
        # the same stage's unshared rate beside the live one (the live spans include the other batch's co-running
        # kernels: the pipelined step is shorter, each span longer)
        out["roofline"]["frac_standalone"] = out["fft_stage_standalone"]["frac"]
    out["roofline_doa"] = entry('doa_scan', per('doa_scan'))
    if ks and 'doa_scan' in src_std:
        out["roofline_doa"]["frac_standalone"] = entry('doa_scan', per_std('doa_scan'))["frac"]
    out["roofline_doa"]["timed"] = (
        "hipEvents over the timed region (pipelined: the scan co-runs with the next batch's K1 / K2, which stretches "
        "its span while the step gets shorter; the unshared rate is kernel_rooflines_standalone.doa_scan)" if ks
        else "hipEvents over the timed region")
    out["kernel_rooflines_standalone"] = {k: entry(k, per_std(k)) for k in big if k in src_std}
    out["kernel_ms_per_step"] = {k: v[0] / max(v[1], 1) * (NS if k not in fft_names else Fl * NS / Ff)
                                 for k, v in kt.items() if v[1]}
    if ks:
        out["kernel_ms_standalone"] = {k: v[0] / max(v[1], 1) for k, v in ks.items() if v[1]}
    return out


def configs_4_frame(ctx, dev, F=400, steps=313, warmup=2):
    """configs[4] frame shape (A16 C256 S1024, the 1 M-frame 8-GPU workload's frame) on this GPU: one rank's share of
    the 1 M frames (313 steps x 400 = 125.2 k frames >= 1 M / 8) through the same full chain, pipelined, with the
    trajectory reduction stepped over every batch (its state carried across all of them), this rank only (no
    collective).  The inputs cycle over two resident 400-frame batches (125 k distinct cubes would be 2.1 TB)."""
    import torch
    A, C, S, Tc = 16, 256, 1024, 102.4e-6
    r = measure_chain(ctx, dev, A, C, Tc, F, steps, warmup, 0, 1, standalone=True, collective=False)
    out = {"what": "configs[4] frame shape (16ch x 256chirp x 1024), full chain pipelined + trajectory, one GPU, "
                   f"{F} frames per step, {steps} timed steps ({F * steps} frames: one rank's share of 1 M frames "
                   "on 8 GPUs; the inputs cycle over two resident batches)", "value": F * steps / r['elapsed'],
           "unit": "frames/s", "ms_per_step": r['elapsed'] / steps * 1e3, "frames_per_step": F,
           "frames_timed": F * steps, "wall_s": r['elapsed'],
           "peaks_per_frame": r['ne'] / F, "cells_per_frame": r['nc'] / F,
           "per_rank_share_1M_frames_8_gpus": {"frames": F * steps, "measured_s": r['elapsed'],
                                               "note": "one rank's share measured on one GPU; 8 ranks running "
                                                       "concurrently on one node unmeasured (no 8-GPU node)"}}
    rf = chain_rooflines(r, A, C, S, F, 'cfg5')
    for k in ('roofline', 'fft_stage_standalone', 'roofline_doa', 'kernel_ms_standalone'):
        if k in rf:
            out[k] = rf[k]
    del r
    torch.cuda.empty_cache()
    return out


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, script=None, grace=300.0):
    """`--gpus N` (N > 1) without an external launcher: bring up N rank processes of this script, one per GPU (rank r
    on device r), the way torch.distributed.run would, and relay rank 0's JSON line.  This process touches no GPU (it
    does not even import torch) and never execs: each rank is a fresh child (subprocess.Popen) with RANK, LOCAL_RANK,
    WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR = 127.0.0.1 and MASTER_PORT in its environment.  If any rank exits
    non-zero the others are terminated and this process exits with that rank's code; ranks still
    running ``grace`` seconds after another one finished are ended too (non-zero).  ``script``: the rank program
    (default this file; tests substitute a stub)."""
    import subprocess
    import threading
    port = int(os.environ.get('MASTER_PORT') or _free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, '-u', script or os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else 2, text=True))  # other ranks: fd 2
    lines = []

    def relay():  # rank 0's stdout (the JSON line and anything else it prints) to this process's stdout
        for line in procs[0].stdout:
            lines.append(line)
            sys.stdout.write(line)
            sys.stdout.flush()
    th = threading.Thread(target=relay, daemon=True)
    th.start()
    rc = 0
    live = set(range(n))
    t_first = None  # when the first rank finished: the others get a grace period, then they are ended
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            t_first = t_first or time.monotonic()
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                sys.stderr.write(f'bench.py: rank {r} exited with {c}; terminating the other ranks\n')
                for q in live:
                    procs[q].terminate()
        if live and t_first is not None and time.monotonic() - t_first > grace:
            sys.stderr.write(f'bench.py: ranks {sorted(live)} still running {grace:g} s after another rank finished; '
                             'terminating them\n')
            for q in live:
                procs[q].terminate()
            rc = rc or 1
            t_first = time.monotonic() + 1e9  # terminate once; the loop then collects their exit codes
        time.sleep(0.05)
    th.join(timeout=10)
    if rc == 0 and not any(l.lstrip().startswith('{') for l in lines):
        sys.stderr.write('bench.py: rank 0 printed no JSON line\n')
        rc = 1
    return rc


def _spectrum_sub(ctx, dev):
    """The configs_1_spectrum sub-object: 1000 frames per step, 6 timed steps over the 3 rotated output buffers."""
    import torch
    try:
        return measure_spectrum(ctx, dev, 1000, 6, 1, 0, 1, collective=False)
    except Exception as e:
        torch.cuda.empty_cache()
        return {"error": repr(e)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--frames-per-step', type=int, default=None,
                    help='frames per GPU per step (default 2000 for cfg2, 400 for cfg5)')
    ap.add_argument('--config', choices=('cfg2', 'cfg5', 'spectrum'), default='cfg2',
                    help='cfg2 = configs[2] (A8 C128 S512, the metric\'s workload); cfg5 = the configs[4] frame shape '
                         '(A16 C256 S1024); spectrum = configs[1] (A8 C128 S512, 1000 frames per step: RDS + peaks + '
                         'the full MUSIC spectrum of every cell, f32 [G, cells]); the last two are second '
                         'measurements, not the metric line')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-pcie', action='store_true', help='skip the PCIe-inclusive side measurement')
    ap.add_argument('--no-extra', action='store_true',
                    help='skip the configs[1] / configs[4]-frame sub-measurements of the default cfg2 line')
    ap.add_argument('--cpu-peaks', type=int, default=3000,
                    help='peaks per frame through the loop-faithful CPU DoA (the bounded sample; <= 0: every peak)')
    ap.add_argument('--cpu-procs', type=int, default=0,
                    help='worker processes of the CPU baseline (0: every host core this process may use)')
    ap.add_argument('--ridge', type=float, default=0.01,
                    help='ridge on (v_x, v_y) of the LS velocity solve (configs[2]: "regularised LS"; the 0.01 of '
                         'velocity_solver_improved.py:261); 0 = the plain VelocitySolver LS')
    ap.add_argument('--no-timing', action='store_true', help='disable per-kernel hipEvent timing')
    ap.add_argument('--streams', type=int, default=int(os.environ.get('RSL_BENCH_STREAMS', '1')),
                    help='concurrent HIP streams per GPU; each runs the chain on F/streams frames of the step')
    ap.add_argument('--pipeline', type=int, default=int(os.environ.get('RSL_BENCH_PIPELINE', '1')),
                    help='1: double-buffered chains on two streams; batch i+1\'s memory-bound front half (RDS, '
                         'detection, offsets) runs concurrently with batch i\'s back half (compaction, DoA, '
                         'velocity, trajectory)')
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit('bench.py: --gpus must be >= 1')
    if 'WORLD_SIZE' in os.environ:  # an external launcher (torch.distributed.run) or launch_ranks brought this rank up
        if int(os.environ['WORLD_SIZE']) != args.gpus:
            raise SystemExit(f'bench.py: WORLD_SIZE={os.environ["WORLD_SIZE"]} but --gpus {args.gpus}: launch one rank '
                             'per GPU (--nproc-per-node = --gpus)')
    elif args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # torch.cuda.device_count() initialises no device on this image (the GPU is first touched by set_device below)
    if 'RSL_BENCH_DEVICE' not in os.environ and local >= torch.cuda.device_count():
        raise SystemExit(f'bench.py: rank {rank} needs device {local} but {torch.cuda.device_count()} are visible '
                         f'(--gpus {args.gpus}; RSL_BENCH_DEVICE=d puts every rank on device d for a rehearsal)')
    global DIST
    # RSL_BENCH_DIST=1: bring the process group up at world size 1 too (torchrun --nproc-per-node 1), so a one-GPU box
    # runs the RCCL initialisation, barriers, the max-over-ranks all-reduce and the trajectory collectives
    DIST = world > 1 or os.environ.get('RSL_BENCH_DIST') == '1'
    if 'RSL_BENCH_DEVICE' in os.environ:  # rehearsal of the N > 1 path on a one-GPU box (all ranks on one device)
        local = int(os.environ['RSL_BENCH_DEVICE'])
    if DIST:
        torch.cuda.set_device(local)
        backend = os.environ.get('RSL_BENCH_BACKEND', 'nccl')  # nccl = RCCL over xGMI; gloo only for rehearsals
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)

    import rsl
    if args.config == 'spectrum':
        return run_spectrum(args, world, rank, local, dev)
    if args.config == 'cfg5':
        # 400 frames per step: the small per-batch kernels (offsets, one velocity workgroup per frame) fill the GPU
        # (23.3 k vs 21.6 k frames/s at 100, gpurun_out/r5ad_cfg5f*); a 1 M-frame run batches at least this many
        A, C, S, Tc, F = 16, 256, 1024, 102.4e-6, args.frames_per_step or 400
    else:
        A, C, S, Tc, F = 8, 128, 512, 51.2e-6, args.frames_per_step or 2000  # 5 steps = configs[2]'s 10 k frames
    ctx = rsl.get_context(local)
    extras = not args.no_extra and world == 1 and args.config == 'cfg2'
    spec_first = os.environ.get('RSL_BENCH_SPEC_FIRST', '1') != '0'
    spec = None
    if extras and spec_first:
        # configs[1] first, in the process's untouched device memory: its 3 x 57 GB of spectrum buffers placed after
        # the cfg2 chain's alloc / free cycle were store-stalled (11.0 vs 9.0-9.4 ms per 1000 frames) in most
        # placements, in untouched memory less often (not never: DESIGN §5)
        spec = _spectrum_sub(ctx, dev)
    r = measure_chain(ctx, dev, A, C, Tc, F, args.steps, args.warmup, rank, world, ridge=args.ridge,
                      pipeline=bool(args.pipeline), streams=args.streams, timing=not args.no_timing)
    elapsed, ne, nc, NS = r['elapsed'], r['ne'], r['nc'], r['NS']
    frames_total = F * args.steps * world
    fps = frames_total / elapsed
    if rank != 0:
        if DIST:
            dist.destroy_process_group()
        return
    G = r['G']
    line = {
        "metric": METRIC, "value": fps, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": ("configs[2]: 8ch x 128chirp x 512" if args.config == 'cfg2' else
                                "configs[4] frame shape: 16ch x 256chirp x 1024") + " synthetic cube, full chain "
                               "(RDS + peaks + MUSIC argmax + ESPRIT + "
                               + (f"regularised LS velocity (ridge {args.ridge:g} on v_x, v_y: the regulariser of "
                                  "velocity_solver_improved.py:261 on velocity_solver.py's unwrapped LS)" if args.ridge
                                  else "plain LS velocity (velocity_solver.py)") + " + trajectory)",
                   "velocity_ridge": args.ridge,
                   "frames_per_step": F, "frames_per_gpu_per_step": F, "antennas": A, "chirps": C, "samples": S,
                   "doa_grid": G, "streams_per_gpu": 2 if args.pipeline else NS,
                   "pipelined": bool(args.pipeline), "parallelism": f"frame-sharded x{world}"},
        "peaks_per_frame": ne / F, "cells_per_frame": nc / F,
    }
    line.update(chain_rooflines(r, A, C, S, F, args.config))
    tl = live_timeline(r.get('spans'), args.steps)
    if tl:
        line["live_timeline"] = tl
    if args.config == 'cfg2':
        # whole-chain HBM traffic per frame (committed PMC profile) beside the chain's algorithmic bytes (SURVEY §8d:
        # FFT stage 2 A C S 8 B + the DoA signature gather 8 M N_p)
        npk = ne / F
        line["chain_traffic_bytes_per_frame"] = chain_traffic_per_frame()
        line["chain_algorithmic_bytes_per_frame"] = 2 * A * C * S * 8 + 8 * A * npk
        line["chain_traffic_source"] = ('sum of every rsl:: chain kernel\'s PMC FETCH_SIZE x 2 + WRITE_SIZE in '
                                        + os.path.relpath(PROFILE, ROOT) + ' / frames per launch')
    del r
    torch.cuda.empty_cache()
    if extras:
        # the other two GPU workloads of BASELINE.json, bounded (a few seconds each), as sub-objects of the metric line
        line["configs_1_spectrum"] = spec if spec is not None else _spectrum_sub(ctx, dev)
        line["configs_1_spectrum"]["measured"] = "before the cfg2 line" if spec_first else "after the cfg2 line"
        try:
            line["configs_4_frame"] = configs_4_frame(ctx, dev)
        except Exception as e:
            line["configs_4_frame"] = {"error": repr(e)}
    if not args.no_pcie and world == 1 and args.config == 'cfg2':
        line["pcie_inclusive"] = pcie_inclusive(ctx, dev)
    if not args.no_cpu_baseline and world == 1:  # the CPU baseline is timed on rank 0 at N = 1 only
        try:
            line["cpu_baseline"] = cpu_baseline(args.cpu_procs, args.cpu_peaks, ridge=args.ridge)
        except Exception as e:  # the baseline is reported, never the target
            line["cpu_baseline"] = {"error": repr(e)}
    print(json.dumps(line), flush=True)
    if DIST:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()

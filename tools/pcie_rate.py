"""PCIe-inclusive throughput of the cfg2 chain: the metric's `value` starts with the cubes resident in
HBM; this measures the rate when every frame's c64 cube [A, C, S] (4 MiB at cfg2) first crosses PCIe from pinned host
memory. Host-to-device copies of batch i+1 run on a copy stream while the chain processes batch i; each batch's
per-frame velocities come back to pinned host memory. Also reports the raw pinned H2D bandwidth.

    python tools/pcie_rate.py [--frames 500] [--steps 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'radar-slam_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--frames', type=int, default=500)
    ap.add_argument('--steps', type=int, default=8)
    args = ap.parse_args()

    import torch
    import rsl
    from bench import SCENE

    dev = torch.device('cuda', 0)
    A, C, Tc, F = 8, 128, 51.2e-6, args.frames
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc)
    ctx = rsl.get_context(0)
    gen = rsl.SyntheticCubes(ctx, SCENE, chirp_duration=Tc, num_chirps=C, num_antennas=A, noise_power=0.01)
    host = []
    for i in range(2):  # two distinct pinned host batches, generated on the device and copied out once
        d = gen.generate(F, seed=1234, frame0=i * F)
        torch.cuda.synchronize()
        h =torch.empty(d.shape, dtype=d.dtype, pin_memory=True)
        h.copy_(d)
        host.append(h)
        del d
    torch.cuda.synchronize()
    dbuf = [torch.empty(host[0].shape, dtype=host[0].dtype, device=dev) for _ in range(2)]
    vel_d = [torch.empty((F, 8), dtype=torch.float64, device=dev) for _ in range(2)]
    vel_h = [torch.empty((F, 8), dtype=torch.float64, pin_memory=True) for _ in range(2)]
    chains = [rsl.RadarChain(cfg, F, ctx, vel_out=vel_d[k]) for k in range(2)]
    bytes_per_batch = host[0].numel() * host[0].element_size()

    # raw pinned H2D bandwidth (one stream)
    cs = torch.cuda.Stream(dev)
    with torch.cuda.stream(cs):
        dbuf[0].copy_(host[0], non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(cs):
        for i in range(4):
            dbuf[i % 2].copy_(host[i % 2], non_blocking=True)
    torch.cuda.synchronize()
    h2d_gbs = 4 * bytes_per_batch / (time.perf_counter() - t0) / 1e9

    ks = torch.cuda.Stream(dev)
    ev_copy = [torch.cuda.Event() for _ in range(2)]
    ev_done = [torch.cuda.Event() for _ in range(2)]
    used = [False, False]

    def step(i):
        k = i % 2
        with torch.cuda.stream(cs):
            if used[k]:
                cs.wait_event(ev_done[k])  # batch i-2 is done with dbuf[k] and vel_d[k]
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
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    fps = args.steps * F / el

    # device-resident rate of the same (unpipelined, one compute stream) loop, for comparison
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(ks):
        for i in range(args.steps):
            chains[i % 2].run(dbuf[i % 2])
    torch.cuda.synchronize()
    fps_res = args.steps * F / (time.perf_counter() - t0)
    ne, nc = chains[0].totals()
    print(json.dumps({
        "what": "cfg2 chain with the c64 cube copied host->device per batch (pinned, copy stream overlapped)",
        "frames_per_batch": F, "steps": args.steps, "bytes_per_frame": bytes_per_batch // F,
        "h2d_pinned_GBps": round(h2d_gbs, 2), "pcie_inclusive_frames_per_s": round(fps, 1),
        "pcie_bound_frames_per_s": round(h2d_gbs * 1e9 / (bytes_per_batch / F), 1),
        "device_resident_frames_per_s_same_loop": round(fps_res, 1),
        "peaks_first_batch": ne, "cells_first_batch": nc}))


if __name__ == '__main__':
    main()

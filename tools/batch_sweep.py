"""Per-kernel device time per frame vs batch size (does a small batch keep `work`/`rds` in the 256 MiB
Infinity Cache?).  Each batch size runs the chain repeatedly on the same cube buffer."""
import os, sys, json, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch, rsl
from bench import make_cubes
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
dev = torch.device('cuda', 0)
for F in [int(x) for x in os.environ.get('FS', '8,16,32,64,128,256,1000').split(',')]:
    ch = rsl.RadarChain(cfg, F, ctx)
    nb = max(1, 2000 // F)
    cubes = make_cubes(torch, dev, 1, F * min(nb, 8), 8, 128, 512, 7)[0].view(min(nb, 8), F, 8, 128, 512)
    reps = max(4, 2000 // F)
    for i in range(3):
        ch.run(cubes[i % cubes.shape[0]])
    torch.cuda.synchronize()
    ctx.timing(True)
    ctx.timing_reset()
    t0 = time.perf_counter()
    for i in range(reps):
        ch.run(cubes[i % cubes.shape[0]])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kt = ctx.timing_read()
    ctx.timing(False)
    per = {k: round(v[0] / (reps * F) * 1e3, 2) for k, v in kt.items() if v[1]}  # us per frame
    print(json.dumps({'F': F, 'fps_wall': round(reps * F / dt), 'us_per_frame': per}), flush=True)
    del ch, cubes
    torch.cuda.empty_cache()

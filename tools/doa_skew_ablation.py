"""K5 (k_doa_toep, the skewed 12-tile kernel the chain runs) ablations on one cfg2 batch, development library
(RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so): RSL_DOA_DBG 1 = no record-tile copies, 3 = no signature loads,
8 = no argmax epilogue (one max per tile), 9 = no tile loop; each with the fused extras (ESPRIT + phase, as the chain
runs it) and without ('noext').  Results of 1-9 are wrong by construction; only the times matter (EXACT=0,... lists the variants whose grid indices
are compared with the chain's)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F = int(os.environ.get('F', '2000'))
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, 8, 128, 51.2e-6, 0)[0]
ch.run(cube)
torch.cuda.synchronize()
L = ch.lists
ref_idx = ch.gidx.clone()
res = {}
for rnd in range(3):
    for v in os.environ.get('VARIANTS', '0,1,3,8,9').split(','):
        for ext in (True, False):
            os.environ['RSL_DOA_DBG'] = v
            idx = torch.empty_like(ch.gidx)
            if ext:
                run = lambda: ctx.doa_extras(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=ch.cell_cap,
                                             n_dev=ch.ncell_dev, esprit_scale=ch.esprit_scale, out_idx=idx,
                                             esprit=ch.ext['esprit'], phase=ch.ext['phase'])
            else:
                run = lambda: ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=ch.cell_cap,
                                      n_dev=ch.ncell_dev, out_idx=idx)
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record()
            torch.cuda.synchronize()
            key = f"dbg{v}{'' if ext else '_noext'}"
            res.setdefault(key, []).append(e0.elapsed_time(e1) / 5)
            if v in os.environ.get('EXACT', '0').split(',') and rnd == 0:
                nc = int(ch.totals()[1])
                res[key + '_idx_equal'] = bool(torch.equal(idx[:nc], ref_idx[:nc]))
os.environ.pop('RSL_DOA_DBG')
print(json.dumps({k: (round(min(x), 4) if isinstance(x, list) else x) for k, x in res.items()}), flush=True)

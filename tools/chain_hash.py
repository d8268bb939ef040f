"""SHA-256 of every output of one cfg2 chain batch (RDS, masks, row counts, peak powers, offsets, lists, DoA, ESPRIT,
phase, velocity) under the library RSL_LIBRARY: equal hashes across two libraries = bit-identical chains.
GPU box:  [CFG=cfg1|cfg2|cfg5] [F=frames] RSL_LIBRARY=... python tools/chain_hash.py"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

A, C, TC = {'cfg1': (8, 64, 25.6e-6), 'cfg2': (8, 128, 51.2e-6), 'cfg5': (16, 256, 102.4e-6)}[os.environ.get('CFG', 'cfg2')]
F = int(os.environ.get('F', '200'))
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, A, C, TC, 0)[0]
ch.run(cube)
torch.cuda.synchronize()
ne, nc = ch.totals()
out = {}
for name, t in (('rds', ch.rds), ('mask', ch.mask), ('row_count', ch.row_count), ('entry_base', ch.offs['entry_base']),
                ('peak_pow', ch.peak_pow.view(-1)[:ne]), ('e_pdb', ch.lists['e_pdb'][:ne]),
                ('c_rc', ch.lists['c_rc'][:nc]), ('gidx', ch.gidx[:nc]), ('esprit', ch.ext['esprit'][:nc]),
                ('phase', ch.ext['phase'][:nc]), ('vel', ch.vel)):
    out[name] = hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()[:12]
print(json.dumps(out), flush=True)

"""k_offsets + k_frame_scan and the compaction (k_emit_cells + k_emit_block) standalone on one cfg2 batch
(development or product library via RSL_LIBRARY): min over 3 rounds of the mean of 20 launches, and a checksum of
every output (equal checksums across two libraries = identical offsets and lists).
GPU box:  RSL_LIBRARY=... python tools/offsets_time.py"""
import hashlib
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
ne, nc = ch.totals()
out = {}
for name, fn in (('offsets', lambda: ctx.offsets(ch.mask, ch.row_count, ch.C, bufs=ch.offs)), ('emit', ch._emit)):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(3):
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) / 20)
    out[name + '_ms'] = round(min(best), 4)
h = hashlib.sha256()
for k in ('entry_row_off', 'cell_row_off', 'entry_base', 'cell_base', 'frame_counts', 'union_mask'):
    h.update(ch.offs[k].cpu().numpy().tobytes())
for k, n in (('e_coord', ne), ('e_cell', ne), ('e_pdb', ne), ('c_frame', nc), ('c_rc', nc), ('c_amask', nc)):
    h.update(ch.lists[k][:n].cpu().numpy().tobytes())
out['sha'] = h.hexdigest()[:16]
print(json.dumps(out), flush=True)

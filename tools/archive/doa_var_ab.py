"""A/B of DoA kernel variants selected by environment settings (e.g. RSL_DOA_SKEW=1), each in its own process, on
one batch of F cfg2 frames: hipEvent average of the fused DoA + ESPRIT + phase launch (REPS launches) and a digest of
its outputs (grid index, ESPRIT, phase) to confirm they are unchanged.   python tools/doa_var_ab.py base RSL_DOA_SKEW=1"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
    import torch
    import rsl
    from bench import make_cubes
    F = int(os.environ.get('F', '2000'))
    ctx = rsl.get_context(0)
    cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
    ch = rsl.RadarChain(cfg, F, ctx)
    cube = make_cubes(ctx, 1, F, 8, 128, 51.2e-6, 0)[0]
    ch.run_front(cube)
    L = ch.lists

    ex = not os.environ.get('DOA_ARGMAX')  # DOA_ARGMAX=1: the argmax-only launch (where the RSL_DOA_DBG ablations apply)

    def go():
        ctx.doa_extras(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=ch.cell_cap, n_dev=ch.ncell_dev,
                       esprit_scale=ch.esprit_scale, out_idx=ch.gidx, esprit=ch.ext['esprit'] if ex else None,
                       phase=ch.ext['phase'] if ex else None)
    go()
    torch.cuda.synchronize()
    nc = int(ch.offs['cell_base'][F].item())
    h = hashlib.sha1()
    for t in (ch.gidx[:nc], ch.ext['esprit'][:nc], ch.ext['phase'][:nc]):
        h.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
    ctx.timing(True)
    ctx.timing_reset()
    for _ in range(int(os.environ.get('REPS', '5'))):
        go()
    torch.cuda.synchronize()
    t = ctx.timing_read()['doa_scan']
    ms = t[0] / max(t[1], 1)
    flops = 3 * 2 * 16 * 384 * nc
    print('RESULT', json.dumps({'doa_ms': ms, 'cells': nc, 'frac_f16': flops / (ms * 1e-3) / 2.5e15,
                                'digest': h.hexdigest()[:16]}), flush=True)


if __name__ == '__main__':
    if os.environ.get('DOA_CHILD'):
        child()
        sys.exit(0)
    for v in sys.argv[1:]:
        env = dict(os.environ, DOA_CHILD='1')
        for part in v.split('+'):
            if '=' in part:
                k, val = part.split('=', 1)
                env[k] = val
        r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith('RESULT')]
        print(v, line[0][7:] if line else ('FAILED rc=%d %s' % (r.returncode, r.stderr[-800:])), flush=True)

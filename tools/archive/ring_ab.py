"""A/B of the one-launch RDS path with the per-XCD L2 ring (RSL_RING=1, k_rds_ring) against the two-kernel path
(K1 + K2): each variant in its own process, F cfg2 frames; reports the stage time (hipEvents, REPS launches), a
digest of rds / mask / row_count and the ring fault word.   python tools/ring_ab.py two ring ring+R6+L3 ..."""
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

    def go():
        return ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                              row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)
    grp = go()
    torch.cuda.synchronize()
    h = hashlib.sha1()
    for t in (ch.rds[:64], ch.rds[-64:], ch.mask, ch.row_count):
        h.update(t.contiguous().view(torch.uint8).reshape(-1).cpu().numpy().tobytes())
    digest = h.hexdigest()[:16]
    ctx.timing(True)
    ctx.timing_reset()
    for _ in range(int(os.environ.get('REPS', '5'))):
        go()
    torch.cuda.synchronize()
    kt = ctx.timing_read()
    out = {k: v[0] / max(v[1], 1) for k, v in kt.items() if v[1]}
    out['stage_ms'] = out.get('range_fft', 0) + out.get('doppler_fft', 0)
    out['frac'] = 2 * 8 * 128 * 512 * 8 * F / (out['stage_ms'] * 1e-3) / 8e12
    out['digest'] = digest
    out['group'] = grp
    out['faults'] = int(ctx.lib.rsl_ring_faults(ctx.h))
    print('RESULT', json.dumps(out), flush=True)


if __name__ == '__main__':
    if os.environ.get('RING_CHILD'):
        child()
        sys.exit(0)
    for v in sys.argv[1:]:
        env = dict(os.environ, RING_CHILD='1')
        for part in v.split('+'):
            if part == 'two':
                env['RSL_RING'] = '0'
            elif part == 'ring':
                env['RSL_RING'] = '1'
            elif '=' in part:  # any other environment setting, e.g. RSL_DD_CP=42
                k, val = part.split('=', 1)
                env[k] = val
            else:
                key, val = part[0], part[1:]
                env[{'R': 'RSL_RING_R', 'L': 'RSL_RING_L', 'B': 'RSL_RING_BPC', 'F': 'F', 'O': 'RSL_RING_OWN', 'C': 'RSL_RING_CB', 'W': 'RSL_RING_WPE', 'Q': 'RSL_RING_Q', 'P': 'RSL_RING_PROF', 'T': 'RSL_RING_CT'}[key]] = val
        r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith('RESULT')]
        print(v, line[0][7:] if line else ('FAILED rc=%d %s' % (r.returncode, r.stderr[-800:])), flush=True)
        prof = [l for l in r.stdout.splitlines() if l.startswith('RINGPROF')]
        if prof:
            print('   ', prof[-1], flush=True)

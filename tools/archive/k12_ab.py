"""A/B of the one-pass RDS kernel variants (k_rds_class cache-policy bits RSL_FUSED_CP, RSL_FUSED=0 for the two-kernel
path): each variant in its own process, 2000 cfg2 frames, hipEvent averages of the two timed launches (K12 / K1 as
'range_fft', finish / K2 as 'doppler_fft') over REPS launches.   python tools/k12_ab.py CP1 CP2 ... [two]"""
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
        ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                       row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)
    go()
    torch.cuda.synchronize()
    ctx.timing(True)
    ctx.timing_reset()
    for _ in range(int(os.environ.get('REPS', '5'))):
        go()
    torch.cuda.synchronize()
    kt = ctx.timing_read()
    out = {k: v[0] / max(v[1], 1) for k, v in kt.items() if v[1]}
    out['stage_ms'] = out.get('range_fft', 0) + out.get('doppler_fft', 0)
    out['frac'] = 2 * 8 * 128 * 512 * 8 * F / (out['stage_ms'] * 1e-3) / 8e12
    print('RESULT', json.dumps(out), flush=True)


if __name__ == '__main__':
    if os.environ.get('K12_CHILD'):
        child()
        sys.exit(0)
    for v in sys.argv[1:]:
        env = dict(os.environ, K12_CHILD='1')
        parts = v.split('+')
        for part in parts:
            if part == 'two':
                env['RSL_FUSED'] = '0'
            else:
                key = part.rstrip('0123456789-').rstrip('m')
                val = part[len(key):].replace('m', '-')
                env[{'cp': 'RSL_FUSED_CP', 'bpc': 'RSL_FUSED_BPC', 'map': 'RSL_FUSED_MAP',
                     'skew': 'RSL_FUSED_SKEW'}[key]] = val
        r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith('RESULT')]
        print(v, line[0][7:] if line else ('FAILED rc=%d %s' % (r.returncode, r.stderr[-500:])), flush=True)

"""bench.py's host-side measurement pieces on CPU (no device): the CPU baseline's structure and arithmetic on a tiny
sample, the host-core detection, and the PMC traffic lookup (named kernels only, stale profiles give None)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_host_cores_reports_quota_or_affinity():
    import bench
    use, aff, quota = bench.host_cores()
    assert 1 <= use <= aff
    assert quota is None or use == max(1, min(aff, int(quota)))


def test_cpu_baseline_structure_small():
    import bench
    r = bench.cpu_baseline(procs=2, kmax=8, vec_frames=1, ridge=0.01)
    assert r['kind'] == 'port' and r['cores'] == 2 and r['unit'] == 'frames/s'
    st = r['seconds_per_frame_per_core']
    assert set(st) == {'range_doppler', 'peak_extraction', 'doa_music_esprit', 'velocity_ls', 'total'}
    assert abs(st['total'] - (st['range_doppler'] + st['peak_extraction'] + st['doa_music_esprit'] + st['velocity_ls'])) \
        < 1e-9 * st['total']
    assert r['value'] == pytest.approx(2 / st['total'])
    v = r['vectorised']
    assert v['cores'] == 2 and v['value'] == pytest.approx(2 / v['seconds_per_frame_per_core']['total'])
    assert 'first 8-8 of the frame' in r['sample']


def test_pmc_traffic_named_kernels(tmp_path, monkeypatch):
    import bench
    prof = {'frames_per_launch': 2000, 'kernels': {
        'rsl::k_range_fft_r512<true, 0>': {'hbm_bytes': 14.8e9},
        'rsl::k_doppler_detect_r128<16, 0>': {'hbm_bytes': 15.4e9}}}
    p = tmp_path / 'p.json'
    p.write_text(json.dumps(prof))
    monkeypatch.setattr(bench, 'PROFILE', str(p))
    assert bench.pmc_traffic('k_range_fft_r512', 1000) == pytest.approx(7.4e9)
    assert bench.pmc_traffic('k_doppler_detect_r128', 2000) == pytest.approx(15.4e9)
    assert bench.pmc_traffic('k_range_fft_p', 2000) is None  # a kernel the profile does not name: no bytes
    assert bench.pmc_traffic('k_range_fft_r512', 2000, config='cfg5') is None


def test_chain_rooflines_live_and_standalone():
    """The FFT-stage and DoA roofline objects carry the live fraction (hipEvent spans of the timed, pipelined steps)
    and the same stage's standalone fraction; the standalone ones follow from kernel_ms_standalone."""
    import bench
    A, C, S, F = 8, 128, 512, 2000
    kt = {'range_fft': (2.6 * 10, 10), 'doppler_fft': (2.8 * 10, 10), 'doa_scan': (5.7 * 10, 10), 'emit': (3.0, 10)}
    ks = {'range_fft': (2.45 * 6, 6), 'doppler_fft': (2.62 * 6, 6), 'doa_scan': (3.44 * 6, 6)}
    r = {'kt': kt, 'ks': ks, 'NS': 1, 'G': 361, 'nc': 71.9e6}
    out = bench.chain_rooflines(r, A, C, S, F, 'cfg2')
    alg = 2 * A * C * S * 8 * F
    assert abs(out['roofline']['frac'] - alg / (5.4e-3) / 1e9 / bench.HBM_PEAK_GBS) < 1e-9
    assert abs(out['roofline']['frac_standalone'] - alg / (5.07e-3) / 1e9 / bench.HBM_PEAK_GBS) < 1e-9
    assert out['roofline']['frac_standalone'] == out['fft_stage_standalone']['frac']
    flops = 3 * 2 * (2 * A - 1) * 71.9e6 * 361
    assert abs(out['roofline_doa']['frac'] - flops / 5.7e-3 / 1e12 / bench.F16_MFMA_PEAK_TFLOPS) < 1e-9
    assert abs(out['roofline_doa']['frac_standalone'] - flops / 3.44e-3 / 1e12 / bench.F16_MFMA_PEAK_TFLOPS) < 1e-9


def _bench(args, env_extra, timeout=120):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_world_size_mismatch_exits():
    """Under an external launcher whose WORLD_SIZE differs from --gpus the bench refuses to run (it would otherwise
    time WORLD_SIZE ranks and report them as --gpus): non-zero exit before any device work."""
    r = _bench(['--gpus', '8', '--steps', '1'], {'WORLD_SIZE': '1', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert r.returncode != 0 and 'WORLD_SIZE=1 but --gpus 8' in (r.stderr + r.stdout)
    r = _bench(['--gpus', '0'], {})
    assert r.returncode != 0


def test_gpus_n_spawns_ranks_and_fails_loudly():
    """`--gpus 2` with no launcher: the parent spawns two rank processes (RANK 0 / 1, WORLD_SIZE 2) and exits
    non-zero when they fail.  Here (no device visible) every rank stops at its device check, so the exit code and the
    rank's message show that the ranks were brought up and that a missing device is loud, never a 1-GPU run."""
    r = _bench(['--gpus', '2', '--steps', '1', '--no-cpu-baseline'], {})
    assert r.returncode != 0
    err = r.stderr
    assert 'needs device' in err and '--gpus 2' in err
    assert 'terminating the other ranks' in err or err.count('needs device') == 2
    assert not any(l.lstrip().startswith('{') for l in r.stdout.splitlines())


STUB = r'''
import json, os, sys, time
r = int(os.environ['RANK'])
mode = sys.argv[1]
if mode == 'fail' and r == 1:
    sys.exit(3)
if mode == 'hang' and r == 1:
    time.sleep(60)
if r == 0:
    print(json.dumps({k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE',
                                                  'MASTER_ADDR', 'MASTER_PORT')}), flush=True)
'''


@pytest.mark.parametrize('mode', ['ok', 'fail', 'hang'])
def test_launch_ranks_protocol(tmp_path, mode, capsys):
    """bench.launch_ranks with a stub rank program: every rank gets RANK / LOCAL_RANK / WORLD_SIZE /
    LOCAL_WORLD_SIZE / MASTER_ADDR = 127.0.0.1 / MASTER_PORT; rank 0's line is relayed; a failing rank's code is the
    launcher's; a rank still running past the grace period after another finished is ended with a non-zero code."""
    import bench
    stub = tmp_path / 'stub.py'
    stub.write_text(STUB)
    t0 = __import__('time').monotonic()
    rc = bench.launch_ranks(3, [mode], script=str(stub), grace=2.0)
    took = __import__('time').monotonic() - t0
    out = capsys.readouterr().out
    lines = [json.loads(l) for l in out.splitlines() if l.startswith('{')]
    if mode == 'ok':
        assert rc == 0 and len(lines) == 1
        e = lines[0]
        assert e['RANK'] == '0' and e['LOCAL_RANK'] == '0' and e['WORLD_SIZE'] == '3' and e['LOCAL_WORLD_SIZE'] == '3'
        assert e['MASTER_ADDR'] == '127.0.0.1' and int(e['MASTER_PORT']) > 0
    elif mode == 'fail':
        assert rc == 3
    else:
        assert rc != 0 and took < 30

"""bench.py --gpus N brings up N ranks itself: a rehearsal on the one-GPU box, two ranks on
device 0 (RSL_BENCH_DEVICE=0) over gloo, no external launcher.  The parent spawns the ranks, rank 0 prints one JSON
line with n_gpus 2, and value is the whole job's frames (2 ranks x F x steps) over the max-over-ranks time.  The
throughput itself is meaningless here (both ranks share one GPU; gloo stages the CUDA tensors through the host)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_spawns_two_ranks():
    F, steps = 200, 2
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(RSL_BENCH_DEVICE='0', RSL_BENCH_BACKEND='gloo')
    r = subprocess.run([sys.executable, '-u', os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--steps', str(steps),
                        '--warmup', '1', '--frames-per-step', str(F), '--no-extra', '--no-pcie', '--no-cpu-baseline'],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    js = [json.loads(l) for l in r.stdout.splitlines() if l.lstrip().startswith('{')]
    assert len(js) == 1, r.stdout[-2000:]
    line = js[0]
    assert line['n_gpus'] == 2 and line['steps'] == steps
    assert line['config']['parallelism'] == 'frame-sharded x2'
    elapsed = line['ms_per_step'] * steps / 1e3
    assert line['value'] == pytest.approx(2 * F * steps / elapsed, rel=1e-9)

"""Submit one gpurun call, waiting out the pool's transient refusals (backoff / no free box / slots busy) in which
NOTHING ran (status "transient", run_s 0): the same command is resubmitted only then, at most --tries times.  Any call
that ran on a box — whatever its outcome — ends this script with that outcome (no retry of a GPU step).
usage: python tools/gpurun_when_free.py --timeout 1500 --tries 8 -- 'bash tools/gpu_run.sh TAG steps...'"""
import argparse
import json
import re
import subprocess
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument('--timeout', type=int, default=1200)
ap.add_argument('--tries', type=int, default=8)
ap.add_argument('cmd', nargs=argparse.REMAINDER)
a = ap.parse_args()
cmd = ' '.join(a.cmd[1:] if a.cmd and a.cmd[0] == '--' else a.cmd)
for k in range(a.tries):
    p = subprocess.run(['/usr/local/graft/bin/gpurun', '--timeout', str(a.timeout), '--', cmd], capture_output=True,
                       text=True)
    out = p.stdout + p.stderr
    try:
        last = json.load(open('gpurun_out/.last_call.json'))
    except (OSError, ValueError):
        last = {}
    transient = last.get('status') == 'transient' and not last.get('run_s')
    print(f'[try {k + 1}] rc {p.returncode} status {last.get("status")} run_s {last.get("run_s")}', flush=True)
    if not transient and 'backing off' not in out:
        print(out[-4000:], flush=True)
        sys.exit(p.returncode)
    m = re.search(r'retry in (\d+)s', out)
    wait = int(m.group(1)) + 10 if m else 150
    print(f'  nothing ran ({out.strip().splitlines()[-2][:120] if len(out.strip().splitlines()) > 1 else out.strip()}); '
          f'waiting {wait} s', flush=True)
    time.sleep(wait)
print('gave up: the pool stayed unavailable', flush=True)
sys.exit(3)

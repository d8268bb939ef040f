"""Summarise bench.py JSON lines of an A/B session: frames/s and standalone per-kernel ms per log."""
import json
import sys

for path in sys.argv[1:]:
    line = None
    for l in open(path):
        if l.startswith('{'):
            line = json.loads(l)
    if line is None:
        print(path, 'no result')
        continue
    ks = line.get('kernel_ms_standalone', {})
    print(f"{path.split('/')[-1]:28s} {line['value'] / 1e3:7.1f} k frames/s  " +
          ' '.join(f"{k}={v:.3f}" for k, v in sorted(ks.items())))

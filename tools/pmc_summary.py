#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/: per-kernel average duration (kernel trace) and per-dispatch
HBM bytes (PMC passes), corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB) x 1024 x 2
(gfx950 tallies 128-B read requests at 64 B), WRITE_SIZE (KiB) x 1024.

    python tools/pmc_summary.py --stats DIR/trace_kernel_stats.csv --fetch DIR1 --write DIR2 \
        [--extra DIR3 ...] --out profiles/rN_pmc.json
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r'^void ', '', name)
    name = name.split('(')[0]
    return name


def counters(d):
    """Mean counter value per dispatch, per (kernel, counter)."""
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[short(row['Kernel_Name'])][row['Counter_Name']].append(float(row['Counter_Value']))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def stats(path):
    out = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            out[short(row['Name'])] = dict(calls=int(row['Calls']), avg_ms=float(row['AverageNs']) / 1e6,
                                           pct=float(row['Percentage']))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--stats')
    ap.add_argument('--fetch')
    ap.add_argument('--write')
    ap.add_argument('--extra', nargs='*', default=[])
    ap.add_argument('--out', required=True)
    ap.add_argument('--note', default='')
    ap.add_argument('--frames-per-launch', type=int, default=1000)
    a = ap.parse_args()
    res = {'note': a.note, 'frames_per_launch': a.frames_per_launch, 'kernels': {}}
    st = stats(a.stats) if a.stats else {}
    fe = counters(a.fetch) if a.fetch else {}
    wr = counters(a.write) if a.write else {}
    ex = {}
    for d in a.extra:
        for k, cs in counters(d).items():
            ex.setdefault(k, {}).update(cs)
    for k in sorted(set(st) | set(fe) | set(wr) | set(ex)):
        e = dict(st.get(k, {}))
        if k in fe and 'FETCH_SIZE' in fe[k]:
            e['hbm_read_bytes'] = fe[k]['FETCH_SIZE'] * 1024 * 2
        if k in wr and 'WRITE_SIZE' in wr[k]:
            e['hbm_write_bytes'] = wr[k]['WRITE_SIZE'] * 1024
        if 'hbm_read_bytes' in e or 'hbm_write_bytes' in e:
            e['hbm_bytes'] = e.get('hbm_read_bytes', 0) + e.get('hbm_write_bytes', 0)
        if k in ex:
            e['counters'] = ex[k]
        res['kernels'][k] = e
    os.makedirs(os.path.dirname(a.out) or '.', exist_ok=True)
    with open(a.out, 'w') as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k, e in sorted(res['kernels'].items(), key=lambda kv: -kv[1].get('pct', 0)):
        print(f"{k:60s} {e.get('avg_ms', 0):9.4f} ms  HBM {e.get('hbm_bytes', 0) / 1e6:10.1f} MB")


if __name__ == '__main__':
    main()

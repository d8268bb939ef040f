"""Live per-kernel time from the two sources of ONE profiled bench run: the rocprofv3 kernel trace
(begin / end of every dispatch) and the bench's own hipEvent spans (`live_timeline.spans_ms` in its JSON line, one
[start, end] per launch of each timing scope).  The trace's dispatches are grouped into the bench's scopes (range_fft =
K1, doppler_fft = K2, offsets = k_offsets + k_frame_scan, emit = k_emit_cells + k_emit_block, doa_scan = k_doa_toep +
k_doa_fixup, velocity = k_velocity), the timed steps are aligned on the first timed K1, and every scope launch is
compared: trace [first kernel begin, last kernel end] against the event span.
usage: python tools/trace_vs_events.py TRACE_kernel_trace.csv BENCH_LOG"""
import csv
import json
import sys

SCOPES = {'k_range_fft': 'range_fft', 'k_doppler_detect': 'doppler_fft', 'k_offsets': 'offsets', 'k_frame_scan': 'offsets',
          'k_emit_cells': 'emit', 'k_emit_block': 'emit', 'k_doa_toep': 'doa_scan', 'k_doa_fixup': 'doa_scan',
          'k_velocity': 'velocity'}
FIRST = {'offsets': 'k_offsets', 'emit': 'k_emit_cells', 'doa_scan': 'k_doa_toep'}
LAST = {'offsets': 'k_frame_scan', 'emit': 'k_emit_block', 'doa_scan': 'k_doa_fixup'}


def short(name):
    n = name.split('(')[0].replace('void ', '').replace('rsl::', '').split('<')[0]
    for k in SCOPES:  # k_range_fft_r512 / k_range_fft_p -> k_range_fft, k_doppler_detect_r128 -> k_doppler_detect
        if n.startswith(k):
            return k
    return n


def main(trace_csv, bench_log):
    line = json.loads([l for l in open(bench_log) if l.startswith('{')][0])
    ev = line['live_timeline']['spans_ms']
    rows = [r for r in csv.DictReader(open(trace_csv)) if 'rsl::' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    # scope launches in the trace: consecutive kernels of one scope on one queue
    launches = {k: [] for k in set(SCOPES.values())}
    open_ = {}
    for r in rows:
        n = short(r['Kernel_Name'])
        sc = SCOPES.get(n)
        if sc is None:
            continue
        s, e = int(r['Start_Timestamp']) * 1e-6, int(r['End_Timestamp']) * 1e-6
        first = FIRST.get(sc, n)
        if n == first:
            open_[sc] = [s, e]
            if LAST.get(sc, n) == n:
                launches[sc].append(open_.pop(sc))
        elif sc in open_:
            open_[sc][1] = e
            if LAST.get(sc) == n:
                launches[sc].append(open_.pop(sc))
    # align: the timed K1 launches are the trace's K1 launches whose gaps match the events' (the last len(ev) of the
    # pipelined ones before the standalone runs): search the offset with the smallest duration mismatch
    k1t = launches['range_fft']
    k1e = ev['range_fft']
    best = None
    for off in range(0, len(k1t) - len(k1e) + 1):
        mis = sum(abs((k1t[off + i][1] - k1t[off + i][0]) - (b - a)) for i, (a, b) in enumerate(k1e))
        if best is None or mis < best[0]:
            best = (mis, off)
    off = best[1]
    t_shift = k1t[off][0] - k1e[0][0]
    print(f'aligned on trace K1 launch {off} (of {len(k1t)}); {len(k1e)} timed steps')
    print(f'{"scope":12s} {"events ms":>10s} {"trace ms":>10s} {"diff %":>7s}   (median over the timed launches; '
          f'trace span = first kernel begin .. last kernel end)')
    out = {}
    for sc, spans in ev.items():
        if sc not in launches:
            continue
        tr = []
        for a, b in spans:  # the trace launch of this scope nearest in start time (shifted clock)
            cand = min(launches[sc], key=lambda x: abs(x[0] - t_shift - a)) if launches[sc] else None
            if cand:
                tr.append(cand[1] - cand[0])
        evd = sorted(b - a for a, b in spans)
        tr.sort()
        me, mt = evd[len(evd) // 2], tr[len(tr) // 2]
        out[sc] = {'events_ms': me, 'trace_ms': mt, 'diff_pct': 100 * (me - mt) / mt}
        print(f'{sc:12s} {me:10.3f} {mt:10.3f} {100 * (me - mt) / mt:7.1f}')
    return out


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])

#!/bin/bash
# A/B of the packed K1 -> K2 hand-off (default at S = 512, C = 128) against c64 rows, in one gpurun call:
# the product library vs the development library with RSL_WORK_C64=1 (same kernels otherwise).
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash tools/pack6_ab.sh
set -e
mkdir -p gpurun_out
for round in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/pack6_ab_pk_$round.log 2>&1
  RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so RSL_WORK_C64=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline \
    > gpurun_out/pack6_ab_c64_$round.log 2>&1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/pack6_ab_*.log')):
    line = [l for l in open(f) if l.startswith('{')][-1]
    d = json.loads(line)
    st = d['kernel_ms_standalone']
    print(f"{f}: {d['value']:.0f} frames/s  K1 {st['range_fft']:.3f}  K2 {st['doppler_fft']:.3f}  "
          f"stage frac {d['fft_stage_standalone']['frac']:.3f} (in step {d['roofline']['frac']:.3f})")
PY

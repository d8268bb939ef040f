set -o pipefail
mkdir -p gpurun_out
for m in none 128:128 160:96 144:112 176:80 256:128 192:192; do
  if [ "$m" = none ]; then unset RSL_BENCH_CUMASK; else export RSL_BENCH_CUMASK=$m; fi
  echo "== $m" >> gpurun_out/r2n_cumask.log
  timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 >> gpurun_out/r2n_cumask.log 2>&1 || exit 1
done

set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r2n_cfg5ab.log
for i in 1 2; do
  for L in new old; do
    echo "== $L" >> gpurun_out/r2n_cfg5ab.log
    if [ $L = old ]; then export RSL_LIBRARY=/root/repo/radar-slam_amd/lib/librsl_old.so; else unset RSL_LIBRARY; fi
    timeout -k 10 200 python -u bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/r2n_cfg5ab.log 2>&1 || exit 1
  done
done

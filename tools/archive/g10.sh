set -o pipefail
mkdir -p gpurun_out/ab10
for r in 1 2 3; do
for nt in 256 1024; do
for eb in 1 2; do
RSL_OFF_NT=$nt RSL_BENCH_EMIT_BACK=$eb timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/ab10/b_${nt}_${eb}_$r.log 2>&1 || exit 1
done; done; done

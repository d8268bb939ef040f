# offsets / compaction (emit) on the front stream (0) vs compaction (1, default) or both (2) on the back stream of the pipelined chain, alternating
set -e
for i in 1 2 3; do
  RSL_BENCH_EMIT_BACK=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/eab_a_$i.json 2>/dev/null
  RSL_BENCH_EMIT_BACK=1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/eab_b_$i.json 2>/dev/null
  RSL_BENCH_EMIT_BACK=2 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/eab_c_$i.json 2>/dev/null
done

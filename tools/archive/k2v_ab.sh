# K2 launch variants re-measured in the current pipelined chain: default vs dispatch-order tiles (RSL_DD_XCD=0) vs
# 27 KiB LDS per workgroup (RSL_DD_LDS=27648: 5 per CU, room for a co-running DoA / compaction workgroup), alternating
set -e
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/k2v_a_$i.json 2>/dev/null
  RSL_DD_XCD=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/k2v_b_$i.json 2>/dev/null
  RSL_DD_LDS=27648 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/k2v_c_$i.json 2>/dev/null
done

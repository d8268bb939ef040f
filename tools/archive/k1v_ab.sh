# K1 variants re-measured with the per-XCD dequeue (default vs 16-row tiles vs 2 workgroups per CU), alternating
set -e
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/k1v_a_$i.json 2>/dev/null
  RSL_RF_CB=16 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/k1v_b_$i.json 2>/dev/null
  RSL_RF_BPC=2 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/k1v_c_$i.json 2>/dev/null
done

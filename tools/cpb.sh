# End-to-end bench A/B: pipelined (default) vs one stream, with K1 variants that only pay off without co-residency
set -e
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/cpb_a_$i.json 2>/dev/null
  timeout -k 10 200 python bench.py --no-cpu-baseline --pipeline 0 > gpurun_out/cpb_b_$i.json 2>/dev/null
  RSL_RF_CB=16 timeout -k 10 200 python bench.py --no-cpu-baseline --pipeline 0 > gpurun_out/cpb_c_$i.json 2>/dev/null
  RSL_RF_PD=2 timeout -k 10 200 python bench.py --no-cpu-baseline --pipeline 0 > gpurun_out/cpb_d_$i.json 2>/dev/null
done

# End-to-end bench A/B of cache-policy knobs (RSL_RF_CP / RSL_DD_CP / RSL_EMIT_NT; tools/cp_ab.py has the RDS kernels alone)
set -e
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/cpb_a_$i.json 2>/dev/null
  RSL_EMIT_NT=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/cpb_b_$i.json 2>/dev/null
done

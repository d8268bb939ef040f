# K1 dequeue A/B: kernel alone (tools/dyn_ab.py), then the bench with and without it, alternating
set -e
timeout -k 10 200 python tools/dyn_ab.py > gpurun_out/dyn_ab.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/dyn_a_$i.json 2>/dev/null
  RSL_RF_DYN=1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/dyn_b_$i.json 2>/dev/null
done

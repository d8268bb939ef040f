# K2 store A/B: kernel alone (tools/pk_ab.py), then the bench default vs RSL_DD_CP=$B_CP, alternating
set -e
timeout -k 10 200 python tools/pk_ab.py > gpurun_out/pk_ab.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/pkb_a_$i.json 2>/dev/null
  RSL_DD_CP=${B_CP:-10} timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/pkb_b_$i.json 2>/dev/null
done

# End-to-end bench A/B (edit the variants; tools/cp_ab.py / rf_pd.py time the kernels alone)
set -e
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config cfg5 --steps 10 > gpurun_out/cpb_a_$i.json 2>/dev/null
  RSL_DD_KB=16 timeout -k 10 200 python bench.py --no-cpu-baseline --config cfg5 --steps 10 > gpurun_out/cpb_b_$i.json 2>/dev/null
done

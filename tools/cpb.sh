# End-to-end bench A/B (edit the variants; tools/cp_ab.py / rf_pd.py time the kernels alone)
set -e
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/cpb_a_$i.json 2>/dev/null
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --frames-per-step 2000 > gpurun_out/cpb_b_$i.json 2>/dev/null
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --frames-per-step 500 > gpurun_out/cpb_c_$i.json 2>/dev/null
done

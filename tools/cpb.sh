# End-to-end bench runs (edit the variants; tools/cp_ab.py / rf_pd.py time the kernels alone)
set -e
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/cpb_a_$i.json 2>/dev/null
done

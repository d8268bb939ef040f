# End-to-end bench A/B (edit the variants; tools/cp_ab.py / rf_pd.py time the kernels alone)
set -e
L=radar-slam_amd/lib
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/cpb_a_$i.json 2>/dev/null
  RSL_LIBRARY=$PWD/$L/librsl_max-memory-clause.so timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/cpb_b_$i.json 2>/dev/null
  RSL_LIBRARY=$PWD/$L/librsl_max-ilp.so timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/cpb_c_$i.json 2>/dev/null
done

# c64 `work` rows (default) vs packed 6-B rows (RSL_WORK_PACK=1) between K1 and K2, alternating, in one call:
#   gpurun -- 'bash tools/pack_ab.sh'   (then read gpurun_out/pack_{a,b}_*.json: value, kernel_ms_per_step, fft_stage_standalone)
set -e
mkdir -p gpurun_out
for i in 1 2; do
  RSL_WORK_PACK=0 timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/pack_a_$i.json 2>/dev/null
  RSL_WORK_PACK=1 timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/pack_b_$i.json 2>/dev/null
done

# A/B against a build of the previous commit checked out in _abtree/ (git worktree): K2 alone, then the bench
set -e
for i in 1 2; do
  RSL_DD_ONLY0=1 timeout -k 10 200 python tools/dd_ablation.py > gpurun_out/dd_a_$i.log 2>/dev/null
  (cd _abtree && timeout -k 10 200 python tools/dd_ablation.py > ../gpurun_out/dd_b_$i.log 2>/dev/null)
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/cpb_a_$i.json 2>/dev/null
  (cd _abtree && timeout -k 10 200 python bench.py --no-cpu-baseline > ../gpurun_out/cpb_b_$i.json 2>/dev/null)
done

# End-to-end bench A/B against a build of the previous commit checked out in _abtree/ (git worktree)
set -e
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/cpb_a_$i.json 2>/dev/null
  (cd _abtree && timeout -k 10 200 python bench.py --no-cpu-baseline > ../gpurun_out/cpb_b_$i.json 2>/dev/null)
done

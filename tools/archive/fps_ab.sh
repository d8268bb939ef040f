# frames-per-step A/B (2000 default vs 3000 / 4000), alternating in one call
set -e
for i in 1 2; do
  for f in 2000 3000 4000; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --frames-per-step $f > gpurun_out/fps_${f}_$i.json 2>/dev/null
  done
done

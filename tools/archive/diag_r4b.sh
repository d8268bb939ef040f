set -u
mkdir -p gpurun_out/diag
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 90 python -u tools/pipelined_repeat.py 2 noguard > gpurun_out/diag/ng_$i.log 2>&1 || { echo "noguard $i rc $?"; break; }
done
for i in 1 2 3 4; do
  timeout -k 10 90 python -u tools/pipelined_repeat.py 2 > gpurun_out/diag/g_$i.log 2>&1 || { echo "guard $i rc $?"; break; }
done
grep -h "mismatching" gpurun_out/diag/*.log
F=1000 REPS=3 bash tools/doa_counters.sh && echo counters ok
timeout -k 10 300 python -u -m pytest tests/test_gpu_traj_dist.py tests/test_gpu_wrapped.py tests/test_gpu_pipelined.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/t_r4b.log 2>&1; echo pytest rc $?

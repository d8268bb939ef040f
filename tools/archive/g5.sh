set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipelined.py tests/test_gpu_edges.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2e_test.log 2>&1 || exit 1
for r in 1 2; do
for nt in 256 1024; do
RSL_OFF_NT=$nt timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r2e_b${nt}_$r.log 2>&1 || exit 1
done; done

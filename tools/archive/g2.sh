set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_traj.py tests/test_gpu_chain.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2b_gputest.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r2b_bench.log 2>&1

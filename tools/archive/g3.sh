set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2c_chain.log 2>&1 ; \
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r2c_bench_fused.log 2>&1 && \
RSL_FUSED=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r2c_bench_two.log 2>&1

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectrum.py tests/test_gpu_dropin.py tests/test_gpu_chain.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2h_test.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config spectrum --steps 5 --warmup 1 > gpurun_out/r2h_spec_bench.log 2>&1

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2l_gputest.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/r2l_bench.log 2>&1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r2l_bench2.log 2>&1

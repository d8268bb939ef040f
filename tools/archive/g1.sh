set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2a_gputest.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2a_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --cpu-budget 5 > gpurun_out/r2a_bench.log 2>&1

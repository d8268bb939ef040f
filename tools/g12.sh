set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_spectrum.py -s > gpurun_out/r2l_spectest.log 2>&1
timeout -k 10 600 python -u bench.py --config spectrum --no-cpu-baseline > gpurun_out/r2l_spec_bench.log 2>&1

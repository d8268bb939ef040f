set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectrum.py tests/test_gpu_dropin.py -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r2g_spec.log 2>&1

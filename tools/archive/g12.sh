set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_spectrum.py -s > gpurun_out/r2m_spectest.log 2>&1

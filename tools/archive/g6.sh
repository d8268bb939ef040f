set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_traj.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2f_eval.log 2>&1

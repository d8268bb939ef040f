set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 env RSL_RING_CT=2 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/r2j_ringtest.log 2>&1
timeout -k 10 700 python -u tools/ring_ab.py two ring+R6+L5+P1 ring+R6+L5+T2+P1 ring+R6+L5+T4+P1 ring+R4+L3+T2+P1 ring+R8+L7+T2+P1 > gpurun_out/r2j_ring6.log 2>&1

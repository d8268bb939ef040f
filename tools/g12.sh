set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ring_ab.py two two+RSL_DD_PERSIST=1 two+RSL_DD_PERSIST=1+RSL_DD_PWPE=6 two two+RSL_DD_PERSIST=1 two+RSL_DD_PERSIST=1+RSL_DD_PWPE=6 > gpurun_out/r2k_k2p.log 2>&1
RSL_DD_PERSIST=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_pipelined.py > gpurun_out/r2k_k2ptest.log 2>&1

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/ring_ab.py two two+RSL_DD_CP=75 two+RSL_DD_CP=79 two+RSL_DD_CP=90 two two+RSL_DD_CP=75 two+RSL_DD_CP=79 two+RSL_DD_CP=90 > gpurun_out/r2l_k2cp.log 2>&1

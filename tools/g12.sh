set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/doa_var_ab.py DOA_ARGMAX=1 DOA_ARGMAX=1+RSL_DOA_SKEW=0 DOA_ARGMAX=1 DOA_ARGMAX=1+RSL_DOA_SKEW=0 > gpurun_out/r2l_doa4.log 2>&1

#!/bin/bash
# SQ counter passes over any command: tools/counters.sh TAG -- python3 script.py args
set -euo pipefail
TAG=$1; shift; shift
OUT=gpurun_out/ctr_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o p -- "$@" > $OUT/p1.log 2>&1
timeout -k 10 180 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT/p2 -o p -- "$@" > $OUT/p2.log 2>&1
timeout -k 10 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/p3 -o p -- "$@" > $OUT/p3.log 2>&1 || true
python3 tools/pmc_summary.py --extra $OUT/p1 $OUT/p2 $OUT/p3 --out $OUT/summary.json > /dev/null

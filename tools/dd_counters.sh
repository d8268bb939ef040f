#!/bin/bash
# SQ counter passes over the RDS kernels alone (tools/dd_only.py: K1 + K2), for bottleneck analysis.
set -euo pipefail
OUT=${OUT:-gpurun_out/dd_ctr}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P="python3 tools/dd_only.py"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o p -- $P > $OUT/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $OUT/p2 -o p -- $P > $OUT/p2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d $OUT/p3 -o p -- $P > $OUT/p3.log 2>&1 || true
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p4 -o p -- $P > $OUT/p4.log 2>&1 || true
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p5 -o p -- $P > $OUT/p5.log 2>&1 || true
python3 tools/pmc_summary.py --extra $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 $OUT/p5 --out $OUT/summary.json

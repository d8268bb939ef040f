#!/bin/bash
# SQ counter passes over every kernel of the batched chain (tools/chain_only.py), for bottleneck analysis.
set -euo pipefail
OUT=gpurun_out/chain_ctr
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P="python3 tools/chain_only.py"
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o t -- $P > $OUT/t.log 2>&1
timeout -k 10 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o p -- $P > $OUT/p1.log 2>&1
timeout -k 10 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/p2 -o p -- $P > $OUT/p2.log 2>&1
timeout -k 10 150 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA FETCH_SIZE --output-format csv -d $OUT/p3 -o p -- $P > $OUT/p3.log 2>&1
timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p4 -o p -- $P > $OUT/p4.log 2>&1
STATS=$(find "$OUT/t" -name '*kernel_stats.csv' | head -1)
python3 tools/pmc_summary.py --stats "$STATS" --fetch $OUT/p3 --write $OUT/p4 --extra $OUT/p1 $OUT/p2 $OUT/p3 --out $OUT/summary.json --frames-per-launch 1000

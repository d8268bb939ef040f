#!/bin/bash
# K12 (range-class one-pass kernel) counter passes on a 2000-frame cfg2 batch: HBM bytes, L2 hits, SQ issue/wait.
set -uo pipefail
TAG=${1:-k12}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export F=2000 REPS=3
CMD="python3 tools/dd_only.py"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o t -- $CMD > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- $CMD > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- $CMD > $OUT/write.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/l2 -o p -- $CMD > $OUT/l2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o p -- $CMD > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT/p2 -o p -- $CMD > $OUT/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/p3 -o p -- $CMD > $OUT/p3.log 2>&1 || exit 1
STATS=$(find $OUT/trace -name '*kernel_stats.csv' | head -1)
python3 tools/pmc_summary.py --stats "$STATS" --fetch $OUT/fetch --write $OUT/write --extra $OUT/l2 $OUT/p1 $OUT/p2 $OUT/p3 --out $OUT/summary.json --frames-per-launch 2000

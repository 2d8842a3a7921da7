#!/bin/bash
# Where the encoder kernels' wave cycles go (stall counters, one pass), on the bench's embed step.
set -o pipefail
OUT=gpurun_out/r5i
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$ROOT/$OUT/stall_enc" -o run -- python3 bench.py \
  --mode embed --steps 2 --warmup 1 > $OUT/stall_enc.out 2> $OUT/stall_enc.err || { tail -20 $OUT/stall_enc.err; exit 1; }
f=$(find $OUT/stall_enc -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_stalls.py "$f" > $OUT/stall_enc.md || exit 1
cat $OUT/stall_enc.md
gzip -f "$f"

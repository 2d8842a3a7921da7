#!/bin/bash
# list the profiler's counters on gfx950 (translation / TLB / EA ones)
set -o pipefail
OUT=gpurun_out/r5lc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || { tail -20 $OUT/counters.txt; exit 1; }
grep -i -E "utcl|tlb|translation|TCC_EA0_RDREQ|TCC_EA0_WRREQ|TCC_HIT|TCC_MISS|TA_BUSY|TCP_PENDING|TCC_REQ" $OUT/counters.txt | sort -u | head -80

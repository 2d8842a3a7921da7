#!/bin/bash
# kernel time split of the bench's search phase (256 i.i.d. queries over 25 M x 768 through spl_search_batch)
set -o pipefail
OUT=gpurun_out/r6s36
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/prof -o run -- python3 bench.py --mode embed --steps 2 --warmup 1 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0 > $OUT/b.out 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>5} total {float(r["TotalDurationNs"])/1e6:8.2f} ms avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
grep -o '"search_qps": [0-9.]*' $OUT/b.out
find $OUT/prof -name '*kernel_trace.csv' -delete

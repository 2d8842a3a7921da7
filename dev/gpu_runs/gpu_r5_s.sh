#!/bin/bash
# exchange rehearsal with each rank on its own half of every XCD (--rank-cus 16) vs time-sliced ranks
set -o pipefail
OUT=gpurun_out/r5s
mkdir -p $OUT
C="--mode kv --steps 10 --warmup 3 --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --mixed5 0 --verify 5000 --value-len 150 --mop 1"
run2() {  # tag extra-args
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) \
    bench.py --gpus 2 --keys-per-gpu 20000000 --batch 4000000 $C --backend gloo --transport peer "${@:2}" > $OUT/$1.out 2> $OUT/$1.err || { tail -20 $OUT/$1.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$1.out') if l.startswith('{')][-1]); print('$1', d['value'], d['ms_per_step'], d['integrity_failures'])"
}
timeout -k 10 600 python bench.py --gpus 1 --keys-per-gpu 40000000 --batch 8000000 $C > $OUT/one.out 2> $OUT/one.err || { tail -20 $OUT/one.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$OUT/one.out') if l.startswith('{')][-1]); print('one', d['value'], d['ms_per_step'], d['integrity_failures'])"
run2 two_part --rank-cus 16
run2 two_shared
run2 two_part2 --rank-cus 16

# round 2, call 46: RCCL all_to_all_single past 768 MiB -- bytes vs elements, bisection, list / explicit-split forms, chunked fix, gloo
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_46
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 scripts/a2a_rootcause.py > $O/a2a.jsonl 2> $O/a2a.err &&
echo done

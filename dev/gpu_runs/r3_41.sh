# round 3, call 41: residual+LN kernel per-tile fixed cost (time vs K at M 32768) and the new ring defaults at
# 16 / 32 threads (alternating with the old ones)
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_41
mkdir -p $O
timeout -k 10 300 python -u scripts/residual_gemm_ab.py --no-blas --rln-variants 222 --ks 128,256,512,768,1536,3072 > $O/rln_k.jsonl 2> $O/rln_k.err || exit 1
H=libsplinter_amd/bin/splinter_hostapi_bench
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 60 $H --seconds 1.5 --keys 20000 "$@" 2>> $O/h.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/h.jsonl; }
for r in 1 2 3 4; do
run new32 X=1 --threads 32 || exit 1
run old32 SPLINTER_RING_OVERSUB_SPIN_US=2 SPLINTER_RING_FIRST_SLEEP_NS=5000 --threads 32 || exit 1
done
run new16 X=1 --threads 16 || exit 1
run new24 X=1 --threads 24 || exit 1
run new1 X=1 --threads 1 || exit 1
echo done

# round 3, call 11: host-API ring thread sweep (oversubscription policy A/B); rocprofv3 kernel trace of the TIMED steps only (roctx pause/resume, SPL_PROFILE_TIMED)
# of bench.py embed mode and the default mixed step; PMC counters of the encoder kernels
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_11
mkdir -p $O
H=libsplinter_amd/bin/splinter_hostapi_bench
cat /sys/fs/cgroup/cpu.max > $O/cpu_max.txt 2>&1 || true
nproc > $O/nproc.txt
for t in 1 8 16 24 32; do timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 >> $O/hostapi_default.jsonl 2>> $O/hostapi.err || exit 1; done
for t in 16 32; do SPLINTER_RING_CPUS=1000 timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 >> $O/hostapi_nooversub.jsonl 2>> $O/hostapi.err || exit 1; done
for t in 16 32; do SPLINTER_RING_CPUS=8 timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 >> $O/hostapi_cpus8.jsonl 2>> $O/hostapi.err || exit 1; done
B="--mode embed --host-api 0 --host-api-threads2 0 --embed-e2e 0 --steps 4 --warmup 2 --keys-per-gpu 1000000 --search-keys 0"
export SPL_PROFILE_TIMED=1
timeout -s KILL 300 rocprofv3 --selected-regions --kernel-trace --stats --output-format csv -d $O/trace_embed -o embed -- python3 bench.py $B > $O/trace_embed.log 2>&1 &&
timeout -s KILL 600 rocprofv3 --selected-regions --kernel-trace --stats --output-format csv -d $O/trace_mixed -o mixed -- python3 bench.py --steps 5 --warmup 3 --host-api 0 --host-api-threads2 0 --embed-e2e 0 --routed-steps 0 --search-batches 2 > $O/trace_mixed.log 2>&1 &&
unset SPL_PROFILE_TIMED &&
P="rocprofv3 --kernel-trace --output-format csv" &&
timeout -s KILL 240 $P --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o enc_mfma -- python3 bench.py $B > $O/enc_mfma.log 2>&1 &&
timeout -s KILL 240 $P --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/pmc -o enc_l2 -- python3 bench.py $B > $O/enc_l2.log 2>&1 &&
echo done

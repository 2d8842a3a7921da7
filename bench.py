#!/usr/bin/env python3
"""Headline benchmark: KV set/get ops/s on the HBM arena (+ Nomic embed vectors/s).

Metric (BASELINE.json): "KV set/get ops/sec + Nomic-768d embed vectors/sec at
1/2/4/8 MI355X".  One process per GPU (torchrun); each rank owns one
hash-shard of the key space in its own HBM arena (format v4, 128-B slots,
256-B values) prepopulated with --keys-per-gpu keys.  A timed step is:

  * KV phase: a batch of --batch client ops per rank (half set, half get,
    uniformly random keys over the whole node's key space) issued as a set
    batch and a get batch on two concurrent HIP streams, so readers race
    writers on the seqlocks (the reference's MRSW/MRMW regime,
    /root/reference/splinter_stress.c, splinter_chi_sao.c).  With N>1 every
    batch is routed to the owning shards and the results are routed back
    (collective C1) inside the timed region: one request and one
    response exchange per step (parallel/xroute.py), own-shard ops in place,
    remote records stored straight into the owners' peer-mapped HBM windows
    over xGMI (--transport peer; rccl = one all-to-all per direction).
  * embed phase (--mode mixed/embed): one batch of synthetic documents through
    the random-init Nomic-BERT encoder on the gfx950 kernels, mean-pooled
    vectors written into their slots of the rank's search arena (--search-keys
    embedded keys per GPU: the config #5 corpus; the 100M-key KV arena has no
    vector slots -- 100M x 3 KiB of vectors would exceed the 288 GB of HBM -- so
    the vectors land in the 25M-key embedding arena beside it, through the same
    seqlocked slot write, in the same step as the KV phase).

The client streams are the same at every N: at N=1 the set / get batches fan out over
--writer-streams / --reader-streams HIP streams; at N>1 the owner fans its own ops and the
request blocks it received out over the same streams (spl_kvs_step_xr).  Outside the timed region:
the routed step at N=1 (routed_kv_ops_per_s), end-to-end embedding, the embedding daemon's
own code path per rank (daemon_vectors_per_s), the per-call C API, and config #5's query phase (batched top-k over the search arenas, broadcast + all-gather
merge at N>1, recall against the exact kernel).

Ops counted exactly as the reference does (every set + get attempt that
completes, splinter_stress.c:212-213); EAGAIN retries are reported separately.
Weak scaling: per-GPU work is fixed as N grows; `value` is the node total.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REF_MRMW_OPS = 15.6e6  # reference MRMW headline (README.md:131), BASELINE.md


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--mode", default="mixed", choices=["kv", "embed", "mixed"])
    p.add_argument("--keys-per-gpu", type=int, default=100_000_000)
    p.add_argument("--slots-factor", type=float, default=2.0)
    p.add_argument("--max-val", type=int, default=256)
    p.add_argument("--value-len", type=int, default=150)
    p.add_argument("--batch", type=int, default=16_000_000, help="client ops per rank per step")
    p.add_argument("--set-frac", type=float, default=0.5)
    p.add_argument("--embed-batch", type=int, default=64, help="documents per rank per step")
    p.add_argument("--embed-seq", type=int, default=512)
    p.add_argument("--verify", type=int, default=20000)
    p.add_argument("--kv-cus", type=int, default=0,
                   help="N>0: overlap the KV and embed phases with the KV streams confined to N CUs per XCD "
                        "and the encoder to the rest (hipExtStreamCreateWithCUMask); 0 = phases back to back")
    p.add_argument("--overlap", action="store_true",
                   help="run the embed batch concurrently with the KV batches (own stream, all CUs)")
    p.add_argument("--overlap-native", type=int, default=0, choices=[0, 1],
                   help="1: the native KV fan-out (32+32 client streams) runs concurrently with the embed batch "
                        "(KV forked from its own origin stream, the encoder on the current stream)")
    p.add_argument("--overlap-kv-cus", type=int, default=0, choices=[0, 8, 16, 24],
                   help="with --overlap-native 1: the KV origin stream is confined to N CUs per XCD (CU mask; the "
                        "fused grid is sized to them) while the encoder keeps every CU, so encoder kernels fill "
                        "the other CUs while the KV grid runs and the whole chip once it ends")
    p.add_argument("--force-routed", action="store_true",
                   help="run the N>1 routed step (pack -> all-to-all -> owner kernels -> all-to-all -> gather) "
                        "even at N=1, to measure the routing overhead on one GPU")
    p.add_argument("--transport", default="peer", choices=["peer", "rccl"],
                   help="N>1 routed exchange: peer = request / response rows stored straight into the owners' "
                        "peer-mapped windows (xGMI), falling back to rccl if any mapping fails; rccl = one "
                        "all-to-all per direction")
    p.add_argument("--backend", default="nccl", help="nccl (= RCCL, one GPU per rank) or gloo (rehearsal: "
                   "ranks may share a GPU, collectives staged through the host)")
    p.add_argument("--writer-streams", type=int, default=32,
                   help="concurrent HIP streams issuing the step's set batch (BASELINE config #2: 32 writer "
                        "streams); each gets an equal share of the batch")
    p.add_argument("--reader-streams", type=int, default=32, help="concurrent HIP streams issuing the get batch")
    p.add_argument("--mop", type=int, default=1, choices=[0, 1, 2],
                   help="store scrub mode (splinter_set_mop): 1 = hybrid, the default of every store the "
                        "reference creates (reference splinter.c:192-193) and of its stress tools; 0 = none")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher check without a GPU: every rank joins a gloo group, rank 0 prints the world "
                        "it sees as JSON and the run ends (tests/test_bench_cpu.py)")
    p.add_argument("--throttle", type=int, default=1, choices=[0, 1],
                   help="1: issue a step's KV launches only after the previous step's encoder finished")
    p.add_argument("--embed-e2e", type=int, default=20, metavar="STEPS",
                   help="after the timed loop, time STEPS end-to-end embedding batches of the splinference path "
                        "(text fetch, WordPiece, varlen batch, slot find, encoder + seqlocked write, labels); 0: off")
    p.add_argument("--host-api", type=int, default=16, metavar="THREADS",
                   help="also measure the per-call C API (splinter_set/get through the device command ring) "
                        "from THREADS host threads, outside the timed region; 0 = skip")
    p.add_argument("--host-api-threads2", type=int, default=32, metavar="THREADS",
                   help="a second per-call C API row at this many host threads (0 = skip)")
    p.add_argument("--search-keys", type=int, default=25_000_000,
                   help="embedded keys per GPU in the search arena (config #5: 200M x 768 over 8 GPUs); the embed "
                        "phase writes its vectors into this arena; 0 = a small side arena, no query phase")
    p.add_argument("--search-queries", type=int, default=256, help="queries per search batch (query phase)")
    p.add_argument("--search-batches", type=int, default=8, help="timed search batches (query phase)")
    p.add_argument("--daemon-docs", type=int, default=512,
                   help="after the timed loop, embed this many pending VARTEXT documents of an hbm: store through "
                        "the splinference daemon's own code path (Splinference.process: batched read, WordPiece, "
                        "encoder, vectors pooled into the slots, +2 epoch check, label updates), per rank; 0 = skip")
    p.add_argument("--exchange-ab", type=int, default=1, choices=[0, 1],
                   help="N=1: after everything else, time the routed exchange honestly in FRESH child processes on "
                        "this GPU: a 2-rank run (both ranks on this device, peer-window transport, gloo for the small "
                        "collectives) and a 1-rank run at identical totals (--exchange-keys keys, --exchange-batch ops "
                        "per step in all) -> exchange_2rank_ops_per_s / exchange_1rank_ops_per_s / exchange_ratio")
    p.add_argument("--exchange-keys", type=int, default=40_000_000, help="total keys of the exchange A/B runs")
    p.add_argument("--exchange-batch", type=int, default=8_000_000, help="total ops per step of the exchange A/B runs")
    p.add_argument("--kv-async-ab", type=int, default=1, choices=[0, 1],
                   help="N=1: config #2's literal form in the record -- KV-only steps with the 32 writer + 32 "
                        "reader client streams each posting its own slice to the resident server grid "
                        "(SPL_KVS_FUSED=3), beside the fused grid, both in fresh child processes")
    p.add_argument("--mixed5", type=int, default=10, metavar="STEPS",
                   help="after the timed loop, time STEPS config-#5 mixed steps (embed a batch -> its vectors "
                        "inserted into the search arena's slots -> a batched top-10 query of --search-queries "
                        "queries over the whole arena, built from the vectors just written); 0 = skip")
    return p.parse_args()


def _launch_ranks(args) -> int:
    """--gpus N > 1 without a torchrun environment: start N ranks as CHILD processes (torchrun,
    one process per GPU, rendezvous on 127.0.0.1) before this process touches the GPU, relay
    their output and exit with their status.  Never exec: this process stays the parent."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def _timed_region_profiler():
    """SPL_PROFILE_TIMED=1: roctxProfilerResume/Pause around the timed steps (for
    `rocprofv3 --selected-regions`), and the region's bounds printed to stderr in the monotonic and
    boot-time clocks, so a full `rocprofv3 --kernel-trace` can be cut to exactly the timed steps
    (scripts/trace_window.py): which kernels run in the measured step, nothing from setup or warm-up."""
    if os.environ.get("SPL_PROFILE_TIMED") != "1":
        return lambda on: None
    import ctypes
    lib = ctypes.CDLL("librocprofiler-sdk-roctx.so.1")
    lib.roctxProfilerResume.argtypes = lib.roctxProfilerPause.argtypes = [ctypes.c_uint64]

    def toggle(on):
        import torch
        torch.cuda.synchronize()
        (lib.roctxProfilerResume if on else lib.roctxProfilerPause)(0)
        # the region's bounds in both host clocks a kernel trace may be stamped in, so a full trace
        # can be cut to the timed steps afterwards (scripts/trace_window.py)
        print(json.dumps({"timed_region": "begin" if on else "end", "monotonic_ns": time.monotonic_ns(),
                          "boottime_ns": time.clock_gettime_ns(time.CLOCK_BOOTTIME)}), file=sys.stderr, flush=True)
    return toggle


def daemon_run(enc, docs: int, seq: int, rank: int, world: int, routed: bool, node: str, rounds: int = 3):
    """Time Splinference.process over `docs` pending documents of this rank's shard of node store
    `node` (the daemon's owner-computes path: each rank embeds its own shard, reference
    splinference.cpp:500-552), `rounds` times after one warm-up round; the producer re-sets every
    document's text between rounds (outside the timing) so each round finds them all pending."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from libsplinter_amd.daemons.splinference import EMBED_LABEL, WAITING_LABEL, Splinference
    from libsplinter_amd.models.tokenizer import WordPieceTokenizer, synthetic_vocab
    from libsplinter_amd.store import SLOT_VARTEXT, Store, unlink
    vocab = synthetic_vocab(enc.cfg.vocab)
    tok = WordPieceTokenizer(vocab)
    words = [t[1:] for t in vocab if t.startswith("▁") and len(t) > 2]
    rng = np.random.default_rng(300 + rank)
    texts = [" ".join(words[int(i)] for i in rng.integers(0, len(words), size=int(rng.integers(seq // 2, seq - 2))))
             for _ in range(docs)]
    from libsplinter_amd.store import NODE_HBM, node_join, node_leave, node_shard_name
    name = node_shard_name(node, rank, NODE_HBM)
    st = Store.create(name, slots=max(4 * docs, 1024), max_val=4096, embeddings=True)
    node_join(node, rank, world, NODE_HBM, st.slots, 4096, True)
    keys = [f"doc{rank}_{i:06d}" for i in range(docs)]

    def produce():
        for k, t in zip(keys, texts):
            st.set(k, t.encode())
            st.set_type(k, SLOT_VARTEXT)
            st.set_label(k, EMBED_LABEL | WAITING_LABEL)

    try:
        d = Splinference(st, enc, tok, group=3, batch_tokens=64 * seq)
        produce()
        d.process(d.pending())  # warm-up: first varlen shapes
        times, done = [], 0
        for _ in range(rounds):
            produce()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            done += d.process(d.pending())
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        dt = torch.tensor([sum(times)], dtype=torch.float64, device="cuda")
        if routed:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return {"vectors_per_s": docs * rounds * world / dt.item(), "embedded": done, "expected": docs * rounds,
                "stale": d.stats["stale"]}
    finally:
        node_leave(node, rank)
        st.close()
        unlink(name)


def exchange_ab(args, dev: int, log):
    """The routed exchange measured against the native step at identical totals, on this GPU, in fresh
    child processes (subprocess, never exec): (a) 2 ranks, both on this device (peer-window transport,
    gloo for the small collectives), keys and ops split between them; (b) 1 rank with every key and op.
    Both KV-only, hybrid mop, same value size.  Returns ops/s of each, their ratio, the transport rank 0
    of (a) settled on and why it fell back if it did, and the integrity failures of both runs."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # pin both children to THIS physical device (on an 8-GPU node the 2-rank run would otherwise
    # spread over two GPUs: a different comparison)
    vis = env.get("HIP_VISIBLE_DEVICES") or env.get("CUDA_VISIBLE_DEVICES")
    phys = vis.split(",")[dev] if vis else str(dev)
    env["HIP_VISIBLE_DEVICES"] = phys
    env.pop("CUDA_VISIBLE_DEVICES", None)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    common = ["--mode", "kv", "--steps", "10", "--warmup", "3", "--host-api", "0", "--host-api-threads2", "0",
              "--embed-e2e", "0", "--daemon-docs", "0", "--search-keys", "0", "--exchange-ab", "0", "--mixed5", "0",
              "--verify", "5000", "--value-len", str(args.value_len), "--mop", str(args.mop)]
    me = os.path.abspath(__file__)
    runs = {}
    for w in (2, 1):
        cmd = [sys.executable, me, "--gpus", str(w), "--keys-per-gpu", str(args.exchange_keys // w),
               "--batch", str(args.exchange_batch // w)] + common
        if w > 1:
            cmd += ["--backend", "gloo", "--transport", "peer"]
        try:
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        except subprocess.TimeoutExpired:
            log(f"[bench] exchange A/B: {w}-rank child timed out")
            return None
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not line:
            log(f"[bench] exchange A/B: {w}-rank child failed (rc {r.returncode}): {r.stderr[-600:]}")
            return None
        runs[w] = json.loads(line[-1])
        log(f"[bench] exchange A/B: {w} rank(s) {runs[w]['value'] / 1e9:.3f} G ops/s, "
            f"{runs[w]['ms_per_step']:.2f} ms/step, integrity {runs[w]['integrity_failures']}")
    coll = runs[2]["config"].get("collectives") or ""
    transport = "peer" if "transport peer" in coll else ("rccl" if "transport rccl" in coll else coll)
    fb = coll.split("(fell back: ", 1)[1].split(")", 1)[0] if "(fell back: " in coll else None
    sync = "device flags" if "device-side posts" in coll else "collectives"
    direct = "direct responses" in coll
    return {"ops2": runs[2]["value"], "ops1": runs[1]["value"], "ratio": runs[2]["value"] / runs[1]["value"],
            "transport": transport, "fallback": fb, "sync": sync, "sync_error": runs[2].get("xr_sync_error"),
            "direct": direct,
            "integrity": runs[2]["integrity_failures"] + runs[1]["integrity_failures"],
            "totals": {"keys": args.exchange_keys, "ops_per_step": args.exchange_batch, "steps": 10,
                       "device": phys, "mode": "kv"}}


def kv_async_ab(args, dev: int, log):
    """Config #2 as written -- 32 concurrent writer + 32 reader client streams, each submitting its own
    slice -- against the default fused grid: two KV-only children at the bench's keys and batch (fresh
    processes, never exec), SPL_KVS_FUSED=3 (each stream posts its slice with a stream-ordered doorbell;
    the resident k_kv_server grid consumes posted slices) and SPL_KVS_FUSED=2.  Returns both rates,
    their ratio and both runs' integrity failures."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    vis = env.get("HIP_VISIBLE_DEVICES") or env.get("CUDA_VISIBLE_DEVICES")
    env["HIP_VISIBLE_DEVICES"] = vis.split(",")[dev] if vis else str(dev)
    env.pop("CUDA_VISIBLE_DEVICES", None)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--mode", "kv", "--steps", "10", "--warmup", "3",
           "--keys-per-gpu", str(args.keys_per_gpu), "--batch", str(args.batch), "--value-len", str(args.value_len),
           "--writer-streams", str(args.writer_streams), "--reader-streams", str(args.reader_streams),
           "--host-api", "0", "--host-api-threads2", "0", "--embed-e2e", "0", "--daemon-docs", "0",
           "--search-keys", "0", "--exchange-ab", "0", "--kv-async-ab", "0", "--mixed5", "0", "--verify", "5000"]
    runs = {}
    for mode in ("3", "2"):
        e = dict(env, SPL_KVS_FUSED=mode)
        try:
            r = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=600)
        except subprocess.TimeoutExpired:
            log(f"[bench] kv async A/B: SPL_KVS_FUSED={mode} child timed out")
            return None
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not line:
            log(f"[bench] kv async A/B: SPL_KVS_FUSED={mode} child failed (rc {r.returncode}): {r.stderr[-600:]}")
            return None
        runs[mode] = json.loads(line[-1])
        log(f"[bench] kv async A/B: SPL_KVS_FUSED={mode} {runs[mode]['value'] / 1e9:.3f} G ops/s, "
            f"{runs[mode]['ms_per_step']:.2f} ms/step, {runs[mode]['config']['kv_submission']}, "
            f"integrity {runs[mode]['integrity_failures']}")
    a, f = runs["3"], runs["2"]
    return {"async": a["value"], "fused": f["value"], "ratio": a["value"] / f["value"],
            "async_ms": a["ms_per_step"], "fused_ms": f["ms_per_step"],
            "submission": a["config"]["kv_submission"], "writer_streams": a["config"]["writer_streams"],
            "reader_streams": a["config"]["reader_streams"],
            "integrity": a["integrity_failures"] + f["integrity_failures"]}


def main():
    args = parse()
    # Hardware queues per priority level for this process (HIP default 4).  Each HIP stream the
    # process uses may claim a queue; with the 32 writer + 32 reader client streams, the store's
    # control / ring streams and torch's stream that is ~8 queues, and the GPU's queue scheduler
    # then time-slices them: the encoder phase ran 15-30 % slower.  2 per priority measured best
    # (profiles/r2_hw_queues.md).  Set before anything initialises HIP (the GPU boxes export 4;
    # override with SPLINTER_BENCH_HW_QUEUES).
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("SPLINTER_BENCH_HW_QUEUES", "2")
    # mixed step: every other writer slice on the low-priority queue pool (arena_kernels.hip
    # spl_kvs_create): +1.2 % on the throttled mixed step, -13 % on the unthrottled KV-only loop
    # (profiles/r2_kvs_order.md), so only for mixed
    os.environ.setdefault("SPL_KVS_SPREAD", "1" if args.mode == "mixed" else "0")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a mislabelled run",
              file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.ones(1)
            dist.all_reduce(t)
            seen = int(t.item())
            dist.destroy_process_group()
        else:
            seen = 1
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": seen}), flush=True)
        return

    routed = world > 1 or args.force_routed
    need_routed = routed
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # config #2's async form, measured FIRST: each child holds its own 100 M-key arena (~77 GB), which
    # next to this process's KV and search arenas would not fit in one GPU's HBM
    kab = None
    if world == 1 and args.kv_async_ab and args.mode != "embed" and not args.force_routed:
        kab = kv_async_ab(args, local % max(torch.cuda.device_count(), 1),
                          lambda *a: print(*a, file=sys.stderr, flush=True))
    dev = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    liveness = None
    if need_routed and world == 1 and "MASTER_ADDR" not in os.environ:
        import socket
        with socket.socket() as so_:
            so_.bind(("127.0.0.1", 0))
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(so_.getsockname()[1]), RANK="0",
                              WORLD_SIZE="1")
    if need_routed:
        # finite collective timeouts + async RCCL error handling, and a heartbeat monitor: a lost
        # rank ends every survivor with a non-zero exit instead of a hung node (parallel/health.py)
        from libsplinter_amd.parallel.health import Liveness, init_distributed
        init_distributed(args.backend, timeout_s=600.0,
                         device_id=torch.device("cuda", dev) if args.backend == "nccl" else None)
        if world > 1:
            liveness = Liveness(period_s=1.0, timeout_s=120.0)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values
    from libsplinter_amd.parallel.sharded import GpuShard, ShardedKV

    log = (lambda *a: print(*a, file=sys.stderr, flush=True)) if rank == 0 else (lambda *a: None)
    kpg = args.keys_per_gpu
    total_keys = kpg * world
    slots = int(kpg * args.slots_factor)
    # the ranks' arenas are the shards of ONE node store, node:<node_tag>kv (node_store.hpp): while the
    # bench runs, any process of the node opens it through the C ABI (splinterctl -u node:..., the
    # Rust / TS bindings) and reaches every rank's keys -- the benched store IS the product's
    node_tag = f"bench{os.environ.get('MASTER_PORT', os.getpid())}"
    t0 = time.time()
    arena = HbmArena.join_node(f"{node_tag}kv", rank, world, slots=slots, max_val=args.max_val, embeddings=False)
    if not (os.environ.get("BENCH_SKIP_MOP") and args.mop == 1):  # diagnosis: stores are created hybrid
        arena.store.set_mop(args.mop)  # 1 = hybrid scrub, the reference's store default
    kv = ShardedKV(GpuShard(arena))
    vstride = (args.max_val + 15) // 16 * 16

    # ---- prepopulate: every rank inserts the global ids it owns ----------
    chunk = 1 << 24
    inserted = 0
    for first in range(0, total_keys, chunk):
        n = min(chunk, total_keys - first)
        K = format_keys(n, "k", 10, 16, first=first)
        if routed:
            own = kv.owned_mask(K)
            ids = torch.nonzero(own).squeeze(1) + first
            K = K[own]
        else:
            ids = None
        V, L = format_values(K.shape[0], 1, args.value_len, vstride, first=first, ids=ids)
        st = arena.set(K, V, L)
        bad = int((st != 0).sum())
        if bad:
            raise RuntimeError(f"prepopulate: {bad} inserts failed (first status {st[st != 0][0].item()})")
        inserted += K.shape[0]
        del K, V, L, st
    torch.cuda.synchronize()
    log(f"[bench] rank0 arena {slots} slots, {inserted} keys inserted in {time.time() - t0:.1f}s "
        f"({arena.slots * 128 / 2**30 + arena.slots * vstride / 2**30:.1f} GiB)")

    # ---- per-step client batches (pre-generated: the client's own keys) ----
    n_set = int(args.batch * args.set_frac) if args.mode != "embed" else 0
    n_get = args.batch - n_set if args.mode != "embed" else 0
    nbuf = min(args.steps + args.warmup, 4)
    g = torch.Generator(device="cuda")
    g.manual_seed(1234 + rank)
    batches = []
    for b in range(nbuf):
        sid = torch.randint(0, total_keys, (n_set,), device="cuda", generator=g)
        gid = torch.randint(0, total_keys, (n_get,), device="cuda", generator=g)
        SK = format_keys(n_set, "k", 10, 16, ids=sid)
        GK = format_keys(n_get, "k", 10, 16, ids=gid)
        SV, SL = format_values(n_set, 2 + b, args.value_len, vstride, ids=sid)
        batches.append((SK, SV, SL, GK, gid))
    gout = torch.empty((n_get, vstride), dtype=torch.uint8, device="cuda")

    # ---- search arena (config #5 corpus): --search-keys embedded keys per GPU -------------
    sarena = None
    if args.search_keys > 0 and args.mode in ("embed", "mixed"):
        t1 = time.time()
        sarena = HbmArena.join_node(f"{node_tag}vec", rank, world, slots=int(args.search_keys * 1.25) + 4096,
                                    max_val=64, embeddings=True)
        g0 = torch.Generator(device="cuda")
        g0.manual_seed(77 + rank)
        ch = 1 << 20
        for first in range(0, args.search_keys, ch):
            n = min(ch, args.search_keys - first)
            K = format_keys(n, f"v{rank}_", 9, 16, first=first)
            V, L = format_values(n, 1, 32, 64, first=first)
            st = sarena.set(K, V, L)
            vec = torch.randn((n, 768), device="cuda", generator=g0)
            st2 = sarena.set_embeddings(K, vec)
            if int((st != 0).sum()) or int((st2 != 0).sum()):
                raise RuntimeError("search arena prepopulation failed")
            del K, V, L, vec, st, st2
        torch.cuda.synchronize()
        log(f"[bench] rank0 search arena {args.search_keys} embedded keys in {time.time() - t1:.1f}s "
            f"({sarena.slots * (3200 + 64) / 2**30:.1f} GiB)")

    # ---- embed phase (model) --------------------------------------------
    embedder = None
    if args.mode in ("embed", "mixed"):
        from libsplinter_amd.models.bench_embed import EmbedPhase
        embedder = EmbedPhase(arena, batch=args.embed_batch, seq=args.embed_seq, rank=rank, doc_arena=sarena)

    # set and get batches race each other on two hardware queues (utils/streams.py: distinct
    # priorities = distinct queue pools).  The embed phase runs AFTER the KV phase, not beside it:
    # the seqlock kernels' agent-scope release/acquire fences write back / invalidate the XCD L2s,
    # which stretched the concurrently running GEMMs 2x and made the overlapped step slower than
    # the serial one (profiles/r1_mixed_overlap.md).
    from libsplinter_amd.utils.streams import stream as hip_stream
    py_streams = bool(args.kv_cus) or args.overlap or bool(os.environ.get("BENCH_PY_STREAMS"))
    s_get, s_set = (hip_stream("high"), hip_stream("normal")) if (py_streams or need_routed) else (None, None)
    # BASELINE config #2: the set batch is issued by --writer-streams concurrent client streams and the
    # get batch by --reader-streams (streams share the HIP runtime's hardware queues, at most
    # GPU_MAX_HW_QUEUES per priority level; readers at high priority, writers at normal)
    nw, nr = max(1, args.writer_streams), max(1, args.reader_streams)
    # Python-side client streams only for the fallback path (--kv-cus masks, BENCH_PY_STREAMS): every
    # stream the process touches can claim a hardware queue (profiles/r2_hw_queues.md)
    w_streams = [s_set] + [hip_stream("normal") for _ in range(nw - 1 if py_streams else 0)]
    r_streams = [s_get] + [hip_stream("high") for _ in range(nr - 1 if py_streams else 0)]
    s_emb = None
    if args.overlap and not args.kv_cus and world == 1:
        s_emb = hip_stream("low")
        log("[bench] overlapped phases on unmasked streams")
    if args.kv_cus and world == 1:
        from libsplinter_amd.utils.streams import cu_mask_bits, masked_stream
        kv_bits, emb_bits = cu_mask_bits(args.kv_cus), cu_mask_bits(32 - args.kv_cus, args.kv_cus)
        w_streams = [masked_stream(kv_bits) for _ in range(nw)]
        r_streams = [masked_stream(kv_bits) for _ in range(nr)]
        s_emb = masked_stream(emb_bits)
        log(f"[bench] overlapped phases: KV on {len(kv_bits)} CUs, encoder on {len(emb_bits)} CUs")
    stats = arena.stats

    def _parts(n, k):
        b = [n * j // k for j in range(k + 1)]
        return [(b[j], b[j + 1]) for j in range(k) if b[j + 1] > b[j]]

    set_parts, get_parts = _parts(n_set, nw), _parts(n_get, nr)
    # native fan-out (spl_kvs_step, arena_kernels.hip): one C call issues every client stream's slice, so 64
    # streams do not make the step host-bound (the per-launch Python path starved the queues)
    kvs = None
    if not py_streams and n_set + n_get:
        from libsplinter_amd.ops.arena import KvStreams
        kvs = KvStreams(nw, nr)
        s_status = torch.empty(max(n_set, 1), dtype=torch.int32, device="cuda")
        g_status = torch.empty(max(n_get, 1), dtype=torch.int32, device="cuda")
        g_lens = torch.empty(max(n_get, 1), dtype=torch.int32, device="cuda")

    # what actually launches the KV work of a step (reported in the JSON config)
    kv_mode = int(os.environ.get("SPL_KVS_FUSED", "2"))
    if kvs is not None and kv_mode == 3:
        kv_launch = {"writer_streams": len(set_parts), "reader_streams": len(get_parts), "launches": 1,
                     "how": f"async: each of the {len(set_parts)} writer + {len(get_parts)} reader client streams posts "
                            "its slice with a stream-ordered doorbell write (hipStreamWriteValue64); ONE resident "
                            "server grid (k_kv_server) consumes the slices as they are posted"}
    elif kvs is not None and kv_mode != 0:
        kv_launch = {"writer_streams": 1, "reader_streams": 1, "launches": 1,
                     "how": f"fused: ONE grid (k_kv_fused) consumes all {len(set_parts)} set + {len(get_parts)} get "
                            "client slices, launched on one stream"}
    elif kvs is not None:
        kv_launch = {"writer_streams": len(set_parts), "reader_streams": len(get_parts),
                     "launches": len(set_parts) + len(get_parts),
                     "how": "per slice: one launch per client slice, each on its own stream (SPL_KVS_FUSED=0)"}
    else:
        kv_launch = {"writer_streams": len(set_parts), "reader_streams": len(get_parts),
                     "launches": len(set_parts) + len(get_parts),
                     "how": "python client streams, one arena.set / arena.get launch per slice"}

    _phase_gap_ms = float(os.environ.get("BENCH_PHASE_GAP_MS", "0"))
    s_kvo = None
    if args.overlap_native and kvs is not None and embedder is not None and world == 1:
        if args.overlap_kv_cus:
            from libsplinter_amd.utils.streams import cu_mask_bits, masked_stream
            s_kvo = masked_stream(cu_mask_bits(args.overlap_kv_cus))
            log(f"[bench] overlapped phases: KV grid on {8 * args.overlap_kv_cus} CUs, encoder on every CU")
        else:
            s_kvo = hip_stream("low")


    # Host submission throttle (--throttle): the next step's KV launches are issued only once
    # this step's encoder has finished.  Work the host has queued on the other hardware queues --
    # even when it is blocked on an event -- makes the queue scheduler time-slice the queue that
    # runs the encoder (profiles/r2_hw_queues.md), so submitting early costs more than the few
    # microseconds of launch latency it hides.
    throttle_ev = [None]
    # encoder phase bracketed by events inside the timed steps (no host sync): its own time per step,
    # so encoder TFLOP/s is quoted over encoder time, not over the mixed step
    emb_events = []
    timing_emb = [False]

    def run_embed():
        if timing_emb[0]:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            embedder.run()
            e1.record()
            emb_events.append((e0, e1))
        else:
            embedder.run()

    def step_local(i):
        SK, SV, SL, GK, _ = batches[i % nbuf]
        cur = torch.cuda.current_stream()
        if args.throttle and throttle_ev[0] is not None:
            throttle_ev[0].synchronize()
        kv_streams = w_streams[:len(set_parts)] + r_streams[:len(get_parts)]
        if kvs is not None and s_emb is None and s_kvo is not None:
            # overlapped phases: the KV fan-out forks from its own origin stream while the encoder
            # runs on the current one (no release / acquire fence left in the default KV kernels)
            s_kvo.wait_stream(cur)
            with torch.cuda.stream(s_kvo):
                kvs.step(arena, SK if n_set else None, SV if n_set else None, SL if n_set else None, s_status,
                         GK if n_get else None, gout if n_get else None, g_lens, g_status)
        elif kvs is not None and s_emb is None:
            kvs.step(arena, SK if n_set else None, SV if n_set else None, SL if n_set else None, s_status,
                     GK if n_get else None, gout if n_get else None, g_lens, g_status)
        elif n_set:
            for s in kv_streams:
                s.wait_stream(cur)
            for s, (a, b) in zip(w_streams, set_parts):
                with torch.cuda.stream(s):
                    arena.set(SK[a:b], SV[a:b], SL[a:b])
            for s, (a, b) in zip(r_streams, get_parts):
                with torch.cuda.stream(s):
                    arena.get(GK[a:b], out=gout[a:b])
            if s_emb is None:
                for s in kv_streams:
                    cur.wait_stream(s)
        if embedder is not None:
            if _phase_gap_ms:  # diagnosis only (BENCH_PHASE_GAP_MS): idle gap between the phases
                torch.cuda.synchronize()
                time.sleep(_phase_gap_ms / 1e3)
            if s_emb is None:
                run_embed()
            else:
                s_emb.wait_stream(cur)
                with torch.cuda.stream(s_emb):
                    embedder.run()
                cur.wait_stream(s_emb)
        if s_emb is not None and n_set:
            for s in kv_streams:
                cur.wait_stream(s)
        if s_kvo is not None:
            cur.wait_stream(s_kvo)
        if args.throttle and embedder is not None:
            throttle_ev[0] = cur.record_event()

    # N > 1: a host-sync-free software pipeline over the routed exchange (parallel/xroute.py).
    # Per step i (parity i % 2 double-buffers every exchange block and client output):
    #   s_set : owner kernels of batch i on the 32 + 32 client streams (own ops in place, peers'
    #           request blocks -> their response blocks), after batch i's requests
    #   main  : embed_i after them (no seqlock kernels beside the GEMMs), as in the local step
    #   s_resp: the response collective + gather of batch i                 (overlaps embed_i)
    #   s_req : pack of batch i+1 straight into the owners' request blocks + the count all-to-all
    #           (waits for finish(i-1): no block is reused while anyone still reads it; overlaps embed_i)
    # All K steps' responses are delivered inside the timed region (device-wide sync at the end).
    xr = None
    if need_routed and n_set + n_get and kvs is not None:
        from libsplinter_amd.parallel.xroute import XRoute
        vw = min((args.value_len + 15) // 16 * 16, vstride)
        xr = XRoute(GpuShard(arena), n_set, n_get, vw, ks=16, group=dist.new_group(backend=args.backend),
                    resp_group=dist.new_group(backend=args.backend), transport=args.transport)
        log(f"[bench] routed exchange: transport {xr.transport}, world {world}, caps {xr.cap_s}/{xr.cap_g}, "
            f"window {xr.g.window_b / 2**30:.2f} GiB")
        s_req, s_resp = hip_stream("low"), hip_stream("low")
        # direct responses (peer transport): the owners write every result into these arrays, which
        # live in this rank's exchange window (no gather kernel)
        r_out = ([xr.outputs(p) for p in range(2)] if xr.direct else
                 [(torch.empty(max(n_set, 1), dtype=torch.int32, device="cuda"),
                   torch.empty((max(n_get, 1), vw), dtype=torch.uint8, device="cuda"),
                   torch.empty(max(n_get, 1), dtype=torch.int32, device="cuda"),
                   torch.empty(max(n_get, 1), dtype=torch.int32, device="cuda")) for _ in range(2)])
        prev_exec = []

    requested = {}  # step -> its request event (issued ahead by the previous step of the same phase)

    def _request(i):
        SK, SV, SL, GK, _ = batches[i % nbuf]
        with torch.cuda.stream(s_req):
            xr.request(i, SK if n_set else None, SV if n_set else None, SL if n_set else None, GK if n_get else None)
            requested[i] = s_req.record_event()

    def step_routed(i, last=False):
        """One routed step, in the local step's order (KV phase, then the encoder), with the exchange
        around it: the owner kernels of batch i run first, the encoder after them, and while it runs
        the responses of batch i are gathered and batch i+1's records packed into the owners' blocks
        (issued here unless i is the last step of its phase: no work of an uncounted step inside the
        timed region)."""
        cur = torch.cuda.current_stream()
        sst, gov, gln, gst = r_out[i % 2]
        # host submission throttle, as the local step: step i's launches are issued once embed_{i-1}
        # has finished, so no KV dispatch waits queued beside the encoder
        if args.throttle and throttle_ev[0] is not None:
            throttle_ev[0].synchronize()
        if i not in requested:
            _request(i)
        s_set.wait_event(requested.pop(i))
        s_set.wait_stream(cur)
        with torch.cuda.stream(s_set):
            xr.execute(i, kvs, sst, gov, gln, gst)
            ev_exec = s_set.record_event()
        if embedder is not None:
            cur.wait_event(ev_exec)
            run_embed()
            if args.throttle:
                throttle_ev[0] = cur.record_event()
        s_resp.wait_event(ev_exec)
        with torch.cuda.stream(s_resp):
            xr.respond(i)
            xr.finish(i, sst, gov, gln, gst)
        if not last:
            _request(i + 1)
        if embedder is None:
            cur.wait_stream(s_resp)

    if routed and xr is None:
        raise SystemExit("[bench] the routed step needs the native client-stream fan-out and a KV batch "
                         "(not --kv-cus / --overlap / BENCH_PY_STREAMS, not --mode embed)")
    step = step_routed if routed else step_local

    for i in range(args.warmup):
        step(i, last=i == args.warmup - 1) if routed else step(i)
    torch.cuda.synchronize()
    arena.reset_stats()
    if xr is not None:
        xr.phase_reset()  # SPLINTER_XR_PHASES=1: attribute the timed steps only
    if routed:
        dist.barrier()
    torch.cuda.synchronize()
    prof = _timed_region_profiler()
    prof(True)
    timing_emb[0] = True
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, last=i == args.steps - 1) if routed else step(args.warmup + i)
    torch.cuda.synchronize()
    if routed:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    prof(False)
    timing_emb[0] = False
    emb_phase_ms = (sum(a.elapsed_time(b) for a, b in emb_events) / len(emb_events)) if emb_events else None
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    st = stats.clone()
    if routed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(st)
    elapsed = t.item()
    attempts, ok, again, miss = [int(x) for x in st.tolist()]

    # ---- integrity: the LAST timed step's own get outputs, sampled over the whole batch, must
    # parse and carry their key's id with a consistent fill (the 'ver:|id:|data:' format is
    # version-independent: any version a racing set wrote is valid), and its sets must have landed
    def check_rows(s_, o, ln, ids, what):
        fails, kinds = 0, {}
        for i in range(len(ids)):
            if s_[i] != 0:
                fails += 1
                kinds[int(s_[i])] = kinds.get(int(s_[i]), 0) + 1
                continue
            v = bytes(o[i, : ln[i]])
            try:
                head, rest = v.split(b"|id:", 1)
                ver = int(head[4:])
                ident = int(rest.split(b"|", 1)[0])
                fill = v[v.index(b"data:") + 5:]
                if ident != ids[i] or fill != bytes([65 + ver % 26]) * len(fill):
                    fails += 1
                    kinds["content"] = kinds.get("content", 0) + 1
                    if kinds["content"] <= 3:
                        log(f"[bench] {what}: bad value for id {ids[i]} (len {ln[i]}): {v[:60]!r}...{v[-20:]!r}")
            except Exception:
                fails += 1
                kinds["parse"] = kinds.get("parse", 0) + 1
                if kinds["parse"] <= 3:
                    log(f"[bench] {what}: unparsable value for id {ids[i]} (len {ln[i]}): {v[:60]!r}...{v[-20:]!r}")
        if kinds:
            log(f"[bench] {what}: integrity failures by kind (rank {rank}): {kinds}")
        return fails

    integrity_fail = integrity_rows = timed_set_fail = 0
    integrity_source = None
    last = args.warmup + args.steps - 1
    if args.verify and n_get:
        gid_last = batches[last % nbuf][4]
        m = min(args.verify, n_get)
        sel = torch.linspace(0, n_get - 1, m, device="cuda").long()
        timed = None
        if routed and xr is not None:
            sst_l, gov_l, gln_l, gst_l = r_out[last % 2]
            timed = (gst_l, gov_l, gln_l, sst_l)
        elif kvs is not None:
            timed = (g_status, gout, g_lens, s_status)
        if timed is not None:
            gs, go, gl, ss = timed
            integrity_fail = check_rows(gs[sel].cpu().numpy(), go[sel].cpu().numpy(), gl[sel].cpu().numpy(),
                                        gid_last[sel].cpu().numpy(), "timed gets")
            timed_set_fail = int((ss[:n_set] != 0).sum().item()) if n_set else 0
            integrity_rows = m
            integrity_source = (f"the last timed step's own get outputs ({m} of {n_get} rows, strided over the "
                                f"batch) + every status of its {n_set} sets")
        else:  # python-stream fallback paths keep no statuses: fresh gets of that step's keys
            GK = batches[last % nbuf][3]
            sts, outv, lens = (kv.get if routed else arena.get)(GK[sel])
            integrity_fail = check_rows(sts.cpu().numpy(), outv.cpu().numpy(), lens.cpu().numpy(),
                                        gid_last[sel].cpu().numpy(), "fresh gets")
            integrity_rows = m
            integrity_source = f"fresh gets of the last timed step's keys ({m} rows)"
        if routed:
            x = torch.tensor([integrity_fail, timed_set_fail, integrity_rows], device="cuda")
            dist.all_reduce(x)
            integrity_fail, timed_set_fail, integrity_rows = [int(v) for v in x.tolist()]
    # stream-posted server (SPL_KVS_FUSED=3): a server that gave up waiting for a post left slices unrun
    kv_async_error = kvs.async_error() if (kvs is not None and kv_mode == 3) else None


    # ---- per-call C API (outside the timed region): splinter_set / splinter_get from host threads
    # through the device command ring of an hbm: store (tools/splinter_hostapi_bench.cpp)
    def host_api_run(threads):
        import subprocess
        tool = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsplinter_amd", "bin",
                            "splinter_hostapi_bench")
        try:
            r = subprocess.run([tool, "--store", f"hbm:hapi{os.getpid()}t{threads}", "--threads", str(threads),
                                "--seconds", "1", "--keys", "65536", "--value-len", str(args.value_len)],
                               capture_output=True, text=True, timeout=120)
            if r.returncode == 0:
                return json.loads(r.stdout.strip().splitlines()[-1])
            log(f"[bench] host-API run failed: {r.stderr[-300:]}")
        except Exception as e:  # the headline stands without it
            log(f"[bench] host-API run failed: {e}")
        return None

    host_api = host_api_run(args.host_api) if args.host_api > 0 and rank == 0 else None
    host_api2 = host_api_run(args.host_api_threads2) if args.host_api_threads2 > 0 and rank == 0 else None

    e2e = None
    if embedder is not None and args.embed_e2e > 0:
        from libsplinter_amd.models.bench_embed import EmbedE2E
        pipe = EmbedE2E(embedder.enc, batch=args.embed_batch, seq=args.embed_seq, rank=rank)
        for _ in range(2):  # warm-up: tokenizer threads, and both key sets' varlen shapes (first-shape GEMM setup)
            pipe.run()
        torch.cuda.synchronize()
        pipe.t_wait = pipe.t_tok = 0.0
        pipe.calls = 0
        t0 = time.perf_counter()
        fails_d = torch.zeros((), dtype=torch.int64, device="cuda")
        for _ in range(args.embed_e2e):  # write failures counted on the device: no per-batch host sync
            fails_d += (pipe.run() != 0).sum()
        torch.cuda.synchronize()
        fails = int(fails_d.item())
        te = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        if routed:
            dist.all_reduce(te, op=dist.ReduceOp.MAX)
        dt = te.item()
        e2e = {"vectors_per_s": pipe.docs * args.embed_e2e * world / dt, "ms_per_batch": dt / args.embed_e2e * 1e3,
               "tokens_per_batch": pipe.tokens, "write_failures": fails,
               "host_wait_ms": pipe.t_wait / max(pipe.calls, 1) * 1e3,
               "host_tokenize_ms": pipe.t_tok / max(pipe.calls, 1) * 1e3}
        pipe.close()

    # ---- the embedding daemon itself, owner computes: each rank's daemon embeds the pending
    # documents of its own store (reference splinference.cpp:500-552)
    daemon = None
    if embedder is not None and args.daemon_docs > 0:
        daemon = daemon_run(embedder.enc, args.daemon_docs, args.embed_seq, rank, world, routed, f"{node_tag}dm")

    # ---- config #5 query phase: batched cosine top-10 over every rank's search arena ---------
    # (the vectors the embed phase wrote are in there too).  Rank 0's queries are broadcast (C3),
    # each GPU scores its arena with the MFMA search pass + fp32 re-score (K7), and the local top-k
    # lists are all-gathered and merged (C4).  Recall@10 of the batched path against the exact fp32
    # kernel on the first 16 queries.
    search = None
    if sarena is not None and args.search_queries > 0 and args.search_batches > 0:
        skv = ShardedKV(GpuShard(sarena))
        gq = torch.Generator(device="cuda")
        gq.manual_seed(4242)
        ids = torch.randint(0, args.search_keys, (args.search_queries,), device="cuda", generator=gq)
        _, base = sarena.get_embeddings(format_keys(args.search_queries, "v0_", 9, 16, ids=ids))
        q = base + 0.5 * torch.randn(base.shape, device="cuda", generator=gq)
        skv.search(q, k=10)  # warm-up (search workspaces, first-shape setup)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.search_batches):
            own_b, sim_b, _, key_b = skv.search(q, k=10)
        torch.cuda.synchronize()
        ts = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(ts, op=dist.ReduceOp.MAX)
        own_e, sim_e, _, key_e = skv.search(q[:16], k=10)  # < 32 queries: the exact fp32 kernel
        kb = [set(bytes(r).split(b"\0", 1)[0] for r in key_b[i].cpu().numpy()) for i in range(16)]
        ke = [set(bytes(r).split(b"\0", 1)[0] for r in key_e[i].cpu().numpy()) for i in range(16)]
        recall = sum(len(a & b) for a, b in zip(kb, ke)) / sum(len(b) for b in ke)
        dt = ts.item()
        search = {"qps": args.search_queries * args.search_batches / dt, "ms_per_batch": dt / args.search_batches * 1e3,
                  "recall_at_10": recall, "keys_total": args.search_keys * world}

    # ---- config #5 mixed steps: embed a batch -> its vectors inserted into the search arena's slots
    # (the pooling kernel's seqlocked slot write) -> a batched top-10 query over the whole arena with
    # queries built from the vectors just written (each must find its own document first) -------
    mixed5 = None
    if sarena is not None and embedder is not None and args.mixed5 > 0 and args.search_queries > 0:
        skv5 = ShardedKV(GpuShard(sarena))
        nq = args.search_queries
        gq5 = torch.Generator(device="cuda")
        gq5.manual_seed(99)
        noise = torch.randn((nq, 768), device="cuda", generator=gq5)
        pick = torch.arange(nq, device="cuda") % embedder.docs_per_step

        def step5():
            vec, _ = embedder.run()  # [docs, 768] fp32, also written into the documents' slots
            v = vec[pick]
            q = v + (0.01 / 768 ** 0.5) * v.norm(dim=1, keepdim=True) * noise  # ~1 % perturbation
            return skv5.search(q, k=10)

        step5()  # warm-up
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.mixed5):
            res5 = step5()
        torch.cuda.synchronize()
        t5 = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(t5, op=dist.ReduceOp.MAX)
        dt5 = t5.item()
        # the last step's top-1 of every query must be the document its query was built from
        keys5 = res5[3][:, 0].cpu().numpy()
        want = embedder.keys[pick].cpu().numpy()
        hit = float(sum(bytes(a).split(b"\0", 1)[0] == bytes(b).split(b"\0", 1)[0] for a, b in zip(keys5, want)))
        mixed5 = {"ms_per_step": dt5 / args.mixed5 * 1e3, "qps": nq * args.mixed5 * world / dt5,
                  "vectors_per_s": embedder.docs_per_step * args.mixed5 * world / dt5, "self_top1": hit / nq}

    # ---- honest exchange measurement on this one GPU (N=1 only, after everything else): fresh child
    # processes, never exec -- a 2-rank KV-only run with both ranks on this device (peer windows; gloo
    # for the small collectives) and a 1-rank run at identical totals
    xab = None
    if world == 1 and args.exchange_ab and args.mode != "embed":
        xab = exchange_ab(args, dev, log)

    kv_ops = (n_set + n_get) * args.steps * world
    kv_ops_s = kv_ops / elapsed if kv_ops else 0.0
    emb_vps = emb_tps = enc_tflops = None
    if embedder is not None:
        emb_vps = embedder.docs_per_step * args.steps * world / elapsed
        emb_tps = embedder.tokens_per_step * args.steps * world / elapsed
        if emb_phase_ms:  # encoder FLOPs over the encoder phase's own (event-timed) time
            enc_tflops = embedder.flops_per_step / (emb_phase_ms * 1e-3) / 1e12
    value = kv_ops_s if args.mode != "embed" else emb_vps
    res = {
        "metric": "KV set/get ops/sec + Nomic-768d embed vectors/sec at 1/2/4/8 MI355X",
        "value": value,
        "unit": "ops/s" if args.mode != "embed" else "vectors/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (value / REF_MRMW_OPS) if args.mode != "embed" else None,
        "dtype": "bf16" if embedder is not None else "u8-kv",
        "data": "synthetic keys k%010d / 150-B 'ver:|id:|data:' payloads; random-init Nomic weights; "
                "random N(0,1) 768-d vectors in the search arenas",
        "config": {
            "model": "hbm-arena-v4 (128-B slots, 256-B values)" + (" + nomic-embed-text-v1.5" if embedder else ""),
            "store": f"node:{node_tag}kv ({world} HBM shard{'s' if world > 1 else ''})",
            "keys_per_gpu": kpg, "slots_per_gpu": slots, "global_batch": args.batch * world,
            "set_frac": args.set_frac, "seq_len": args.embed_seq if embedder else None,
            "parallelism": f"hash-shard{world}" + (" + dp" if embedder else ""),
            "mode": args.mode, "phases": ("serial" if s_kvo is None else
                                                 f"overlapped (KV grid on {8 * args.overlap_kv_cus} CUs)"
                                                 if args.overlap_kv_cus else "overlapped"), "mop": args.mop, "value_len": args.value_len,
            # how the step's KV work is submitted: the batch is split into --writer-streams set slices and
            # --reader-streams get slices (the config's concurrent clients); in the default fused mode ONE
            # grid consumes every slice from one stream, so the streams that actually launch are counted here
            "client_slices": {"writer": nw, "reader": nr},
            "writer_streams": kv_launch["writer_streams"], "reader_streams": kv_launch["reader_streams"],
            "kv_launches_per_step": kv_launch["launches"], "kv_submission": kv_launch["how"],
            "hw_queues_per_priority": int(os.environ["GPU_MAX_HW_QUEUES"]),
            "collectives": (f"routed exchange, transport {xr.transport}"
                            + (f" (fell back: {xr.fallback_reason})" if xr.fallback_reason else "") + ": request / response rows "
                            + ("stored into the owners' peer-mapped windows over xGMI, "
                               if xr.transport == "peer" else "moved by one all-to-all per direction, ")
                            + ("step ordered by device-side posts into the peer windows (no collective per step)"
                               if xr.sync == "flags" else "one count all-to-all + one response all-to-all per step")
                            + ("; owners write results straight into the requesters' client arrays (direct "
                               "responses, no gather)" if xr.direct else ""))
            if routed and xr else None,
            "search_keys_per_gpu": args.search_keys if sarena is not None else 0,
            # bytes each GPU stores into its W-1 peers per routed step (own-shard ops never leave the GPU):
            # set request key + len + value prefix and its status back, get request key and its status +
            # len + value prefix back; spread over W-1 point-to-point links (one per peer), and the
            # per-link time at the ~153 GB/s per-link figure of the task statement
            "xgmi_bytes_per_step_per_gpu": (xr.g.wire_bytes(n_set * (world - 1) / world, n_get * (world - 1) / world)
                                            if routed and xr else 0),
            "xgmi_link_ms_per_step": (xr.g.wire_bytes(n_set * (world - 1) / world, n_get * (world - 1) / world)
                                      / (world - 1) / 153e9 * 1e3 if routed and xr and world > 1 else 0),
        },
        "kv_ops_per_s": kv_ops_s,
        "embed_vectors_per_s": emb_vps,
        "embed_tokens_per_s": emb_tps,
        "embed_e2e_vectors_per_s": e2e["vectors_per_s"] if e2e else None,
        "embed_e2e_ms_per_batch": e2e["ms_per_batch"] if e2e else None,
        "embed_e2e_tokens_per_batch": e2e["tokens_per_batch"] if e2e else None,
        "embed_e2e_write_failures": e2e["write_failures"] if e2e else None,
        # per batch on the host: waiting for the GPU vs tokenizing + packing the next batch (a wait
        # near 0 means the tokenizer, not the encoder, bounds the pipeline)
        "embed_e2e_host_wait_ms": e2e["host_wait_ms"] if e2e else None,
        "embed_e2e_host_tokenize_ms": e2e["host_tokenize_ms"] if e2e else None,
        "embed_phase_ms_per_step": emb_phase_ms,
        "encoder_tflops": enc_tflops,
        "kv_attempts": attempts, "kv_ok": ok, "kv_eagain_retries": again, "kv_miss": miss,
        "successful_ops_per_s": ok / elapsed if elapsed else 0.0,
        "integrity_failures": integrity_fail,
        "integrity_rows_checked": integrity_rows,
        "integrity_source": integrity_source,
        "timed_set_failures": timed_set_fail, "kv_async_error": kv_async_error,
        "host_api_threads": args.host_api if host_api else None,
        "host_api_ops_per_s": host_api["ops_per_s"] if host_api else None,
        "host_api_p50_us": host_api["p50_us"] if host_api else None,
        "host_api_p99_us": host_api["p99_us"] if host_api else None,
        "host_api_threads2": args.host_api_threads2 if host_api2 else None,
        "host_api2_ops_per_s": host_api2["ops_per_s"] if host_api2 else None,
        "host_api2_p50_us": host_api2["p50_us"] if host_api2 else None,
        "routed_kv_ops_per_s": kv_ops_s if routed else None,
        "exchange_2rank_ops_per_s": xab["ops2"] if xab else None,
        "exchange_1rank_ops_per_s": xab["ops1"] if xab else None,
        "exchange_ratio": xab["ratio"] if xab else None,
        "exchange_transport": xab["transport"] if xab else None,
        "exchange_fallback_reason": xab["fallback"] if xab else None,
        "exchange_sync": xab["sync"] if xab else None, "exchange_sync_error": xab["sync_error"] if xab else None,
        "exchange_direct_responses": xab["direct"] if xab else None,
        "xr_sync_error": (xr.sync_error() if (routed and xr is not None) else None),
        "exchange_integrity_failures": xab["integrity"] if xab else None,
        # SPLINTER_XR_PHASES=1 on a routed run: device ms per phase of a timed step, host ms in collectives
        "xr_phases_ms": xr.phase_summary() if xr is not None else None,
        # config #2 literally: every one of the client streams submits its own slice (SPL_KVS_FUSED=3)
        "kv_async_ops_per_s": kab["async"] if kab else None,
        "kv_fused_only_ops_per_s": kab["fused"] if kab else None,
        "kv_async_ratio": kab["ratio"] if kab else None,
        "kv_async_ms_per_step": kab["async_ms"] if kab else None,
        "kv_async_submission": kab["submission"] if kab else None,
        "kv_async_streams": {"writer": kab["writer_streams"], "reader": kab["reader_streams"]} if kab else None,
        "kv_async_integrity_failures": kab["integrity"] if kab else None,
        "exchange_totals": xab["totals"] if xab else None,
        "mixed5_ms_per_step": mixed5["ms_per_step"] if mixed5 else None,
        "mixed5_qps": mixed5["qps"] if mixed5 else None,
        "mixed5_vectors_per_s": mixed5["vectors_per_s"] if mixed5 else None,
        "mixed5_self_top1": mixed5["self_top1"] if mixed5 else None,
        "daemon_vectors_per_s": daemon["vectors_per_s"] if daemon else None,
        "daemon_docs_embedded": daemon["embedded"] if daemon else None,
        "daemon_docs_expected": daemon["expected"] if daemon else None,
        "search_qps": search["qps"] if search else None,
        "search_path": ("spl_search_batch (C ABI: device query prep, bf16 MFMA candidate passes, fp32 re-score, keys "
                        "with the hits)" if GpuShard.capi_search else "ops/search.py VectorSearch.search_batch")
        if search else None,
        "search_ms_per_batch": search["ms_per_batch"] if search else None,
        "search_recall_at_10": search["recall_at_10"] if search else None,
        "search_keys_total": search["keys_total"] if search else None,
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    if liveness is not None:
        dist.barrier()
        liveness.stop()
    if xr is not None:
        xr.close()
    if sarena is not None:
        sarena.close()
    arena.close()
    if need_routed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

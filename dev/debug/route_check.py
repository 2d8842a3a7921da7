"""Routed set/get integrity check on the real backend (torchrun; N=1 works with RCCL too).

Sequential (every phase on the current stream) and pipelined (the bench's four-stream schedule)
routed sets of known values, then a local read-back of every key of this rank's shard.
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--mode", default="seq", choices=["seq", "pipe"])
    ap.add_argument("--backend", default="nccl")
    a = ap.parse_args()
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    dev = int(os.environ.get("LOCAL_RANK", 0)) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    dist.init_process_group(a.backend, device_id=torch.device("cuda", dev) if a.backend == "nccl" else None)
    from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values
    from libsplinter_amd.parallel.routed import RoutedKV, route_capacity
    from libsplinter_amd.parallel.sharded import GpuShard, ShardedKV
    from libsplinter_amd.utils.streams import stream as hip_stream
    n = a.keys
    arena = HbmArena.create(f"rc{os.getpid()}", slots=4 * n * world, max_val=256, embeddings=False)
    arena.store.set_mop(0)
    kv = ShardedKV(GpuShard(arena))
    rkv = RoutedKV(GpuShard(arena), group=dist.new_group(backend=a.backend),
                   resp_group=dist.new_group(backend=a.backend))
    ids = torch.arange(rank, n * world, world, device="cuda")  # every rank sets n keys, all ranks' ids disjoint
    K = format_keys(ids.numel(), "k", 10, 16, ids=ids)
    cap = route_capacity(ids.numel(), world)
    bad_total = 0
    for ver in (3, 4, 5):
        V, L = format_values(ids.numel(), ver, 150, 256, ids=ids)
        if a.mode == "seq":
            op = rkv.begin_set(K, V, L, cap, 160)
            rkv.execute(op)
            rkv.respond(op)
            st = rkv.finish(op)
        else:
            s_req, s_set, s_resp = hip_stream("low"), hip_stream("normal"), hip_stream("low")
            cur = torch.cuda.current_stream()
            s_req.wait_stream(cur)
            with torch.cuda.stream(s_req):
                op = rkv.begin_set(K, V, L, cap, 160)
                ev = s_req.record_event()
            s_set.wait_event(ev)
            with torch.cuda.stream(s_set):
                rkv.execute(op)
                ev2 = s_set.record_event()
            s_resp.wait_event(ev2)
            with torch.cuda.stream(s_resp):
                rkv.respond(op)
                st = rkv.finish(op)
            cur.wait_stream(s_resp)
        torch.cuda.synchronize()
        dist.barrier()
        nbad_status = int((st != 0).sum())
        # read back this rank's OWN shard locally: every key whose owner is this rank
        allids = torch.arange(0, n * world, device="cuda")
        AK = format_keys(allids.numel(), "k", 10, 16, ids=allids)
        own = kv.owned_mask(AK)
        gst, out, ol = arena.get(AK[own].contiguous())
        exp, el = format_values(int(own.sum()), ver, 150, 256, ids=allids[own])
        okrow = (gst == 0) & (ol == el) & (out[:, :160] == exp[:, :160]).all(1)
        bad = int((~okrow).sum())
        bad_total += bad + nbad_status
        print(f"[rank {rank}] {a.mode} ver {ver}: set status!=0 {nbad_status}, bad rows {bad} / {int(own.sum())}",
              flush=True)
    dist.barrier()
    arena.close()
    dist.destroy_process_group()
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Does the ORDER of a KV batch matter?  The fused KV grid (KvStreams, 32 set + 32 get client slices)
on bench.py's config #2 arena (100 M keys, 200 M slots, hybrid scrub, 150-B values), each step's
batch as generated (random keys) vs the same batch sorted by home slot (hash % slots), interleaved.
The sort itself is NOT timed: this measures what address locality (UTCL1 / UTCL2 translation reuse,
DRAM row hits) is worth, to decide whether an in-step bucketing pass pays.

python scripts/kv_order_ab.py [--keys 100000000] [--batch 16000000] [--rounds 5] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=100_000_000)
    ap.add_argument("--batch", type=int, default=16_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--bucket-bits", type=int, default=0, help="sort by the top bits of the home slot only")
    a = ap.parse_args()
    import torch
    from libsplinter_amd import _native as N
    from libsplinter_amd.ops.arena import HbmArena, KvStreams, format_keys, format_values, _stream
    slots = 2 * a.keys
    arena = HbmArena.create(f"kvord{os.getpid()}", slots=slots, max_val=256, embeddings=False)
    arena.store.set_mop(1)
    t0 = time.time()
    for first in range(0, a.keys, 1 << 24):
        n = min(1 << 24, a.keys - first)
        K = format_keys(n, "k", 10, 16, first=first)
        V, L = format_values(n, 1, 150, 256, first=first)
        assert int((arena.set(K, V, L) != 0).sum()) == 0
        del K, V, L
    torch.cuda.synchronize()
    print(f"prepopulated {a.keys} keys in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    ns = ng = a.batch // 2
    sid = torch.randint(0, a.keys, (ns,), device="cuda", generator=g)
    gid = torch.randint(0, a.keys, (ng,), device="cuda", generator=g)
    SK = format_keys(ns, "k", 10, 16, ids=sid)
    GK = format_keys(ng, "k", 10, 16, ids=gid)
    SV, SL = format_values(ns, 2, 150, 256, ids=sid)

    def home(K):
        h = torch.empty(K.shape[0], dtype=torch.int64, device="cuda")
        rc = N.hip_lib().spl_hash_keys(K.data_ptr(), K.shape[1], K.shape[0], h.data_ptr(), _stream())
        assert rc == 0
        hu = h.view(torch.int64)
        # unsigned 64-bit modulo in int64 arithmetic: (hi * 2^32 + lo) % slots
        hi = (hu >> 32) & 0xFFFFFFFF
        lo = hu & 0xFFFFFFFF
        r = ((hi % slots) * (1 << 32) % slots + lo) % slots
        if a.bucket_bits:
            r = r * (1 << a.bucket_bits) // slots
        return r

    os_ = torch.argsort(home(SK))
    og = torch.argsort(home(GK))
    variants = {"random": (SK, SV, SL, GK), "sorted": (SK[os_].contiguous(), SV[os_].contiguous(), SL[os_].contiguous(),
                                                        GK[og].contiguous())}
    kvs = KvStreams(32, 32)
    s_status = torch.empty(ns, dtype=torch.int32, device="cuda")
    g_status = torch.empty(ng, dtype=torch.int32, device="cuda")
    g_lens = torch.empty(ng, dtype=torch.int32, device="cuda")
    gout = torch.empty((ng, 256), dtype=torch.uint8, device="cuda")
    res = {k: [] for k in variants}
    bad = {k: 0 for k in variants}
    for r in range(a.rounds):
        for name, (sk, sv, sl, gk) in variants.items():
            kvs.step(arena, sk, sv, sl, s_status, gk, gout, g_lens, g_status)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                kvs.step(arena, sk, sv, sl, s_status, gk, gout, g_lens, g_status)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / a.steps)
            bad[name] += int((s_status != 0).sum()) + int((g_status != 0).sum())
    for name, ts in res.items():
        ts = sorted(ts)
        print(json.dumps({"order": name, "bucket_bits": a.bucket_bits, "ms_per_step_median": ts[len(ts) // 2],
                          "ms_best": ts[0], "ops_per_s": a.batch / (ts[len(ts) // 2] / 1e3),
                          "nonzero_status": bad[name]}), flush=True)
    kvs.close()
    arena.close()


if __name__ == "__main__":
    main()

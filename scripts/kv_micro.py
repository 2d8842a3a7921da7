#!/usr/bin/env python3
"""Micro-benchmark of the HBM arena kernels: set-only, get-only and concurrent
set||get batches on a prepopulated arena."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=100_000_000)
    ap.add_argument("--batch", type=int, default=4_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--value-len", type=int, default=150)
    ap.add_argument("--kstride", type=int, default=16)
    args = ap.parse_args()
    import torch
    from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values

    a = HbmArena.create(f"micro{os.getpid()}", slots=2 * args.keys, max_val=256, embeddings=False)
    a.store.set_mop(0)
    chunk = 1 << 24
    t0 = time.time()
    for first in range(0, args.keys, chunk):
        n = min(chunk, args.keys - first)
        K = format_keys(n, "k", 10, args.kstride, first=first)
        V, L = format_values(n, 1, args.value_len, 256, first=first)
        st = a.set(K, V, L)
        assert int((st != 0).sum()) == 0
    torch.cuda.synchronize()
    fill = time.time() - t0
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    ids = torch.randint(0, args.keys, (args.batch,), device="cuda", generator=g)
    K = format_keys(args.batch, "k", 10, args.kstride, ids=ids)
    V, L = format_values(args.batch, 2, args.value_len, 256, ids=ids)
    out = torch.empty((args.batch, 256), dtype=torch.uint8, device="cuda")

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return min(ts), sorted(ts)[len(ts) // 2]

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def both():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            a.set(K, V, L)
        with torch.cuda.stream(s2):
            a.get(K, out=out)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    res = {"keys": args.keys, "batch": args.batch,
           "fill_s": round(fill, 3)}
    for name, fn in [("set", lambda: a.set(K, V, L)), ("get", lambda: a.get(K, out=out)), ("set||get", both)]:
        mn, med = timeit(fn)
        ops = args.batch * (2 if name == "set||get" else 1)
        res[name + "_ms"] = round(med, 3)
        res[name + "_Mops"] = round(ops / med / 1e3, 1)
    st, o, ln = a.get(K[:1000])
    res["check_ok"] = bool((st == 0).all().item())
    print(json.dumps(res), flush=True)
    a.close()


if __name__ == "__main__":
    main()

"""Characterise the RCCL all_to_all_single corruption past 768 MiB (profiles/r1_routed_integrity.md).

Questions the round-1 verdict asked:
  * is the limit in BYTES or in ELEMENTS (the same byte sizes as uint8 / int32 / int64 tensors)?
  * where exactly does it start (bisection of the failing size), and what is wrong past it
    (zeros / stale / shifted data)?
  * is it the single-call all_to_all_single path only (grouped send/recv of the same bytes)?
  * does gloo on the same host buffers agree (the reference result)?

One GPU, world 1 (RCCL's self-send path, as the round-1 evidence):
  python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 dev/debug/a2a_rootcause.py
Prints one JSON line per case.
"""
import json
import os

import torch
import torch.distributed as dist


def pattern(nbytes, dtype, dev):
    n = nbytes // torch.tensor([], dtype=dtype).element_size()
    x = torch.arange(n, device=dev, dtype=torch.int64) * 2654435761 + 12345
    return x.to(dtype) if dtype != torch.uint8 else (x & 0xFF).to(torch.uint8)


def check(tag, y, x, extra=None):
    yb, xb = y.view(torch.uint8), x.view(torch.uint8)
    diff = yb != xb
    nbad = int(diff.sum())
    rec = {"case": tag, "bytes": xb.numel(), "elems": x.numel(), "dtype": str(x.dtype).replace("torch.", ""),
           "bad_bytes": nbad}
    if nbad:
        first = int(torch.nonzero(diff)[0].item())
        rec["first_bad"] = first
        tail = yb[first:]
        rec["tail_zero_frac"] = round(float((tail == 0).float().mean()), 4)
        # is the tail a copy of an earlier part of the input (an offset wrap)?
        probe = tail[:4096]
        for shift in (first, 1 << 30, 1 << 31, 768 << 20, 512 << 20):
            src = first - shift
            if 0 <= src and src + probe.numel() <= xb.numel() and torch.equal(xb[src:src + probe.numel()], probe):
                rec["tail_equals_input_at"] = src
                break
    if extra:
        rec.update(extra)
    print(json.dumps(rec), flush=True)
    return nbad


def main():
    dev = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    assert dist.get_world_size() == 1, "run with one rank: the self-send path of the round-1 evidence"
    MiB = 1 << 20
    # 1) bytes or elements: 1.5 GiB as uint8 / int32 / int64
    for dtype in (torch.uint8, torch.int32, torch.int64):
        x = pattern(1536 * MiB, dtype, "cuda")
        y = torch.empty_like(x)
        dist.all_to_all_single(y, x)
        torch.cuda.synchronize()
        check("a2a_single", y, x)
        del x, y
    # 2) bisect the failing byte size (uint8) between 1 GiB (exact in round 1) and 1.5 GiB
    lo, hi = 1024 * MiB, 1536 * MiB
    x = pattern(hi, torch.uint8, "cuda")
    while hi - lo > MiB:
        mid = (lo + hi) // 2 // MiB * MiB
        y = torch.empty(mid, dtype=torch.uint8, device="cuda")
        dist.all_to_all_single(y, x[:mid])
        torch.cuda.synchronize()
        bad = int((y != x[:mid]).sum())
        if bad:
            hi = mid
        else:
            lo = mid
        del y
    print(json.dumps({"case": "bisect_uint8", "largest_exact_bytes": lo, "smallest_bad_bytes": hi}), flush=True)
    # 3) same bytes through the grouped send/recv all_to_all (list form)
    y = torch.empty_like(x)
    dist.all_to_all([y], [x])
    torch.cuda.synchronize()
    check("a2a_list_grouped", y, x)
    # 4) uneven splits (the _route path): one destination, explicit split sizes
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x, [x.numel()], [x.numel()])
    torch.cuda.synchronize()
    check("a2a_single_explicit_splits", y, x)
    del y
    # 5) the chunked fix of parallel/sharded.py
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from libsplinter_amd.parallel.sharded import _Coll
    y = torch.empty_like(x)
    _Coll(None).all_to_all(y, x)
    torch.cuda.synchronize()
    check("sharded_chunked", y, x)
    y = torch.empty_like(x)
    _Coll(None).all_to_all(y, x, [x.numel()], [x.numel()])
    torch.cuda.synchronize()
    check("sharded_chunked_uneven", y, x)
    del x, y
    dist.destroy_process_group()
    # 6) gloo on host buffers of the same size (reference behaviour)
    os.environ["MASTER_PORT"] = str(int(os.environ.get("MASTER_PORT", "29500")) + 1)
    dist.init_process_group("gloo")
    xh = pattern(1536 * MiB, torch.uint8, "cpu")
    yh = torch.empty_like(xh)
    dist.all_to_all_single(yh, xh)
    check("gloo_a2a_single", yh, xh)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

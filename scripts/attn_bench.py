"""A/B the attention kernels (interleaved rounds, one process), random data.

python scripts/attn_bench.py [--docs 64] [--seq 512]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=64)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch
    from libsplinter_amd.models.nomic import Batch, _chk, _lib, _stream
    L = _lib()
    b128 = Batch([[0] * a.seq for _ in range(a.docs)])
    qkv = torch.randn(b128.T_pad, 3 * 768, device="cuda").bfloat16()
    out = torch.empty(b128.T_pad, 768, device="cuda", dtype=torch.bfloat16)
    cur = {"v": 13}

    def run():
        b = b128
        _chk(L.nomic_attention(qkv.data_ptr(), out.data_ptr(), b.cu.data_ptr(), b.qblocks.data_ptr(), b.nqb, 12,
                               0.125, _stream()), "attn")

    VARIANTS = tuple(int(v) for v in os.environ.get("ATTN_VARIANTS", "13,6").split(","))
    times = {v: [] for v in VARIANTS}
    for _ in range(a.rounds):
        for v in VARIANTS:
            L.nomic_attention_set_variant(v)
            cur["v"] = v
            run()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                run()
            e.record()
            torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / a.iters)
    L.nomic_attention_set_variant(13)
    fl = 4.0 * a.docs * a.seq * a.seq * 64 * 12
    for v in VARIANTS:
        t = np.array(times[v])
        print(json.dumps({"kernel": f"attn_v{v}", "docs": a.docs, "seq": a.seq, "ms_median": float(np.median(t)),
                          "tflops_median": fl / np.median(t) / 1e9, "tflops_best": fl / t.min() / 1e9}))


if __name__ == "__main__":
    main()

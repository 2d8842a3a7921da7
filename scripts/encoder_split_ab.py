"""A/B the encoder's document-group split (NOMIC_SPLIT: each group's layer chain on its own stream) on
the bench shape (64 x 512 tokens, 12 layers), interleaved rounds in one process.

python scripts/encoder_split_ab.py [--parts 1,2,3,4] [--rounds 7]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", default="1,2,3,4")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--docs", type=int, default=64)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--vary", type=int, default=0)
    a = ap.parse_args()
    import numpy as np
    import torch
    from libsplinter_amd.models.nomic import Batch, NomicConfig, NomicEncoder, NomicWeights, random_weights
    cfg = NomicConfig()
    w = NomicWeights.from_numpy(cfg, random_weights(cfg, seed=0))
    rng = np.random.default_rng(1)
    lens = rng.integers(a.seq // 2, a.seq + 1, size=a.docs) if a.vary else np.full(a.docs, a.seq)
    b = Batch([rng.integers(1000, cfg.vocab, size=int(n)).tolist() for n in lens])
    enc = NomicEncoder(w, max_tokens=b.T_pad)
    parts = [int(p) for p in a.parts.split(",")]
    tt = {p: [] for p in parts}
    outs = {}
    for r in range(a.rounds):
        for p in parts:
            enc.split_parts = p
            enc.hidden(b)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                enc.hidden(b)
            e1.record()
            torch.cuda.synchronize()
            tt[p].append(e0.elapsed_time(e1) / 5)
            if r == 0:
                outs[p] = enc.hidden(b).float().clone()
    for p in parts:
        d = (outs[p] - outs[parts[0]]).abs().max().item()
        print(json.dumps({"parts": p, "ms_median": float(np.median(tt[p])), "ms_best": float(np.min(tt[p])),
                          "max_abs_diff_vs_first": d, "tokens": int(b.T)}), flush=True)


if __name__ == "__main__":
    main()

"""A/B the persistent register-epilogue GEMM (NOMIC_GEMM 300, gemm_pt.hip) against the launch-per-tile
256^2 kernel (256) on the encoder's K = 768 shapes, interleaved rounds in one process (guide §5.4 rule
24), random operands; then the 12-layer 64 x 512 forward with each.

python scripts/gemm_pt_ab.py [--tokens 32768] [--rounds 7]
One JSON line per (shape, variant): median / best microseconds and TFLOP/s.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="256,300")
    ap.add_argument("--encoder", type=int, default=1)
    ap.add_argument("--ksweep", type=int, default=0, help="also time plain-store GEMMs at K = 768, 1536, 3072 "
                    "(N = 6144): per-tile overhead vs K-loop time of each variant")
    a = ap.parse_args()
    import numpy as np
    import torch
    from libsplinter_amd.models.nomic import _chk, _lib, _stream, pack_qkv, pack_upgate
    L = _lib()
    M, d, F = a.tokens, 768, 3072
    torch.manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1)  # noqa: E731
    x = rnd(M, d).bfloat16()
    wqkv = pack_qkv((rnd(3 * d, d) * 0.05).bfloat16())
    wug = pack_upgate((rnd(F, d) * 0.05).bfloat16(), (rnd(F, d) * 0.05).bfloat16())
    tab = torch.randn(8192, 64, device="cuda")
    inv = 1000.0 ** (-np.arange(0, 64, 2) / 64)
    ang = np.arange(8192)[:, None] * inv[None, :]
    tab = torch.from_numpy(np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32).reshape(8192, -1)).cuda()
    pos = (torch.arange(M, device="cuda", dtype=torch.int32) % 512).contiguous()
    qkv = torch.empty(M, 3 * d, device="cuda", dtype=torch.bfloat16)
    ffn = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    shapes = {
        "qkv_rope": (lambda: L.nomic_gemm(3, x.data_ptr(), d, wqkv.data_ptr(), d, M, 3 * d, d, qkv.data_ptr(), 3 * d,
                                           None, 0, tab.data_ptr(), pos.data_ptr(), 2 * d, _stream()), 2 * M * d * 3 * d),
        "upgate_swiglu": (lambda: L.nomic_gemm(2, x.data_ptr(), d, wug.data_ptr(), d, M, 2 * F, d, ffn.data_ptr(), F,
                                                None, 0, None, None, 0, _stream()), 2 * M * d * 2 * F),
    }
    if a.ksweep:
        for kk in (768, 1536, 3072):
            xk = rnd(M, kk).bfloat16()
            wk = (rnd(6144, kk) * 0.05).bfloat16()
            ok = torch.empty(M, 6144, device="cuda", dtype=torch.bfloat16)
            shapes[f"store_k{kk}"] = ((lambda xk=xk, wk=wk, ok=ok, kk=kk: L.nomic_gemm(
                0, xk.data_ptr(), kk, wk.data_ptr(), kk, M, 6144, kk, ok.data_ptr(), 6144, None, 0, None, None, 0,
                _stream())), 2 * M * kk * 6144)
    variants = [int(v) for v in a.variants.split(",")]
    res = {(s, v): [] for s in shapes for v in variants}
    for r in range(a.rounds):
        for sname, (fn, flops) in shapes.items():
            for v in variants:
                L.nomic_gemm_set_variant(v)
                _chk(fn(), sname)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[(sname, v)].append(e0.elapsed_time(e1) * 1e3 / a.iters)
    for (sname, v), ts in res.items():
        flops = shapes[sname][1]
        print(json.dumps({"shape": sname, "variant": v, "tokens": M, "median_us": float(np.median(ts)),
                          "best_us": float(np.min(ts)), "tflops_median": flops / np.median(ts) / 1e6}), flush=True)
    if a.encoder:
        from libsplinter_amd.models.nomic import Batch, NomicConfig, NomicEncoder, NomicWeights, random_weights
        cfg = NomicConfig()
        w = NomicWeights.from_numpy(cfg, random_weights(cfg, seed=0))
        rng = np.random.default_rng(1)
        b = Batch([rng.integers(1000, cfg.vocab, size=512).tolist() for _ in range(64)])
        enc = NomicEncoder(w, max_tokens=b.T_pad)
        outs = {}
        tt = {v: [] for v in variants}
        for r in range(a.rounds):
            for v in variants:
                L.nomic_gemm_set_variant(v)
                enc.hidden(b)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    enc.hidden(b)
                e1.record()
                torch.cuda.synchronize()
                tt[v].append(e0.elapsed_time(e1) / 5)
                outs[v] = enc.hidden(b).float().clone()
        for v in variants:
            diff = (outs[v] - outs[variants[0]]).norm().item() / outs[variants[0]].norm().item()
            print(json.dumps({"encoder_ms_median": float(np.median(tt[v])), "encoder_ms_best": float(np.min(tt[v])),
                              "variant": v, "rel_diff_vs_first": diff, "flops": enc.flops(b),
                              "tflops": enc.flops(b) / np.median(tt[v]) / 1e9}), flush=True)


if __name__ == "__main__":
    main()

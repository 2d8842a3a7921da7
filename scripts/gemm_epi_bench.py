"""A/B the encoder GEMM epilogues: plain modes vs the LayerNorm-fold / statistics modes
(nomic_api.h 5-8) on the encoder's shapes, interleaved rounds in one process, plus the LayerNorm
and row-statistics kernels the fold replaces / adds.

python scripts/gemm_epi_bench.py [--tokens 32768] [--rounds 7]
One JSON line per (shape, mode): median / best microseconds.
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
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch
    from libsplinter_amd.models.nomic import _chk, _lib, _stream, fold_ln, pack_qkv, pack_upgate
    L = _lib()
    M, d, F = a.tokens, 768, 3072
    torch.manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1)  # noqa: E731
    h = (rnd(M, d) * 2).bfloat16()
    x = rnd(M, d).bfloat16()
    attn = rnd(M, d).bfloat16()
    ffn_in = rnd(M, F).bfloat16()
    g = (1 + 0.2 * rnd(d)).bfloat16()
    b = (0.1 * rnd(d)).bfloat16()
    wqkv = pack_qkv((rnd(3 * d, d) * 0.05).bfloat16())
    wug = pack_upgate((rnd(F, d) * 0.05).bfloat16(), (rnd(F, d) * 0.05).bfloat16())
    wo = (rnd(d, d) * 0.05).bfloat16()
    wd = (rnd(d, F) * 0.05).bfloat16()
    wqkv_f, qc1, qc2 = fold_ln(wqkv, g, b)
    wug_f, uc1, uc2 = fold_ln(wug, g, b)
    part = torch.empty(M, 2 * (d // 128), device="cuda")
    v = h.float().reshape(M, -1, 128)
    mu = v.mean(2)
    ph = torch.stack([mu, ((v - mu[..., None]) ** 2).sum(2)], 2).reshape(M, -1).contiguous()
    st_out = torch.empty(M, 2, device="cuda")
    rope = torch.randn(8192, 64, device="cuda")
    pos = torch.randint(0, 512, (M,), device="cuda", dtype=torch.int32)
    qkv = torch.empty(M, 3 * d, device="cuda", dtype=torch.bfloat16)
    ffn = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(M, d, device="cuda", dtype=torch.bfloat16)
    P = lambda t: t.data_ptr() if t is not None else None  # noqa: E731

    def gemm(mode, A, W, o, res=None, s=None, c1=None, c2=None, ln=False, pt=None):
        N, K = W.shape
        _chk(L.nomic_gemm_ln(mode, A.data_ptr(), A.stride(0), W.data_ptr(), K, M, N, K, o.data_ptr(), o.stride(0),
                             P(res), res.stride(0) if res is not None else 0, rope.data_ptr(), pos.data_ptr(), 2 * d,
                             P(s), d // 128 if s is not None else 0, 1e-12, P(c1), P(c2), P(g) if ln else None,
                             P(b) if ln else None, P(pt), _stream()), f"mode {mode}")

    cases = {
        ("qkv", "rope"): lambda: gemm(3, x, wqkv, qkv),
        ("qkv", "rope_fold"): lambda: gemm(5, h, wqkv_f, qkv, s=ph, c1=qc1, c2=qc2),
        ("o_proj", "residual"): lambda: gemm(1, attn, wo, out, res=x),
        ("o_proj", "res_stats"): lambda: gemm(7, attn, wo, out, res=x, pt=part),
        ("o_proj", "res_ln_stats"): lambda: gemm(8, attn, wo, out, res=h, s=ph, ln=True, pt=part),
        ("upgate", "swiglu"): lambda: gemm(2, x, wug, ffn),
        ("upgate", "swiglu_fold"): lambda: gemm(6, h, wug_f, ffn, s=ph, c1=uc1, c2=uc2),
        ("down", "residual"): lambda: gemm(1, ffn_in, wd, out, res=x),
        ("down", "res_ln_stats"): lambda: gemm(8, ffn_in, wd, out, res=h, s=ph, ln=True, pt=part),
        ("ln", "layernorm"): lambda: _chk(L.nomic_layernorm(h.data_ptr(), M, g.data_ptr(), b.data_ptr(), 1e-12,
                                                            x.data_ptr(), _stream()), "ln"),
        ("ln", "row_stats"): lambda: _chk(L.nomic_row_stats(part.data_ptr(), d // 128, M, 1e-12, st_out.data_ptr(),
                                                            _stream()), "row_stats"),
    }
    times = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, fn in cases.items():
            fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / a.iters * 1e3)
    for (shape, mode), t in times.items():
        t = np.array(t)
        print(json.dumps({"shape": shape, "mode": mode, "M": M, "us_median": round(float(np.median(t)), 2),
                          "us_best": round(float(t.min()), 2)}))


if __name__ == "__main__":
    main()

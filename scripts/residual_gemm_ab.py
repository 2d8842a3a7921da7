"""Post-LN layers of the encoder (o-proj K 768, down K 3072; N 768, M tokens), three ways, interleaved
rounds in one process on random data:

  fused_rln       nomic_gemm_res_ln: GEMM + residual + LayerNorm in one row-complete kernel (shipped)
  split           nomic_gemm EPI_RESIDUAL (MFMA) then the nomic_layernorm kernel
  hipblaslt_ln    torch addmm_ (hipBLASLt, beta = 1 in place) then nomic_layernorm -- a VALIDATION
                  BASELINE only (the round-2 default); no product path calls it

One JSON line per (shape, impl): median / min microseconds and TFLOP/s of the GEMM part.
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
    ap.add_argument("--no-blas", action="store_true")
    ap.add_argument("--rln-variants", default="11", help="comma list of nomic_gemm_res_ln variants "
                    "(PIPE*10 + EPI, csrc/hip/gemm_rln.hip) timed as separate arms")
    ap.add_argument("--ks", default="", help="comma list of K values to time instead of the o-proj / down shapes "
                    "(per-tile fixed cost = intercept of time vs K)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from libsplinter_amd.models.nomic import _chk, _lib, _stream
    L = _lib()
    M = a.tokens
    torch.manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1)  # noqa: E731
    cases = {}
    shapes = [(f"k{k}", int(k)) for k in a.ks.split(",")] if a.ks else [("o_proj", 768), ("down", 3072)]
    for name, K in shapes:
        A = rnd(M, K).bfloat16()
        W = (rnd(768, K) * (1.0 / K ** 0.5)).bfloat16()
        x0 = rnd(M, 768).bfloat16()
        g = (1 + 0.2 * rnd(768)).bfloat16()
        b = (0.1 * rnd(768)).bfloat16()
        bufs = {k: x0.clone() for k in ("fused", "split", "blas")}
        h = torch.empty_like(x0)

        def fused(A=A, W=W, x=bufs["fused"], g=g, b=b, K=K):
            _chk(L.nomic_gemm_res_ln(A.data_ptr(), K, W.data_ptr(), K, M, 768, K, x.data_ptr(), 768, g.data_ptr(),
                                     b.data_ptr(), 1e-12, x.data_ptr(), 768, _stream()), "rln")

        def split(A=A, W=W, x=bufs["split"], h=h, g=g, b=b, K=K):
            _chk(L.nomic_gemm(1, A.data_ptr(), K, W.data_ptr(), K, M, 768, K, h.data_ptr(), 768, x.data_ptr(), 768,
                              None, None, 0, _stream()), "gemm")
            _chk(L.nomic_layernorm(h.data_ptr(), M, g.data_ptr(), b.data_ptr(), 1e-12, x.data_ptr(), _stream()), "ln")

        def blas(A=A, W=W, x=bufs["blas"], g=g, b=b):
            x.addmm_(A, W.t())
            _chk(L.nomic_layernorm(x.data_ptr(), M, g.data_ptr(), b.data_ptr(), 1e-12, x.data_ptr(), _stream()), "ln")

        impls = {}
        for v in [int(x) for x in a.rln_variants.split(",")]:
            def fv(v=v, fused=fused):
                prev = L.nomic_gemm_res_ln_set_variant(v)
                fused()
                L.nomic_gemm_res_ln_set_variant(prev)
            impls[f"fused_rln_v{v}"] = fv
        impls["split"] = split
        if not a.no_blas:
            impls["hipblaslt_ln"] = blas
        ref = torch.nn.functional.layer_norm(A.float() @ W.float().T + x0.float(), (768,), g.float(), b.float(),
                                             1e-12)
        for tag, fn in impls.items():
            key = "fused" if tag.startswith("fused") else {"split": "split", "hipblaslt_ln": "blas"}[tag]
            bufs[key].copy_(x0)
            fn()
            torch.cuda.synchronize()
            got = bufs[key]
            err = ((got.float() - ref).norm() / ref.norm()).item()
            print(json.dumps({"shape": name, "impl": tag, "rel_err": round(err, 6)}), flush=True)
            cases[(name, K, tag)] = fn
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
    for (shape, K, impl), t in times.items():
        t = np.array(t)
        print(json.dumps({"shape": shape, "impl": impl, "M": M, "K": K, "us_median": round(float(np.median(t)), 2),
                          "us_min": round(float(t.min()), 2),
                          "gemm_tflops": round(2.0 * M * 768 * K / np.median(t) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()

"""Residual projections of the encoder (o-proj K 768, down K 3072; N 768, M tokens): our MFMA kernel
with the fused residual epilogue vs hipBLASLt's own beta = 1 epilogue (x += A W^T in place, a plain
library GEMM), interleaved rounds in one process, random data.  One JSON line per (shape, impl).
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
    from libsplinter_amd.models.nomic import _chk, _lib, _stream
    L = _lib()
    M = a.tokens
    torch.manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1)  # noqa: E731
    cases = {}
    for name, K in (("o_proj", 768), ("down", 3072)):
        A = rnd(M, K).bfloat16()
        W = (rnd(768, K) * 0.05).bfloat16()
        x = rnd(M, 768).bfloat16()
        h = torch.empty_like(x)
        xx = x.clone()

        def ours(A=A, W=W, x=x, h=h, K=K):
            _chk(L.nomic_gemm(1, A.data_ptr(), K, W.data_ptr(), K, M, 768, K, h.data_ptr(), 768, x.data_ptr(), 768,
                              None, None, 0, _stream()), "gemm")

        def blas_inplace(A=A, W=W, xx=xx):
            xx.addmm_(A, W.t())

        cases[(name, "mfma_residual_epilogue")] = ours
        cases[(name, "hipblaslt_addmm_inplace")] = blas_inplace
        # numerics: one application each from the same x
        ours()
        y = x.clone()
        y.addmm_(A, W.t())
        ref = x.float() + A.float() @ W.float().T
        for tag, got in (("ours", h), ("blas", y)):
            err = ((got.float() - ref).norm() / ref.norm()).item()
            print(json.dumps({"shape": name, "impl": tag, "rel_err": err}), flush=True)
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
    for (shape, impl), t in times.items():
        t = np.array(t)
        K = 768 if shape == "o_proj" else 3072
        print(json.dumps({"shape": shape, "impl": impl, "M": M, "us_median": round(float(np.median(t)), 2),
                          "tflops": round(2.0 * M * 768 * K / np.median(t) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()

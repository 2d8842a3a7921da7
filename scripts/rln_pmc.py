"""Drive one post-LN implementation (scripts/residual_gemm_ab.py names) at the encoder's shapes for
rocprofv3 --pmc passes: python scripts/rln_pmc.py --impl v30|blas --iters 10."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", default="v30")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tokens", type=int, default=32768)
    a = ap.parse_args()
    import torch
    from libsplinter_amd.models.nomic import _chk, _lib, _stream
    L = _lib()
    M = a.tokens
    rnd = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1)  # noqa: E731
    for K in (768, 3072):
        A = rnd(M, K).bfloat16()
        W = (rnd(768, K) * (1.0 / K ** 0.5)).bfloat16()
        x = rnd(M, 768).bfloat16()
        g = (1 + 0.2 * rnd(768)).bfloat16()
        b = (0.1 * rnd(768)).bfloat16()
        for _ in range(a.iters):
            if a.impl == "blas":
                x.addmm_(A, W.t())
                _chk(L.nomic_layernorm(x.data_ptr(), M, g.data_ptr(), b.data_ptr(), 1e-12, x.data_ptr(), _stream()), "ln")
            else:
                L.nomic_gemm_res_ln_set_variant(int(a.impl[1:]))
                _chk(L.nomic_gemm_res_ln(A.data_ptr(), K, W.data_ptr(), K, M, 768, K, x.data_ptr(), 768, g.data_ptr(),
                                         b.data_ptr(), 1e-12, x.data_ptr(), 768, _stream()), "rln")
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()

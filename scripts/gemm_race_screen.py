"""Race screen of a GEMM main-loop variant: the same operands through the reference schedule and the
variant, many launches, outputs compared BITWISE (both accumulate every output in the same MFMA order,
so any difference is a synchronisation error, not rounding).

python scripts/gemm_race_screen.py [--runs 30] [--knob pp]
One JSON line per shape: runs, mismatching runs, max |diff|.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=30)
    ap.add_argument("--knob", default="pp", choices=["pp", "as128", "rln", "variant"])
    ap.add_argument("--value", type=int, default=1, help="knob setting screened against 0")
    a = ap.parse_args()
    import torch
    from libsplinter_amd.models.nomic import _chk, _lib, _stream
    L = _lib()
    base = {"pp": 0, "as128": 0, "rln": 222, "variant": 512}[a.knob]
    set_knob = {"pp": L.nomic_gemm_set_pp, "as128": L.nomic_gemm_set_as128,
                "rln": L.nomic_gemm_res_ln_set_variant, "variant": L.nomic_gemm_set_variant}[a.knob]
    torch.manual_seed(5)
    # (name, mode, M, N, K): the encoder's SwiGLU shape, a partial row tile, a long K, the qkv shape
    shapes = [("ffn_swiglu", 2, 32768, 6144, 768), ("swiglu_tail", 2, 5000, 2048, 768),
              ("store_k3072", 0, 4096, 1024, 3072), ("qkv_store", 0, 32768, 2304, 768)]
    if a.knob == "rln":  # mode -1: the row-complete residual + LayerNorm kernel (N = 768)
        shapes = [("o_proj", -1, 32768, 768, 768), ("down", -1, 32768, 768, 3072), ("tail", -1, 4100, 768, 3072)]
    pv = L.nomic_gemm_set_variant(128 if a.knob == "as128" else 256)
    pp_prev = L.nomic_gemm_set_pp(2)
    try:
        for name, mode, M, N, K in shapes:
            A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
            W = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
            nout = N // 2 if mode == 2 else N
            ref = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
            out = torch.empty_like(ref)
            R = torch.randn(M, N, device="cuda").bfloat16()
            g = (1 + 0.3 * torch.randn(N, device="cuda")).bfloat16()
            b = (0.1 * torch.randn(N, device="cuda")).bfloat16()

            def run(o):
                if mode < 0:
                    _chk(L.nomic_gemm_res_ln(A.data_ptr(), K, W.data_ptr(), K, M, N, K, R.data_ptr(), N, g.data_ptr(),
                                             b.data_ptr(), 1e-12, o.data_ptr(), N, _stream()), name)
                else:
                    _chk(L.nomic_gemm(mode, A.data_ptr(), K, W.data_ptr(), K, M, N, K, o.data_ptr(), nout, None, 0,
                                      None, None, 0, _stream()), name)

            set_knob(base)
            run(ref)
            set_knob(a.value)
            bad, worst = 0, 0.0
            for _ in range(a.runs):
                out.fill_(0)
                run(out)
                torch.cuda.synchronize()
                if not torch.equal(out, ref):
                    bad += 1
                    worst = max(worst, (out.float() - ref.float()).abs().max().item())
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "knob": a.knob, "value": a.value, "runs": a.runs,
                              "mismatching_runs": bad, "max_abs_diff": worst}), flush=True)
            del A, W, ref, out
    finally:
        set_knob(base if a.knob == "rln" else (2 if a.knob == "pp" else 0))
        L.nomic_gemm_set_variant(pv)
        L.nomic_gemm_set_pp(pp_prev)


if __name__ == "__main__":
    main()

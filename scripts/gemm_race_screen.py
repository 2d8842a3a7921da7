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
    ap.add_argument("--knob", default="pp", choices=["pp"])
    a = ap.parse_args()
    import torch
    from libsplinter_amd.models.nomic import _chk, _lib, _stream
    L = _lib()
    set_knob = {"pp": L.nomic_gemm_set_pp}[a.knob]
    torch.manual_seed(5)
    # (name, mode, M, N, K): the encoder's SwiGLU shape, a partial row tile, a long K, the qkv shape
    shapes = [("ffn_swiglu", 2, 32768, 6144, 768), ("swiglu_tail", 2, 5000, 2048, 768),
              ("store_k3072", 0, 4096, 1024, 3072), ("qkv_store", 0, 32768, 2304, 768)]
    pv = L.nomic_gemm_set_variant(256)
    try:
        for name, mode, M, N, K in shapes:
            A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
            W = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
            nout = N // 2 if mode == 2 else N
            ref = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
            out = torch.empty_like(ref)

            def run(o):
                _chk(L.nomic_gemm(mode, A.data_ptr(), K, W.data_ptr(), K, M, N, K, o.data_ptr(), nout, None, 0,
                                  None, None, 0, _stream()), name)

            set_knob(0)
            run(ref)
            set_knob(1)
            bad, worst = 0, 0.0
            for _ in range(a.runs):
                out.fill_(0)
                run(out)
                torch.cuda.synchronize()
                if not torch.equal(out, ref):
                    bad += 1
                    worst = max(worst, (out.float() - ref.float()).abs().max().item())
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "knob": a.knob, "runs": a.runs,
                              "mismatching_runs": bad, "max_abs_diff": worst}), flush=True)
            del A, W, ref, out
    finally:
        L.nomic_gemm_set_variant(pv)
        set_knob(0)


if __name__ == "__main__":
    main()

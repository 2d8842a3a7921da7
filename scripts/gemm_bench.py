"""A/B the two GEMM kernels on the encoder's shapes (interleaved rounds, one process).

python scripts/gemm_bench.py [--tokens 32768] [--rounds 5]
Prints one JSON line per (shape, variant) with median / min TFLOP/s on random data.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--square", type=int, default=0, help="also time a plain MxNxK = S x S x S GEMM (loop throughput)")
    ap.add_argument("--variants", default="514,512,513,256,128", help="NOMIC_GEMM kernel variants")
    ap.add_argument("--ilvs", default="0", help="DMA interleave settings of the 256^2 kernels (nomic_gemm_set_ilv)")
    ap.add_argument("--shapes", default="", help="comma list of shape names (default: all)")
    ap.add_argument("--as128", default="0", help="asm LDS-DMA in the 128^2 kernel (nomic_gemm_set_as128)")
    ap.add_argument("--pps", default="0", help="ping-pong main loop of the 256^2 kernel (nomic_gemm_set_pp)")
    ap.add_argument("--sregs", default="1", help="register SwiGLU epilogue of the 256^2 kernel (nomic_gemm_set_swiglu_reg)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from libsplinter_amd.models.nomic import _chk, _lib, _stream
    L = _lib()
    M = a.tokens
    torch.manual_seed(0)
    shapes = [("qkv_rope", 3, 2304, 768), ("attn_out_res", 1, 768, 768), ("ffn_swiglu", 2, 6144, 768),
              ("ffn_down_res", 1, 768, 3072)]
    if a.shapes:
        shapes = [sh for sh in shapes if sh[0] in a.shapes.split(",")]
    if a.square:
        shapes = [("square", 0, a.square, a.square)]
        M = a.square
    bufs = {}
    for name, mode, N, K in shapes:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        W = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
        nout = N // 2 if mode == 2 else N
        out = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
        res = torch.randn(M, nout, device="cuda").bfloat16() if mode == 1 else None
        rope = torch.randn(8192, 64, device="cuda") if mode == 3 else None
        pos = torch.randint(0, 512, (M,), device="cuda", dtype=torch.int32) if mode == 3 else None
        bufs[name] = (mode, N, K, A, W, out, res, rope, pos)

    def run(name):
        mode, N, K, A, W, out, res, rope, pos = bufs[name]
        _chk(L.nomic_gemm(mode, A.data_ptr(), K, W.data_ptr(), K, M, N, K, out.data_ptr(), out.shape[1],
                          None if res is None else res.data_ptr(), 0 if res is None else res.shape[1],
                          None if rope is None else rope.data_ptr(), None if pos is None else pos.data_ptr(),
                          1536, _stream()), name)

    ilvs = [int(x) for x in a.ilvs.split(",")]
    sregs = [int(x) for x in a.sregs.split(",")]
    pps = [int(x) for x in a.pps.split(",")]
    VARS = [(int(v), il, sr, pp) for v in a.variants.split(",") for il in (ilvs if int(v) in (256, 512) else [0])
            for sr in (sregs if int(v) == 256 else [1]) for pp in (pps if int(v) == 256 else
                                                                     [int(x) for x in a.as128.split(",")] if int(v) == 128
                                                                     else [0])]
    times = {(n, v): [] for n, *_ in shapes for v in VARS}
    for r in range(a.rounds):
        for name, *_ in shapes:
            for v in VARS:
                L.nomic_gemm_set_variant(v[0])
                L.nomic_gemm_set_ilv(v[1])
                L.nomic_gemm_set_swiglu_reg(v[2])
                if v[0] == 128:
                    L.nomic_gemm_set_as128(v[3])
                else:
                    L.nomic_gemm_set_pp(v[3])
                run(name)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    run(name)
                e.record()
                torch.cuda.synchronize()
                times[(name, v)].append(s.elapsed_time(e) / a.iters)
    # library reference point: hipBLASLt via torch.matmul (plain GEMM, no fused epilogue)
    ref = {}
    for name, mode, N, K in shapes:
        A, W = bufs[name][3], bufs[name][4]
        torch.matmul(A, W.T)
        ts = []
        for _ in range(a.rounds):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                torch.matmul(A, W.T)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / a.iters)
        ref[name] = float(np.median(ts))
    for name, mode, N, K in shapes:
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "variant": "torch.matmul(hipBLASLt)",
                          "ms_median": ref[name], "tflops_median": fl / ref[name] / 1e9}))
        for v in VARS:
            t = np.array(times[(name, v)])
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "variant": v[0], "ilv": v[1], "swiglu_reg": v[2], "pp": v[3],
                              "ms_median": float(np.median(t)),
                              "tflops_median": fl / np.median(t) / 1e9, "tflops_best": fl / t.min() / 1e9}))


if __name__ == "__main__":
    main()

"""Microbenchmark of the per-token decode kernels at llama-7B shapes: dec_attn_decode over cache
lengths (H 32, KVH 8, hd 128) and dec_sample over vocabulary sizes, flat (random-init-like) and
spread logits.  One JSON line per case: microseconds per call (median of 5 rounds x 200 calls)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from libsplinter_amd.models.decoder import CausalLM, DecoderConfig  # noqa: E402

m = CausalLM.random(DecoderConfig(layers=1), seed=1, device="cuda")
L_ = m.L
H, KVH, hd = 32, 8, 128


def timeit(fn, n=200, rounds=5):
    out = []
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) / n * 1e3)
    return sorted(out)[len(out) // 2]


g = torch.Generator(device="cuda").manual_seed(0)
for L in (16, 128, 512, 2048, 8192):
    q = torch.randn(H * hd, device="cuda", generator=g).to(torch.bfloat16)
    k = torch.randn((L, KVH * hd), device="cuda", generator=g).to(torch.bfloat16)
    v = torch.randn((L, KVH * hd), device="cuda", generator=g).to(torch.bfloat16)
    o = torch.empty(H * hd, device="cuda", dtype=torch.bfloat16)
    us = timeit(lambda: L_.dec_attn_decode(q.data_ptr(), k.data_ptr(), v.data_ptr(), KVH * hd, L, H, KVH, hd,
                                           hd ** -0.5, o.data_ptr(), None))
    print(json.dumps({"kernel": "dec_attn_decode", "L": L, "H": H, "KVH": KVH, "hd": hd, "us": us,
                      "kv_GB_per_s": 2 * L * KVH * hd * 2 / (us * 1e-6) / 1e9}), flush=True)
if "--attn-only" in sys.argv:
    sys.exit(0)
st = torch.zeros(4, dtype=torch.int32, device="cuda")
for V in (32000, 128256):
    for kind, scale in (("flat", 0.05), ("spread", 4.0)):
        lg = (torch.randn(V, device="cuda", generator=g) * scale).float()
        us = timeit(lambda: L_.dec_sample(lg.data_ptr(), V, None, 0.9, 0.7, 1234, st.data_ptr(), 0, None, None))
        print(json.dumps({"kernel": "dec_sample", "V": V, "logits": kind, "us": us}), flush=True)
        ws = torch.empty(L_.dec_sample_ws_floats(), dtype=torch.float32, device="cuda")
        us = timeit(lambda: L_.dec_sample_ws(lg.data_ptr(), V, None, 0.9, 0.7, 1234, st.data_ptr(), 0, None,
                                             ws.data_ptr(), None))
        print(json.dumps({"kernel": "dec_sample_ws (64-block chain)", "V": V, "logits": kind, "us": us}), flush=True)

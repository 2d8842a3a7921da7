"""Per-token decode latency of the splainference decoder with bf16 vs 4-bit (Q4G32) weights.

Llama-7B-shaped layers (d 4096, 32 heads, 8 kv heads, ffn 11008, vocab 32000) with --layers layers,
random init.  Each token is one replay of the DecodeEngine HIP graph (all GEMVs, RoPE + KV append,
decode attention, sampler).  Prints one JSON line per quant: ms/token and the projection bytes
streamed per token divided by the step time (the decode step is weight-bandwidth bound)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from libsplinter_amd.models.decoder import CausalLM, DecodeEngine, DecoderConfig, Q4Weight  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layers", type=int, default=4)
ap.add_argument("--prompt", type=int, default=128)
ap.add_argument("--tokens", type=int, default=64)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
cfg = DecoderConfig(vocab=32000, d=4096, layers=a.layers, heads=32, kv_heads=8, ffn=11008,
                    n_ctx=a.prompt + a.rounds * (a.tokens + 8) + 16)


def weight_bytes(m):
    ws = [m.head] + [lw[k] for lw in m.layers for k in ("qkv", "o", "ug", "down")]
    return sum(w.nbytes() if isinstance(w, Q4Weight) else w.numel() * w.element_size() for w in ws)


engines = {}
for q in ("bf16", "q4"):
    t0 = time.time()
    m = CausalLM.random(cfg, seed=0, device="cuda", quant=q)
    engines[q] = (DecodeEngine(m, seed=7, use_graph=True), weight_bytes(m))
    print(f"[decode_q4_bench] {q} model built in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
prompt = [1] + [100 + i % 200 for i in range(a.prompt - 1)]
res = {q: [] for q in engines}
toks = {}
for r in range(a.rounds):
    for q, (eng, nb) in engines.items():
        toks[q] = [eng.first_token(prompt)]
        for _ in range(4):
            toks[q].append(eng.next_token())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.tokens):
            toks[q].append(eng.next_token())
        res[q].append((time.perf_counter() - t0) / a.tokens * 1e3)
for q, (eng, nb) in engines.items():
    ms = sorted(res[q])[len(res[q]) // 2]
    print(json.dumps({"quant": q, "ms_per_token_median": ms, "ms_per_token_all": res[q],
                      "weight_GB": nb / 1e9, "weight_TB_per_s": nb / (ms * 1e-3) / 1e12, "layers": a.layers,
                      "d": cfg.d, "ffn": cfg.ffn, "vocab": cfg.vocab, "ctx": a.prompt, "first_tokens": toks[q][:8]}),
          flush=True)

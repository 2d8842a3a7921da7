"""Per-token decode latency of the splainference decoder: dec_attn_decode vs torch SDPA (A/B).

Random-init 7B-shaped layers are too big for a quick A/B, so this uses the default DecoderConfig
with --layers layers, prefills --prefill tokens, then times --steps single-token decode steps."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from libsplinter_amd.models.decoder import CausalLM, DecoderConfig

ap = argparse.ArgumentParser()
ap.add_argument("--layers", type=int, default=4)
ap.add_argument("--prefill", type=int, default=1024)
ap.add_argument("--steps", type=int, default=128)
ap.add_argument("--kv-heads", type=int, default=8)
a = ap.parse_args()
cfg = DecoderConfig(layers=a.layers, kv_heads=a.kv_heads, n_ctx=a.prefill + a.steps + 8)
m = CausalLM.random(cfg, seed=0, device="cuda")
res = {}
for mode in (False, True, False, True):
    m.attn_kernel = mode
    m.reset()
    m.forward([1] * a.prefill)
    for _ in range(4):
        m.forward([65])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        m.forward([65])
    torch.cuda.synchronize()
    res["kernel" if mode else "sdpa"] = (time.perf_counter() - t0) / a.steps * 1e3
print(json.dumps({"ms_per_token": res, "layers": a.layers, "ctx": a.prefill, "d": cfg.d, "heads": cfg.heads,
                  "kv_heads": a.kv_heads}))

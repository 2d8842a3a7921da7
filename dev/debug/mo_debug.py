import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values
a = HbmArena.create(f"dbg{os.getpid()}", slots=1 << 22, max_val=256, embeddings=False)
a.store.set_mop(0)
n = 1 << 20
K = format_keys(n, "k", 10, 16)
V, L = format_values(n, 1, 150, 256)
st = a.set(K, V, L, retries=64)
torch.cuda.synchronize()
u, c = torch.unique(st, return_counts=True)
print("MO", os.environ.get("SPLINTER_ARENA_MO"), "insert status", dict(zip(u.tolist(), c.tolist())), "stats", a.stats.tolist())
st2, out, ol = a.get(K)
u, c = torch.unique(st2, return_counts=True)
print("get status", dict(zip(u.tolist(), c.tolist())))
bad = (st != 0).nonzero().flatten()[:5].tolist()
print("bad idx", bad, [bytes(K[i].cpu().numpy()).rstrip(b'\0') for i in bad])
a.close()

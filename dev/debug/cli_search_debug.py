#!/usr/bin/env python3
"""Step-by-step check of the CLI against an hbm: store owned by this process (debug aid)."""
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from libsplinter_amd.ops.arena import HbmArena, format_keys, pack_values  # noqa: E402

name = f"clidbg{os.getpid()}"
a = HbmArena.create(name, slots=int(sys.argv[1]) if len(sys.argv) > 1 else 4096, max_val=64, embeddings=True)
env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
cli = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "libsplinter_amd", "bin", "splinterctl")
n = 1000
K = format_keys(n, "doc", 6, 16)
V, L = pack_values([b"text"] * n, 16)
a.set(K, V, L)
a.set_embeddings(K, torch.randn(n, 768, device="cuda"))
torch.cuda.synchronize()
for args in (["get", "doc000001"], ["set", "k1", "v1"], ["label", "k1", "1"], ["bump", "k1"], ["list"],
             ["search", "--json", "--timeout", "3000", "--limit", "3", "probe"]):
    t0 = time.time()
    try:
        r = subprocess.run([cli, "-u", f"hbm:{name}", *args], capture_output=True, text=True, timeout=60, env=env)
        print(args[0], "rc", r.returncode, f"{time.time() - t0:.2f}s", r.stdout[:200].replace("\n", " | "),
              "ERR:", r.stderr[-300:], flush=True)
    except subprocess.TimeoutExpired:
        print(args[0], "TIMEOUT", flush=True)
        break
a.close()

#!/usr/bin/env python3
"""Time a second process attaching an hbm: arena of N slots (debug aid for large IPC imports)."""
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402,F401
from libsplinter_amd.ops.arena import HbmArena  # noqa: E402

slots = int(sys.argv[1])
name = f"ipcdbg{os.getpid()}"
a = HbmArena.create(name, slots=slots, max_val=64, embeddings=True)
gb = (5440 + slots * (3200 + 64)) / 2**30
code = f"""
import time, faulthandler, sys
faulthandler.dump_traceback_later(40, exit=True)
t0 = time.time()
import torch
sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))!r})
from libsplinter_amd import _native as N
import ctypes
L = N.core_lib()
t1 = time.time()
err = ctypes.c_int(0)
h = L.spl_store_open(b"hbm:{name}", ctypes.byref(err))
t2 = time.time()
print("open", bool(h), err.value, f"import {{t1-t0:.2f}}s open {{t2-t1:.2f}}s", flush=True)
"""
env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
t0 = time.time()
try:
    r = subprocess.run([sys.executable, "-u", "-c", code], capture_output=True, text=True, timeout=60, env=env)
    print(f"slots {slots} ({gb:.2f} GiB): rc {r.returncode} {time.time() - t0:.1f}s", r.stdout.strip(),
          r.stderr.strip()[-400:], flush=True)
except subprocess.TimeoutExpired:
    print(f"slots {slots} ({gb:.2f} GiB): TIMEOUT", flush=True)
a.close()

#!/usr/bin/env python3
"""Which HIP runtime does a torch process use, and does a second process attach a VMM arena."""
import ctypes
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
v = ctypes.c_int(0)
hip.hipRuntimeGetVersion(ctypes.byref(v))
print("torch process HIP runtime", v.value, torch.version.hip, flush=True)
r = subprocess.run(["bash", "-c", "ldd " + os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                    "libsplinter_amd/bin/splinterctl") + " | grep -i amdhip || true"], capture_output=True, text=True)
print("CLI links:", r.stdout.strip(), flush=True)

"""Does a device-wide synchronize in the store's owner wait for its resident ring-server worker?
Times torch.cuda.synchronize() right after (a) a per-call op of the owner's own thread, (b) per-call
ops of a client process (the worker then launched by the owner's supervisor thread), with the
worker idle timeout given by SPLINTER_RING_IDLE_US.  One JSON line."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from libsplinter_amd import Store  # noqa: E402


def timed_sync():
    t = time.perf_counter()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) * 1e3, 3)


def main():
    name = f"hbm:sp{os.getpid()}"
    st = Store.create(name, slots=4096, max_val=256, embeddings=False)
    out = {"idle_us": os.environ.get("SPLINTER_RING_IDLE_US")}
    try:
        torch.zeros(1, device="cuda")
        torch.cuda.synchronize()
        st.set("k", b"v")
        out["own_op_then_sync_ms"] = timed_sync()
        time.sleep(1.5)
        tool = os.path.join(ROOT, "libsplinter_amd", "bin", "splinter_hostapi_bench")
        p = subprocess.run([tool, "--attach", "--store", name, "--threads", "1", "--seconds", "0.2", "--keys", "1"],
                           capture_output=True, text=True, timeout=60,
                           env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
        out["client_rc"] = p.returncode
        out["client_op_then_sync_ms"] = timed_sync()
        time.sleep(1.5)
        st.set("k", b"v2")
        out["own_op_again_then_sync_ms"] = timed_sync()
    finally:
        st.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

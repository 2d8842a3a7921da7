"""Encoder step time beside per-call clients: one process owns an hbm: store and runs the encoder
(the embedding daemon's work, EmbedPhase 64 x 512) while C clients in other processes hammer the
store's per-call API (splinter_hostapi_bench --attach, 8 threads each).

  shared   the clients submit to the owner's ONE ring server (cmd_ring.hpp RingSegHdr, default)
  private  SPLINTER_RING_SHARED=0 in the clients: each runs its own resident ring worker
  cpu      the same clients on a host shm store (no GPU work at all): the host-side share of the
           slowdown (CPU contention with the encoder's launching thread)
  idle     the clients call for 0.3 s and exit BEFORE the encoder is timed: with
           SPLINTER_RING_IDLE_US set long, the owner's worker stays resident but idle
  held     as shared, with each encoder step inside a ring hold (store.ring_hold: the owner's
           worker is off the GPU during the step; calls wait for the gaps)
--client-args: extra splinter_hostapi_bench arguments (e.g. "--set-frac 0": gets only)

Prints one JSON line: encoder ms/step alone and beside the clients in either mode, the slowdown,
and the clients' aggregate ops/s.

  python scripts/ring_interference.py [--clients 4] [--threads 8] [--steps 20]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from libsplinter_amd import Store  # noqa: E402
from libsplinter_amd import _native as N  # noqa: E402
from libsplinter_amd.models.bench_embed import EmbedPhase  # noqa: E402

TOOL = os.path.join(ROOT, "libsplinter_amd", "bin", "splinter_hostapi_bench")


STEPS = []  # per-step encoder ms of the last time_steps (events on the encoder's stream)


SYNC = {}  # how long the device-wide synchronizes around the last time_steps took (ms)


HOLD = [False, None]  # hold on?, the store to hold (None: this process's rings)


def _step(ph):
    if HOLD[0]:
        from libsplinter_amd.store import ring_hold
        with ring_hold(HOLD[1]):
            ph.run()
            torch.cuda.current_stream().synchronize()
    else:
        ph.run()


_OWNER = r"""
import sys
from libsplinter_amd import Store
st = Store.create(sys.argv[1], slots=2 * int(sys.argv[2]) + 1024, max_val=4096, embeddings=False)
keys = [f"hk{i:08d}" for i in range(int(sys.argv[2]))]
st.set_batch(keys, [b"v" * 150] * len(keys))
print("ready", flush=True)
sys.stdin.readline()
st.close()
"""


def time_steps(ph, n):
    # stream-level synchronisation only: a device-wide synchronize waits for this process's resident
    # ring worker, which does not idle out while clients call -- it would time the encoder after them
    ts = time.perf_counter()
    torch.cuda.current_stream().synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    t0 = time.perf_counter()
    SYNC["before_ms"] = round((t0 - ts) * 1e3, 3)
    ev[0].record()
    for i in range(n):
        _step(ph)
        ev[i + 1].record()
    ev[n].synchronize()
    t1 = time.perf_counter()
    SYNC["after_ms"] = 0.0
    STEPS[:] = [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(n)]
    return (t1 - t0) / n * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=4)
    ap.add_argument("--threads", default="2,8", help="client threads per process, comma list")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--keys", type=int, default=20000)
    ap.add_argument("--modes", default="shared,private,cpu")
    ap.add_argument("--client-args", default="")
    ap.add_argument("--owner-proc", action="store_true",
                    help="the store (and its ring server) is owned by a separate process; this encoder process "
                         "is one of its clients (held mode then holds the store: ring_hold(store))")
    ap.add_argument("--settle", type=float, default=4.0,
                    help="seconds between starting the clients and timing (their HIP start-up and store attach, "
                         "which maps the arena into their GPU address space, are over by then)")
    a = ap.parse_args()
    name = f"hbm:ri{os.getpid()}"
    owner = None
    if a.owner_proc:
        owner = subprocess.Popen([sys.executable, "-c", _OWNER, name, str(a.keys)], stdin=subprocess.PIPE,
                                 stdout=subprocess.PIPE, text=True, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
        assert owner.stdout.readline().strip() == "ready"
        st = Store.open(name)
        HOLD[1] = st
    else:
        st = Store.create(name, slots=2 * a.keys + 1024, max_val=4096, embeddings=False)
    out = {"clients": a.clients, "cpus": len(os.sched_getaffinity(0)), "owner_ring_mode": N.hip_lib().spl_hbm_ring_mode(st.handle)}
    try:
        keys = [f"hk{i:08d}" for i in range(a.keys)]
        if owner is None:
            status = st.set_batch(keys, [b"v" * 150] * a.keys)
            assert int((status != 0).sum()) == 0
        ph = EmbedPhase(batch=64, seq=512)
        for _ in range(3):
            ph.run()
        out["encoder_ms_alone"] = round(time_steps(ph, a.steps), 3)
        secs = max(3.0, a.steps * out["encoder_ms_alone"] / 1e3 * 3 + 2.0) + a.settle
        shm = f"ri{os.getpid()}shm"
        hs = Store.create(shm, slots=2 * a.keys + 1024, max_val=4096, embeddings=False)
        hs.set_batch(keys, [b"v" * 150] * a.keys)
        for threads in [int(t) for t in a.threads.split(",")]:
            for mode in a.modes.split(","):
                env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0",
                           SPLINTER_RING_SHARED="0" if mode == "private" else "1")
                target = shm if mode == "cpu" else name
                dur = 0.3 if mode == "idle" else secs
                procs = [subprocess.Popen([TOOL, "--attach", "--store", target, "--threads", str(threads), "--seconds",
                                           str(dur), "--keys", str(a.keys)] + a.client_args.split(), env=env,
                                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                         for _ in range(a.clients)]
                HOLD[0] = mode == "held"
                try:
                    if mode == "idle":
                        for p in procs:
                            p.wait(timeout=120)
                    else:
                        time.sleep(a.settle)  # the clients are attached and calling
                    n0 = N.hip_lib().spl_hbm_ring_launches(st.handle)
                    ms = time_steps(ph, a.steps)
                    launches = N.hip_lib().spl_hbm_ring_launches(st.handle) - n0
                    rate, fails, modes = 0.0, 0, []
                    for p in procs:
                        o, e = p.communicate(timeout=secs + 60)
                        if p.returncode != 0:
                            fails += 1
                            print(e[-500:], file=sys.stderr)
                            continue
                        c, ok, f, el, p50 = o.split()[:5]
                        modes.append(int(o.split()[5]) if len(o.split()) > 5 else None)
                        rate += int(c) / float(el)
                        fails += int(f)
                finally:
                    HOLD[0] = False
                    for p in procs:
                        if p.poll() is None:
                            p.kill()
                out[f"{mode}_t{threads}"] = {"encoder_ms": round(ms, 3),
                                             "slowdown_pct": round(100.0 * (ms / out["encoder_ms_alone"] - 1), 2),
                                             "client_ops_per_s": round(rate, 1), "client_failures": fails,
                                             "worker_launches_while_timed": launches, "client_ring_modes": modes,
                                             "step_ms": STEPS[:], "device_sync_ms": dict(SYNC)}
                print(json.dumps(out), file=sys.stderr, flush=True)
        out["encoder_ms_alone_after"] = round(time_steps(ph, a.steps), 3)
        ph.close()
        hs.close()
        from libsplinter_amd import store as S
        S.unlink(shm)
    finally:
        st.close()
        if owner is not None:
            owner.stdin.write("done\n")
            owner.stdin.flush()
            owner.wait(timeout=60)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Per-call API of hbm: stores through the device command ring (csrc/hip/cmd_ring.hip):
latency / throughput from host threads, atomic device append, device-side BIGUINT promotion,
and the event bus waking a separate process on batched device writes."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")


def _hostapi(store, threads, seconds=1.0, append=0):
    tool = os.path.join(ROOT, "libsplinter_amd", "bin", "splinter_hostapi_bench")
    cmd = [tool, "--store", store, "--threads", str(threads), "--seconds", str(seconds), "--keys", "20000"]
    if append:
        cmd += ["--append-check", str(append)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=ENV)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(res))
    return res


def test_hostapi_single_thread_latency(uniq):
    res = _hostapi(f"hbm:{uniq}", 1)
    assert res["failures"] == 0
    assert res["p50_us"] < 100.0  # ring round trip, not a launch + sync per call


def test_hostapi_many_threads_and_concurrent_append(uniq):
    """16 host threads: no failures, and 16 x 16 concurrent appends to one key all land, each
    thread's records in its own order (append holds the slot seqlock on the device)."""
    res = _hostapi(f"hbm:{uniq}", 16, append=16)
    assert res["failures"] == 0 and res["append_check"] == 1
    assert res["ops_per_s"] > 100_000


def test_append_semantics_on_hbm(uniq):
    from libsplinter_amd import Store
    s = Store.create(f"hbm:{uniq}", slots=256, max_val=64, embeddings=False)
    try:
        s.set("log", b"abc")
        assert s.append("log", b"def") == 6
        assert s.get("log") == b"abcdef"
        with pytest.raises(OSError):
            s.append("log", b"x" * 60)  # EMSGSIZE: 6 + 60 > 64
        assert s.get("log") == b"abcdef"
        with pytest.raises(OSError):
            s.append("missing", b"x")
        e0 = s.epoch("log")
        s.append("log", b"!")
        assert s.epoch("log") == e0 + 2
    finally:
        s.close()


def test_biguint_promotion_on_device(uniq):
    """reference splinter.c:637-680: a short value becomes a u64 -- ASCII parsed with
    strtoull(.., 0) (decimal / 0x hex / 0 octal), other bytes taken raw (little endian)."""
    from libsplinter_amd import Store
    s = Store.create(f"hbm:{uniq}", slots=256, max_val=64, embeddings=False)
    try:
        cases = {"dec": (b"41", 41), "hex": (b"0x1f", 31), "oct": (b"017", 15), "raw": (b"\x05\x01", 0x0105)}
        for k, (v, want) in cases.items():
            s.set(k, v)
            s.set_type(k, 1 << 2)
            assert s.get_u64(k) == want, k
            assert s.integer_op(k, 4, 1) == want + 1  # INC
        s.set("long", b"123456789")  # >= 8 bytes: left as is, only the type changes
        s.set_type("long", 1 << 2)
        assert s.get("long") == b"123456789"
    finally:
        s.close()


def test_header_ops_through_ring(uniq):
    from libsplinter_amd import Store
    s = Store.create(f"hbm:{uniq}", slots=256, max_val=64, embeddings=False)
    try:
        assert s.get_mop() == 1
        s.set_mop(0)
        assert s.get_mop() == 0
        s.set_mop(2)
        assert s.get_mop() == 2
        h = s.header()
        assert h["slots"] == 256 and h["max_val_sz"] == 64
        s.set("a", "1")
        assert s.watch_label(1 << 3, 7)
        s.set_label("a", 1 << 3)
        c0 = s.signal_count(7)
        s.bump("a")
        assert s.signal_count(7) == c0 + 1
    finally:
        s.close()


_WAITER = r"""
import sys, time
from libsplinter_amd import Store
s = Store.open(sys.argv[1])
s.event_bus_init()
fd = s.event_bus_open()
print("ready", flush=True)
ok = Store.event_bus_wait(fd, 20000)
print("woke" if ok else "timeout", flush=True)
print("dirty", sum(bin(w).count("1") for w in s.dirty_mask()), flush=True)
"""


def test_event_bus_wakes_other_process_on_batched_device_write(uniq):
    """A separate process owns the event bus and blocks in splinter_event_bus_wait; THIS process
    writes a key with a batched set kernel (no per-call API): the kernel's notify store reaches
    the owner's proxy thread, which signals the eventfd; the dirty mask is marked on the device."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena, pack_keys, pack_values
    arena = HbmArena.create(uniq, slots=4096, max_val=256, embeddings=False)
    K = pack_keys(["evt"], 16)
    V, L = pack_values([b"v0"], 16)
    assert (arena.set(K, V, L) == 0).all()
    torch.cuda.synchronize()
    p = subprocess.Popen([sys.executable, "-c", _WAITER, f"hbm:{uniq}"], cwd=ROOT, env=ENV, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().strip() == "ready"
        time.sleep(0.2)
        V, L = pack_values([b"v1"], 16)
        assert (arena.set(K, V, L) == 0).all()
        torch.cuda.synchronize()
        out, err = p.communicate(timeout=60)
    finally:
        if p.poll() is None:
            p.kill()
        arena.close()
    assert p.returncode == 0, err[-2000:]
    lines = out.split()
    assert lines[0] == "woke", out + err[-1000:]
    assert int(lines[-1]) >= 1


def test_raw_ptr_on_hbm_is_zero_copy(uniq):
    """splinter_get_raw_ptr on an hbm: store returns a pointer INTO the arena (the CPU mapping of
    its dmabuf chunks), as the reference's pointer into shm: a later device write shows through
    the same view, and the epoch moves with it (reference splinter.c:747-762)."""
    from libsplinter_amd import Store
    s = Store.create(f"hbm:{uniq}", slots=512, max_val=256, embeddings=False)
    try:
        s.set("rk", b"hello world")
        got = s.raw("rk")
        assert got is not None
        view, e0 = got
        assert bytes(view) == b"hello world" and e0 == s.epoch("rk")
        s.set("rk", b"HELLO WORLD")  # a device write (command ring kernel)
        assert bytes(view[:11]) == b"HELLO WORLD"  # same memory: zero-copy
        assert s.epoch("rk") == e0 + 2
        assert s.raw("missing") is None
    finally:
        s.close()



def test_ring_worker_idle_exit_and_relaunch(uniq, monkeypatch):
    """With a 2 ms idle timeout the ring worker exits between bursts and the next call (or a waiter
    that sees it gone) relaunches it: calls straddling the idle exit from 8 threads are all served
    with the right values, and spl_hbm_ring_launches counts the relaunches."""
    import random
    import threading
    from libsplinter_amd import Store
    from libsplinter_amd import _native as N
    monkeypatch.setenv("SPLINTER_RING_IDLE_US", "2000")
    s = Store.create(f"hbm:{uniq}", slots=4096, max_val=64, embeddings=False)
    launches = lambda: N.hip_lib().spl_hbm_ring_launches(s.handle)  # noqa: E731
    try:
        s.set("k0", b"v0")
        n0 = launches()
        assert n0 >= 1
        time.sleep(0.05)  # > idle timeout: the worker has left
        assert s.get("k0") == b"v0"
        assert launches() > n0
        errors = []

        def worker(t):
            rng = random.Random(t)
            try:
                for i in range(60):
                    k = f"t{t}_{i}"
                    s.set(k, f"{t}:{i}".encode())
                    if s.get(k) != f"{t}:{i}".encode():
                        errors.append(k)
                    time.sleep(rng.choice((0.0, 0.0005, 0.003, 0.006)))
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        n1 = launches()
        th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join(120)
        assert not errors, errors[:5]
        assert launches() > n1  # the worker idled out and came back during the run
    finally:
        s.close()


def test_hostapi_32_threads(uniq):
    """32 host threads (more than the box's CPU share on a loaded host): every call served."""
    res = _hostapi(f"hbm:{uniq}", 32)
    assert res["failures"] == 0


def test_open_second_store_beside_live_ring_traffic(uniq):
    """Creating another hbm: store on the device while a thread keeps per-call traffic flowing
    through the first store's resident ring worker finishes promptly: store set-up waits only for
    its own stream, never for the device (the worker exits only after SPLINTER_RING_IDLE_US idle)."""
    import threading
    from libsplinter_amd import Store
    a = Store.create(f"hbm:{uniq}a", slots=1024, max_val=64, embeddings=False)
    stop = threading.Event()
    calls = [0]

    def traffic():
        while not stop.is_set():
            a.set("hot", b"x" * 16)
            assert a.get("hot") == b"x" * 16
            calls[0] += 1

    t = threading.Thread(target=traffic)
    t.start()
    try:
        time.sleep(0.2)
        t0 = time.perf_counter()
        b = Store.create(f"hbm:{uniq}b", slots=1024, max_val=64, embeddings=False)
        b.set("k", b"v")
        assert b.get("k") == b"v"
        dt = time.perf_counter() - t0
        b.close()
    finally:
        stop.set()
        t.join(30)
        a.close()
    assert calls[0] > 100
    assert dt < 5.0, f"second store took {dt:.2f}s beside live traffic"


_CLIENT = r"""
import sys
from libsplinter_amd import Store
from libsplinter_amd import _native as N
s = Store.open(sys.argv[1])
mode = N.hip_lib().spl_hbm_ring_mode(s.handle)
for i in range(200):
    s.set(f"c{i}", f"child{i}".encode())
for i in range(300):
    s.integer_op("ctr", 4, 1)
print(mode, s.get("o5").decode(), flush=True)
if len(sys.argv) > 2:  # keep calling after the owner closed the store
    print("ready", flush=True)
    sys.stdin.readline()
    s.set("after", b"owner-gone")
    print(s.get("after").decode(), flush=True)
s.close()
"""


def test_ring_server_shared_by_processes(uniq):
    """The store's owner hosts ONE ring server (mode 1); a second process submits its per-call ops
    to it (mode 2, no worker of its own): its sets are visible to the owner, and 300 + 300
    concurrent device increments from both processes all land."""
    from libsplinter_amd import Store
    from libsplinter_amd import _native as N
    s = Store.create(f"hbm:{uniq}", slots=4096, max_val=64, embeddings=False)
    try:
        assert N.hip_lib().spl_hbm_ring_mode(s.handle) == 1
        s.set("ctr", b"0")
        s.set_type("ctr", 1 << 2)
        for i in range(10):
            s.set(f"o{i}", f"owner{i}".encode())
        p = subprocess.Popen([sys.executable, "-c", _CLIENT, f"hbm:{uniq}"], cwd=ROOT, env=ENV,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        try:
            for i in range(300):
                s.integer_op("ctr", 4, 1)
            out, err = p.communicate(timeout=90)
        finally:
            if p.poll() is None:
                p.kill()
        assert p.returncode == 0, err[-2000:]
        mode, o5 = out.split()[:2]
        assert mode == "2" and o5 == "owner5"
        assert s.get_u64("ctr") == 600
        assert all(s.get(f"c{i}") == f"child{i}".encode() for i in range(200))
    finally:
        s.close()


def test_ring_client_survives_owner_close(uniq):
    """A client whose owner closed the store falls back to a private ring worker on its own
    import of the arena: later calls still work."""
    from libsplinter_amd import Store
    s = Store.create(f"hbm:{uniq}", slots=4096, max_val=64, embeddings=False)
    s.set("ctr", b"0")
    s.set_type("ctr", 1 << 2)
    s.set("o5", b"owner5")
    p = subprocess.Popen([sys.executable, "-c", _CLIENT, f"hbm:{uniq}", "stay"], cwd=ROOT, env=ENV,
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().split() == ["2", "owner5"]
        assert p.stdout.readline().strip() == "ready"
        s.close()
        s = None
        p.stdin.write("go\n")
        p.stdin.flush()
        out, err = p.communicate(timeout=90)
    finally:
        if p.poll() is None:
            p.kill()
        if s is not None:
            s.close()
    assert p.returncode == 0, err[-2000:]
    assert out.strip() == "owner-gone"


def test_hostapi_four_processes_one_server(uniq):
    """4 processes x 8 threads against one hbm: store: every call served by the owner's one ring
    server (the children are its clients)."""
    tool = os.path.join(ROOT, "libsplinter_amd", "bin", "splinter_hostapi_bench")
    r = subprocess.run([tool, "--store", f"hbm:{uniq}", "--procs", "4", "--threads", "8", "--seconds", "1.0",
                        "--keys", "20000"], capture_output=True, text=True, timeout=150, env=ENV)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(res))
    assert res["failures"] == 0 and res["ring_mode"] == 1 and len(res["procs_p50_us"]) == 4


_HOLD_CLIENT = r"""
import sys, time
from libsplinter_amd import Store
s = Store.open(sys.argv[1])
print("ready", flush=True)
sys.stdin.readline()
t = time.perf_counter()
s.set("held", b"after-hold")
print(round((time.perf_counter() - t) * 1e3, 1), flush=True)
s.close()
"""


def test_ring_hold_defers_calls_until_release(uniq):
    """store.ring_hold in the owner: no ring worker runs inside the block, a client's call waits
    and is served once the hold ends; the owner's own calls work again afterwards."""
    from libsplinter_amd import Store
    from libsplinter_amd.store import ring_hold
    s = Store.create(f"hbm:{uniq}", slots=1024, max_val=64, embeddings=False)
    p = subprocess.Popen([sys.executable, "-c", _HOLD_CLIENT, f"hbm:{uniq}"], cwd=ROOT, env=ENV,
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        s.set("pre", b"1")
        assert p.stdout.readline().strip() == "ready"
        with ring_hold():
            p.stdin.write("go\n")
            p.stdin.flush()
            time.sleep(0.4)
            assert p.poll() is None  # the client's set is still waiting
        out, err = p.communicate(timeout=60)
        assert p.returncode == 0, err[-2000:]
        assert float(out.strip()) >= 300.0
        assert s.get("held") == b"after-hold"
        s.set("post", b"2")
        assert s.get("post") == b"2"
    finally:
        if p.poll() is None:
            p.kill()
        s.close()


_STORE_HOLDER = r"""
import sys, time
from libsplinter_amd import Store
from libsplinter_amd.store import ring_hold
s = Store.open(sys.argv[1])
with ring_hold(s):
    print("held", flush=True)
    time.sleep(0.5)
print("released", flush=True)
s.close()
"""


def test_store_ring_hold_from_another_process(uniq):
    """ring_hold(store) in a client process stops the OWNER's ring worker for that store: the
    owner's own per-call op waits until the client releases, then completes."""
    from libsplinter_amd import Store
    s = Store.create(f"hbm:{uniq}", slots=1024, max_val=64, embeddings=False)
    p = subprocess.Popen([sys.executable, "-c", _STORE_HOLDER, f"hbm:{uniq}"], cwd=ROOT, env=ENV,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        s.set("pre", b"1")
        assert p.stdout.readline().strip() == "held"
        t = time.perf_counter()
        s.set("during", b"2")  # waits for the release (~0.5 s)
        dt = time.perf_counter() - t
        out, err = p.communicate(timeout=60)
        assert p.returncode == 0, err[-2000:]
        assert out.strip() == "released"
        assert dt >= 0.3, dt
        assert s.get("during") == b"2"
    finally:
        if p.poll() is None:
            p.kill()
        s.close()


_BUSY_OWNER = r"""
import sys
from libsplinter_amd import Store
s = Store.create(sys.argv[1], slots=4096, max_val=64, embeddings=False)
s.set("o", b"owner")
print("ready", flush=True)
sys.stdin.readline()
s.close()
print("closed", flush=True)
"""

_BUSY_CLIENT = r"""
import sys, time
from libsplinter_amd import Store
s = Store.open(sys.argv[1])
print("running", flush=True)
t_end = time.time() + float(sys.argv[2])
n = bad = err = 0
while time.time() < t_end:
    k = f"c{n % 64}"
    v = f"v{n}".encode()
    try:
        s.set(k, v)
        if s.get(k) != v:
            bad += 1
    except OSError:
        err += 1  # a call in flight when the server vanished fails (EIO); the next one fails over
    n += 1
print(n, bad, err, flush=True)
s.close()
"""


def test_owner_close_while_client_is_calling(uniq):
    """The owner closes the store while a client process is issuing per-call ops through the owner's
    ring server: the owner's teardown completes (it stops its supervisor before taking the quiesce
    gate, so a supervisor woken by the client cannot block it), and the client's calls fall over to
    a private worker with every set read back intact."""
    name = f"hbm:{uniq}"
    own = subprocess.Popen([sys.executable, "-c", _BUSY_OWNER, name], cwd=ROOT, env=ENV, stdin=subprocess.PIPE,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    cli = None
    try:
        assert own.stdout.readline().strip() == "ready"
        cli = subprocess.Popen([sys.executable, "-c", _BUSY_CLIENT, name, "4.0"], cwd=ROOT, env=ENV,
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        assert cli.stdout.readline().strip() == "running"
        time.sleep(1.0)  # client traffic in flight on the owner's server
        own.stdin.write("close\n")
        own.stdin.flush()
        out, err = own.communicate(timeout=60)
        assert own.returncode == 0 and out.strip() == "closed", err[-2000:]
        cout, cerr = cli.communicate(timeout=90)
        assert cli.returncode == 0, cerr[-2000:]
        n, bad, err = map(int, cout.split())
        # no wrong bytes ever; at most the few calls in flight at the failover fail (EIO, never
        # retried by the library: a set / get could be, an increment or append could not)
        assert n > 100 and bad == 0 and err <= 4, (n, bad, err)
    finally:
        for p in (own, cli):
            if p is not None and p.poll() is None:
                p.kill()


_DYING_HOLDER = r"""
import os, sys
from libsplinter_amd import Store
from libsplinter_amd.store import ring_hold
s = Store.open(sys.argv[1])
h = ring_hold(s)
h.__enter__()
print("held", flush=True)
os._exit(0)  # dies holding the store's ring
"""


def test_hold_of_a_dead_process_is_taken_back(uniq):
    """A process that dies inside ring_hold(store) leaves its count in the store's hold word; the
    owner's next call finds the holder dead, takes its count back and is served (instead of every
    call on the store timing out)."""
    from libsplinter_amd import Store
    s = Store.create(f"hbm:{uniq}", slots=1024, max_val=64, embeddings=False)
    try:
        s.set("pre", b"1")
        r = subprocess.run([sys.executable, "-c", _DYING_HOLDER, f"hbm:{uniq}"], cwd=ROOT, env=ENV,
                           capture_output=True, text=True, timeout=90)
        assert r.stdout.strip() == "held", r.stderr[-2000:]
        t = time.perf_counter()
        s.set("after", b"2")
        assert time.perf_counter() - t < 10.0
        assert s.get("after") == b"2"
    finally:
        s.close()

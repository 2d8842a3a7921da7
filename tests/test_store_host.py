"""Host (shm/file) backend through the Python bindings + the native TAP suite."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from libsplinter_amd import Store, SplinterBusy, SplinterError, unlink
from libsplinter_amd import _native as N
from libsplinter_amd import store as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_tap_suite():
    exe = os.path.join(ROOT, "libsplinter_amd", "bin", "splinter_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "not ok" not in r.stdout


def test_native_tap_suite_on_node_store_of_shm_shards():
    """The same 134-check suite through a node store ("node:", 8 shm shards): routing, replicated
    mop / label map, summed signal counts, merged list / enumerate, node-wide shard bids and the node
    event bus, against the reference semantics (the per-arena capacity checks are skipped)."""
    exe = os.path.join(ROOT, "libsplinter_amd", "bin", "splinter_test")
    env = dict(os.environ, SPLINTER_TEST_PREFIX="node:", SPLINTER_NODE_BACKEND="shm", SPLINTER_NODE_SHARDS="8")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "not ok" not in r.stdout and "# passed 130/130" in r.stdout, r.stdout[-500:]


@pytest.fixture
def store(uniq):
    s = Store.create(uniq, slots=512, max_val=1024, embeddings=True)
    yield s
    s.close()
    unlink(uniq)


def test_roundtrip_and_snapshot(store):
    store.set("a", b"\x00\x01binary")
    assert store.get("a") == b"\x00\x01binary"
    snap = store.snapshot("a")
    assert snap["val_len"] == 8 and snap["key"] == "a" and snap["epoch"] % 2 == 0
    assert store.header()["magic"] == 0x534C4E54
    assert store.get("zz") is None
    with pytest.raises(SplinterError):
        store.set("big", b"x" * 2000)


def test_layout_is_reference_v4(store):
    """Byte-level layout: header fields and slot placement match format v4."""
    store.set("k1", b"v1")
    mv = store.region()
    hdr = np.frombuffer(mv[:64], dtype=np.uint32)
    assert hdr[0] == 0x534C4E54 and hdr[1] == 4 and hdr[2] == 512 and hdr[3] == 1024
    idx = store.find_slot("k1")
    off = 5440 + idx * 3200
    slot = bytes(mv[off: off + 128])
    assert int.from_bytes(slot[:8], "little") == S.hash_key("k1")
    assert slot[64:66] == b"k1"
    voff = 5440 + 512 * 3200 + idx * 1024
    assert bytes(mv[voff: voff + 2]) == b"v1"


def test_fnv1a_matches_reference_definition():
    def fnv(s: bytes):
        h = 14695981039346656037
        for c in s:
            h = ((h ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
        return h
    for k in [b"", b"a", b"test_key", b"k00000001", b"x" * 63]:
        assert S.hash_key(k) == fnv(k)


def test_embeddings_and_retrain(store):
    store.set("d", "doc")
    v = np.random.default_rng(1).standard_normal(768).astype(np.float32)
    store.set_embedding("d", v)
    np.testing.assert_array_equal(store.get_embedding("d"), v)
    assert store.retrain("d") and store.epoch("d") == 4
    assert not store.get_embedding("d").any()


def test_labels_signals_enumerate(store):
    for i in range(5):
        store.set(f"e{i}", "x")
    store.set_label("e1", 1 << 3)
    store.set_label("e4", 1 << 3)
    assert sorted(k for k, _ in store.enumerate(1 << 3)) == ["e1", "e4"]
    store.watch_label(1 << 3, 9)
    c = store.signal_count(9)
    store.bump("e1")
    assert store.signal_count(9) == c + 1


def test_integer_ops(store):
    store.set("n", (10).to_bytes(8, "little"))
    store.set_type("n", S.SLOT_BIGUINT)
    assert store.integer_op("n", S.OP_INC, 5) == 15
    assert store.integer_op("n", S.OP_DEC, 1) == 14
    assert store.integer_op("n", S.OP_XOR, 14) == 0
    store.set("t", "text")
    store.set_type("t", S.SLOT_VARTEXT)
    with pytest.raises(SplinterError):
        store.integer_op("t", S.OP_INC, 1)


def test_shard_election(store):
    far = 1 << 60
    store.shard_claim(0x10, S.INTENT_WILLNEED, 5, far)
    store.shard_claim(0x11, S.INTENT_DONTNEED, 250, far)
    assert store.shard_election() == (0x10, S.INTENT_WILLNEED)
    store.shard_release(0x10)
    assert store.shard_election()[0] == 0x11
    t = store.shard_table()
    assert len(t) == 32 and sum(r["sovereign"] for r in t) == 1
    store.shard_release(0x11)


def test_two_stores_in_one_process(uniq):
    a = Store.create(uniq + "A", 64, 64, embeddings=False)
    b = Store.create(uniq + "B", 64, 64, embeddings=False)
    try:
        a.set("x", "in-a")
        b.set("x", "in-b")
        assert a.get("x") == b"in-a" and b.get("x") == b"in-b"
    finally:
        a.close(); b.close(); unlink(uniq + "A"); unlink(uniq + "B")


def test_cross_process_visibility(uniq):
    s = Store.create(uniq, 128, 128, embeddings=False)
    try:
        code = ("import sys; sys.path.insert(0, %r)\n"
                "from libsplinter_amd import Store\n"
                "s = Store.open(%r); s.set('from_child', 'hi'); print(s.get('parent').decode())\n") % (ROOT, uniq)
        s.set("parent", "p-value")
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        assert r.stdout.strip() == "p-value"
        assert s.get("from_child") == b"hi"
    finally:
        s.close(); unlink(uniq)


def test_open_rejects_garbage(tmp_path):
    p = tmp_path / "junk"
    p.write_bytes(b"\0" * 8192)
    with pytest.raises(SplinterError):
        Store.open(str(p))


def test_watchdog_stuck_writer_host(store):
    import ctypes
    store.set("victim", "data")
    i = store.find_slot("victim")
    assert i >= 0 and store.stuck_slots(hold_ms=1) == []
    reg = store.region()
    off = 5440 + i * store.stride + 8
    ep = ctypes.c_uint64.from_buffer(reg, off)
    ep.value |= 1  # writer "crashed" mid-write
    assert store.stuck_slots(hold_ms=5) == [i]
    assert store.retrain("victim")
    assert store.stuck_slots(hold_ms=1) == [] and store.epoch("victim") == 4


def test_list_copy_for_ffi_bindings(store):
    """spl_list_copy backs the TS binding's list() (bindings/ts/splinter.ts)."""
    import ctypes
    from libsplinter_amd import _native as N
    for k in ("k1", "key_two"):
        store.set(k, "v")
    store.use()
    L = N.core_lib()
    L.spl_list_copy.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    L.spl_list_copy.restype = ctypes.c_long
    need = -L.spl_list_copy(None, 0)
    buf = ctypes.create_string_buffer(need)
    n = L.spl_list_copy(buf, need)
    assert n == need and sorted(buf.raw[:n].split(b"\0")[:-1]) == [b"k1", b"key_two"]


def test_hostapi_bench_reports_cpu_per_call(uniq):
    """splinter_hostapi_bench on a shm store: every call succeeds, and the JSON line carries the
    process CPU accounting of the timed window (user / system seconds, CPU us per call)."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tool = os.path.join(root, "libsplinter_amd", "bin", "splinter_hostapi_bench")
    r = subprocess.run([tool, "--store", uniq, "--threads", "4", "--seconds", "0.3", "--keys", "2000"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["failures"] == 0 and res["calls"] > 0
    assert res["cpu_usr_s"] + res["cpu_sys_s"] > 0 and res["cpu_us_per_call"] > 0

"""Node stores of HBM shards on one GPU (4 shards on device 0), through the C ABI.

The 8-GPU node runs one shard per GPU; on the 1-GPU lease every shard sits on device 0 and the
same NodeStore code (csrc/core/node_store.cpp) routes per-call ops to each shard's command ring,
sums signal counts, merges list / enumerate, merges the per-shard device search, and the
data-parallel splinference (one daemon per shard, owner computes) embeds every shard's keys.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def hbm_node(uniq, monkeypatch):
    monkeypatch.setenv("SPLINTER_NODE_BACKEND", "hbm")
    monkeypatch.setenv("SPLINTER_NODE_SHARDS", "4")
    import torch  # noqa: F401  (HIP runtime order)
    from libsplinter_amd import store as S
    s = S.Store.create(f"node:{uniq}", slots=4 * 4096, max_val=4096, embeddings=True)
    yield S, s, uniq
    s.close()


def test_node_hbm_kv_signals_and_list(hbm_node):
    S, s, name = hbm_node
    assert s.backend == "node" and s.nshards == 4
    assert all(s.shard(i).backend == "hbm" for i in range(4))
    keys = [f"k{i}" for i in range(300)]
    for k in keys:
        s.set(k, f"value of {k}".encode())
    assert s.get("k123") == b"value of k123"
    assert sorted(s.keys()) == sorted(keys)
    per = [len(s.shard(i).keys()) for i in range(4)]
    assert sum(per) == 300 and min(per) > 30, per
    for i, k in enumerate(keys[:40]):
        assert s.shard(S.node_shard_of(k, 4)).get(k) == f"value of {k}".encode()
    s.watch_label(0x1, 9)
    before = s.signal_count(9)
    for k in keys[:40]:
        assert s.set_label(k, 0x1) and s.bump(k)
    assert s.signal_count(9) - before == 40  # pulses on 4 GPUs' arenas summed (C2)
    assert sorted(k for k, _ in s.enumerate(0x1)) == sorted(keys[:40])
    s.set("n", b"7")
    s.set_type("n", S.SLOT_BIGUINT)
    s.integer_op("n", S.OP_INC, 5)
    assert s.get_u64("n") == 12
    assert s.header()["slots"] == 4 * 4096


def test_node_hbm_cli_and_device_search(hbm_node):
    """splinterctl -u node:NAME from another process (the shards attach through their dmabuf
    chunk servers), and spl_hbm_search over the node (per-shard device scoring, merged top-k)."""
    import ctypes
    from libsplinter_amd import _native as N
    S, s, name = hbm_node
    rng = np.random.default_rng(2)
    vecs = rng.standard_normal((64, 768)).astype(np.float32)
    for i in range(64):
        s.set(f"doc{i}", f"text {i}".encode())
        s.set_embedding(f"doc{i}", vecs[i])
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cli = os.path.join(ROOT, "libsplinter_amd", "bin", "splinterctl")
    r = subprocess.run([cli, "-u", f"node:{name}", "get", "doc17"], capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0 and "text 17" in r.stdout, (r.stdout, r.stderr[-2000:])
    r = subprocess.run([cli, "-u", f"node:{name}", "set", "from_cli", "hello"], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert s.get("from_cli") == b"hello"
    fn = N.hip_lib().spl_hbm_search
    fn.restype = ctypes.c_long
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_float, ctypes.c_float, ctypes.c_long,
                   ctypes.c_void_p]
    q = np.ascontiguousarray(vecs[5] + 0.1 * rng.standard_normal(768).astype(np.float32))
    out = (ctypes.c_uint8 * (96 * 8))()  # spl_search_hit: 96 B
    n = fn(s.handle, q.ctypes.data, 0, 0.0, 0.0, 5, out)
    assert n == 65  # every key with a value: 64 docs + "from_cli"
    first = bytes(out[0:64]).split(b"\0", 1)[0].decode()
    assert first == "doc5"
    sims = vecs @ q / (np.linalg.norm(vecs, axis=1) * np.linalg.norm(q))
    got = [bytes(out[96 * i: 96 * i + 64]).split(b"\0", 1)[0].decode() for i in range(5)]
    assert got == [f"doc{i}" for i in np.argsort(-sims)[:5]]


def test_node_hbm_checkpoint_roundtrip(hbm_node, tmp_path):
    import ctypes
    from libsplinter_amd import _native as N
    S, s, name = hbm_node
    for i in range(100):
        s.set(f"c{i}", f"v{i}".encode())
    L = N.hip_lib()
    L.spl_hbm_checkpoint.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    L.spl_hbm_restore.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    path = str(tmp_path / "node.img")
    assert L.spl_hbm_checkpoint(s.handle, path.encode()) == 0
    assert all(os.path.exists(f"{path}.s{i}") for i in range(4))
    for i in range(100):
        s.unset(f"c{i}")
    assert s.get("c3") is None
    assert L.spl_hbm_restore(s.handle, path.encode()) == 0
    assert s.get("c3") == b"v3" and len([k for k in s.keys() if k.startswith("c")]) == 100


def test_dp_splinference_embeds_every_shard(hbm_node):
    """One daemon per shard (rank 0..3, oneshot), each embedding only its own shard's pending keys
    on its GPU; together they cover the node, and each vector equals the encoder's output for the
    key's text.  Odd ranks embed inside a ring hold of their shard (hold_ring)."""
    import torch
    from libsplinter_amd.daemons.splinference import Splinference, build_encoder
    S, s, name = hbm_node
    texts = {f"doc{i}": f"document {i} about sharded vector stores and gpus" for i in range(48)}
    for k, t in texts.items():
        s.set(k, t.encode())
        s.set_type(k, S.SLOT_VARTEXT)
        s.set_label(k, 0x1 | 0x40)
    enc, tok = build_encoder(None, True, layers=2, max_tokens=1 << 14)
    done = {}
    for r in range(4):
        d = Splinference(s, enc, tok, group=3, rank=r, hold_ring=bool(r & 1))
        assert d.arena is not None  # the shard's batched device path
        d.run(oneshot=True)
        done[r] = d.stats["embedded"]
    owners = [S.node_shard_of(k, 4) for k in texts]
    assert [done[r] for r in range(4)] == [owners.count(r) for r in range(4)], done
    from libsplinter_amd.models.nomic import Batch
    ids, offs, _ = tok.encode_batch([t.encode() for t in texts.values()], 2000)
    ref = enc.embed(Batch([ids[offs[i]: offs[i + 1]] for i in range(len(texts))])).float().cpu().numpy()
    for j, k in enumerate(texts):
        v = s.get_embedding(k)
        assert v is not None and np.linalg.norm(v) > 0, k
        np.testing.assert_allclose(v, ref[j], rtol=2e-2, atol=2e-3)
        assert not (s.snapshot(k)["bloom"] & 0x40)


def test_dp_splinference_cli_on_node(hbm_node):
    """The daemon binary with a node store and --rank: runs on its shard only."""
    S, s, name = hbm_node
    for i in range(16):
        s.set(f"x{i}", f"some text {i}".encode())
        s.set_type(f"x{i}", S.SLOT_VARTEXT)
        s.set_label(f"x{i}", 0x1)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", SPLINTER_NODE_BACKEND="hbm")
    mine = [f"x{i}" for i in range(16) if S.node_shard_of(f"x{i}", 4) == 2]
    r = subprocess.run([sys.executable, "-m", "libsplinter_amd.daemons.splinference", "--oneshot", "--random-init",
                        "--layers", "2", "--rank", "2", f"node:{name}", "none.gguf", "3"], cwd=ROOT,
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "shard 2/4" in r.stderr
    for i in range(16):
        v = s.get_embedding(f"x{i}")
        has = v is not None and float(np.linalg.norm(v)) > 0
        assert has == (f"x{i}" in mine), (i, has)


@pytest.mark.parametrize("prefix,shards", [("hbm:", None), ("node:", "2")], ids=["hbm", "node_hbm"])
def test_native_tap_suite_on_hbm(prefix, shards):
    """The reference-parity TAP suite (tools/splinter_test.cpp, mirroring the reference
    splinter_test.c) on an HBM arena and on a node store of HBM shards, through the C ABI."""
    exe = os.path.join(ROOT, "libsplinter_amd", "bin", "splinter_test")
    env = dict(os.environ, SPLINTER_TEST_PREFIX=prefix, HSA_ENABLE_IPC_MODE_LEGACY="0")
    if shards:
        env.update(SPLINTER_NODE_BACKEND="hbm", SPLINTER_NODE_SHARDS=shards)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    fails = [ln for ln in r.stdout.splitlines() if ln.startswith("not ok")]
    print(r.stdout[-400:])
    assert r.returncode == 0 and not fails, (fails, r.stderr[-2000:])


def test_bench_store_is_a_node_store_the_cli_opens(uniq):
    """bench.py's ranks create their arenas with HbmArena.join_node: the benched store is node
    store node:<tag>kv, so a C-ABI client in another process (splinterctl) reads the keys the
    batch kernels wrote, while the bench's process holds it (reference splinter.c:235-248: every
    process maps the one store)."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values
    a = HbmArena.join_node(f"{uniq}kv", 0, 1, slots=1 << 16, max_val=256, embeddings=False)
    try:
        K = format_keys(1000, "k", 10, 16)
        V, L = format_values(1000, 7, 150, 256)
        assert (a.set(K, V, L) == 0).all()
        torch.cuda.synchronize()
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        cli = os.path.join(ROOT, "libsplinter_amd", "bin", "splinterctl")
        r = subprocess.run([cli, "-u", f"node:{uniq}kv", "get", "k0000000417"], capture_output=True, text=True,
                           timeout=120, env=env)
        assert r.returncode == 0 and "id:417|" in r.stdout, (r.stdout, r.stderr[-2000:])
        # and the batch C ABI over the same node, from this process
        from libsplinter_amd import store as S
        with S.Store.open(f"node:{uniq}kv") as s:
            st, out, ln = s.get_batch([f"k{i:010d}" for i in range(0, 1000, 7)], width=256)
            assert (st == 0).all() and all(b"id:%d|" % i in bytes(out[j, : ln[j]])
                                           for j, i in enumerate(range(0, 1000, 7)))
    finally:
        a.close()
    assert not os.path.exists(f"/dev/shm/{uniq}kv.node")  # the last shard out removed the node

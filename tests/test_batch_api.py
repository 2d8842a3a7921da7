"""The host-array batch C ABI (splinter_ext.h spl_*_batch, csrc/core/batch_host.cpp) on host and
node stores (CPU) and on hbm: / node: stores of HBM shards (GPU): batch results must be the
per-call results, op for op."""
import os

import numpy as np
import pytest


def _check_store(S, s, n=3000):
    keys = [f"bk-{i:06d}" for i in range(n)]
    vals = [f"value-{i}-".encode() * (1 + i % 4) for i in range(n)]
    st = s.set_batch(keys, vals)
    assert (st == 0).all(), np.unique(st, return_counts=True)
    # per-call reads see every batch write
    for i in range(0, n, 97):
        assert s.get(keys[i]) == vals[i]
    # batch reads of per-call writes
    for i in range(0, n, 89):
        s.set(keys[i], b"percall-" + keys[i].encode())
    st, out, ln = s.get_batch(keys + ["missing-key"], width=256)
    assert st[-1] == -2 and ln[-1] == 0
    for i in range(n):
        want = b"percall-" + keys[i].encode() if i % 89 == 0 else vals[i]
        assert st[i] == 0 and bytes(out[i, : ln[i]]) == want, (i, st[i])
    # narrow rows: EMSGSIZE exactly where the value does not fit
    st, out, ln = s.get_batch(keys[:200], width=16)
    for i in range(200):
        want = b"percall-" + keys[i].encode() if i % 89 == 0 else vals[i]
        assert (st[i] == 0) == (len(want) <= 16), (i, st[i], len(want))
    # integer ops: BIGUINT counters
    ctr = [f"ctr-{j}" for j in range(40)]
    for c in ctr:
        s.set(c, (0).to_bytes(8, "little"))
        s.set_type(c, S.SLOT_BIGUINT)
    ops = np.full(400, S.OP_INC, dtype=np.int32)
    st, res = s.integer_op_batch([ctr[i % 40] for i in range(400)], ops, np.ones(400, dtype=np.uint64))
    assert (st == 0).all()
    for c in ctr:
        assert s.get_u64(c) == 10
    st, _ = s.integer_op_batch(keys[:3], np.full(3, S.OP_INC, dtype=np.int32))
    assert (st == -91).all()  # EPROTOTYPE: not BIGUINT
    if s.embeddings:
        vecs = np.random.default_rng(1).standard_normal((50, 768)).astype(np.float32)
        assert (s.set_embedding_batch(keys[:50], vecs) == 0).all()
        np.testing.assert_array_equal(s.get_embedding(keys[7]), vecs[7])


def test_batch_api_host_store():
    from libsplinter_amd import store as S
    name = f"bapi{os.getpid()}"
    s = S.Store.create(name, slots=16384, max_val=256, embeddings=True)
    try:
        _check_store(S, s)
    finally:
        s.close()
        S.unlink(name)


def test_batch_api_node_store_shm(monkeypatch):
    monkeypatch.setenv("SPLINTER_NODE_BACKEND", "shm")
    monkeypatch.setenv("SPLINTER_NODE_SHARDS", "4")
    from libsplinter_amd import store as S
    name = f"bnode{os.getpid()}"
    s = S.Store.create(f"node:{name}", slots=4 * 8192, max_val=256, embeddings=True)
    try:
        _check_store(S, s)
        # every key landed on (only) its owning shard
        for i in range(0, 3000, 211):
            k = f"bk-{i:06d}"
            owner = S.node_shard_of(k, 4)
            with S.Store.open(S.node_shard_name(name, owner, S.NODE_SHM)) as sh:
                assert sh.get(k) is not None
    finally:
        s.close()
        S.unlink(f"node:{name}")


@pytest.mark.gpu
def test_batch_api_hbm_store(uniq):
    from libsplinter_amd import store as S
    s = S.Store.create(f"hbm:{uniq}", slots=16384, max_val=256, embeddings=True)
    try:
        _check_store(S, s)
    finally:
        s.close()
        S.unlink(f"hbm:{uniq}")


@pytest.mark.gpu
def test_batch_api_node_store_hbm(uniq, monkeypatch):
    monkeypatch.setenv("SPLINTER_NODE_SHARDS", "4")
    from libsplinter_amd import store as S
    s = S.Store.create(f"node:{uniq}", slots=4 * 8192, max_val=256, embeddings=True)
    try:
        assert s.nshards == 4
        _check_store(S, s)
    finally:
        s.close()
        S.unlink(f"node:{uniq}")


@pytest.mark.gpu
def test_batch_api_hbm_large_pinned_and_pageable(uniq):
    """A multi-chunk batch (SPLINTER_BATCH_CHUNK_MB small) from pageable numpy arrays and through the
    C tool's pinned arrays: every op lands, reads back intact."""
    import json
    import subprocess
    from libsplinter_amd import store as S
    s = S.Store.create(f"hbm:{uniq}", slots=1 << 18, max_val=256, embeddings=False)
    try:
        n = 100000
        K = np.zeros((n, 16), dtype=np.uint8)
        V = np.zeros((n, 160), dtype=np.uint8)
        for i in range(n):
            k = f"lk{i:08d}".encode()
            K[i, : len(k)] = np.frombuffer(k, dtype=np.uint8)
            V[i, :150] = (i * 7 + np.arange(150)) % 251
        L = np.full(n, 150, dtype=np.uint32)
        assert (s.set_batch(K, V, L) == 0).all()
        st, out, ln = s.get_batch(K, width=160)
        assert (st == 0).all() and (ln == 150).all() and np.array_equal(out[:, :150], V[:, :150])
    finally:
        s.close()
        S.unlink(f"hbm:{uniq}")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tool = os.path.join(root, "libsplinter_amd", "bin", "splinter_hostapi_bench")
    r = subprocess.run([tool, "--store", f"hbm:{uniq}t", "--batch", "500000", "--keys", "1000000", "--seconds", "1"],
                       capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, SPLINTER_BATCH_CHUNK_MB="16"))
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["get_check_failures"] == 0 and res["backend"] == "hbm"


@pytest.mark.gpu
def test_batch_api_node_hbm_pipelined_chunks(uniq, monkeypatch):
    """A node batch larger than SPLINTER_NODE_BATCH_CHUNK runs as pipelined chunks (the next chunk
    partitioned while the shards execute the current one): every op lands in client order."""
    monkeypatch.setenv("SPLINTER_NODE_SHARDS", "4")
    monkeypatch.setenv("SPLINTER_NODE_BATCH_CHUNK", "7000")
    from libsplinter_amd import store as S
    s = S.Store.create(f"node:{uniq}", slots=4 * 16384, max_val=256, embeddings=False)
    try:
        n = 30000
        K = np.zeros((n, 16), dtype=np.uint8)
        V = np.zeros((n, 64), dtype=np.uint8)
        for i in range(n):
            k = f"pk{i:08d}".encode()
            K[i, : len(k)] = np.frombuffer(k, dtype=np.uint8)
            V[i, :48] = (i * 13 + np.arange(48)) % 251
        L = np.full(n, 48, dtype=np.uint32)
        assert (s.set_batch(K, V, L) == 0).all()
        perm = np.random.default_rng(1).permutation(n)
        st, out, ln = s.get_batch(K[perm], width=64)
        assert (st == 0).all() and (ln == 48).all() and np.array_equal(out[:, :48], V[perm, :48])
        assert all(s.get(f"pk{i:08d}") == bytes(V[i, :48]) for i in range(0, n, 997))
    finally:
        s.close()
        S.unlink(f"node:{uniq}")


def test_batch_api_node_store_shm_pipelined(monkeypatch):
    """The chunked node-batch pipeline (partition of chunk i+1 beside the shards' work on chunk i),
    forced on a host-shard node with small chunks: results in client order, op for op."""
    monkeypatch.setenv("SPLINTER_NODE_SHARDS", "4")
    monkeypatch.setenv("SPLINTER_NODE_BACKEND", "shm")
    monkeypatch.setenv("SPLINTER_NODE_BATCH_PIPELINE", "1")
    monkeypatch.setenv("SPLINTER_NODE_BATCH_CHUNK", "700")
    from libsplinter_amd import store as S
    name = f"node:bpp{os.getpid()}"
    s = S.Store.create(name, slots=4 * 4096, max_val=256, embeddings=False)
    try:
        _check_store(S, s, n=5000)
    finally:
        s.close()
        S.unlink(name)


def test_batch_api_node_store_after_fork(monkeypatch):
    """The node batch thread pool is per process: a child forked after a batch (pool threads not
    inherited) runs its own batches to completion."""
    monkeypatch.setenv("SPLINTER_NODE_SHARDS", "4")
    monkeypatch.setenv("SPLINTER_NODE_BACKEND", "shm")
    from libsplinter_amd import store as S
    name = f"node:bfk{os.getpid()}"
    s = S.Store.create(name, slots=4 * 65536, max_val=64, embeddings=False)
    try:
        keys = [f"fk-{i:07d}" for i in range(70000)]  # above the threaded-partition threshold
        assert (s.set_batch(keys, [b"parent"] * len(keys)) == 0).all()
        pid = os.fork()
        if pid == 0:
            ok = False
            try:
                ok = bool((s.set_batch(keys, [b"child"] * len(keys)) == 0).all())
            finally:
                os._exit(0 if ok else 1)
        _, code = os.waitpid(pid, 0)
        assert os.WEXITSTATUS(code) == 0
        st, out, ln = s.get_batch(keys, width=16)
        assert (st == 0).all() and all(bytes(out[i, : ln[i]]) == b"child" for i in range(0, len(keys), 997))
    finally:
        s.close()
        S.unlink(name)

"""Node stores ("node:NAME", csrc/core/node_store.hpp) through the C ABI, on host shards (CPU).

The same NodeStore code drives HBM shards on a GPU box (tests/test_node_gpu.py); here every shard
is a shm store, so routing, replication (C6), summed signal counts (C2), merged list / enumerate
(C5), the node event bus and the per-rank join protocol are checked without a GPU -- including a
world-8 rehearsal where 8 processes each create and join one shard.
"""
import multiprocessing as mp
import os
import subprocess

import pytest


@pytest.fixture
def shm_node(monkeypatch):
    monkeypatch.setenv("SPLINTER_NODE_BACKEND", "shm")
    monkeypatch.setenv("SPLINTER_NODE_SHARDS", "8")
    from libsplinter_amd import store as S
    name = f"nodet{os.getpid()}"
    s = S.Store.create(f"node:{name}", slots=8 * 512, max_val=256, embeddings=True)
    yield S, s, name
    s.close()
    S.unlink(f"node:{name}")


def test_node_routing_matches_python_shard_of(shm_node):
    import torch
    from libsplinter_amd.parallel.sharded import shard_of
    S, s, name = shm_node
    assert s.backend == "node" and s.nshards == 8
    keys = [f"key-{i}" for i in range(3000)]
    hs = torch.tensor([S.N.core_lib().spl_hash_key(k.encode()) for k in keys], dtype=torch.uint64).view(torch.int64)
    want = shard_of(hs, 8).tolist()
    got = [S.node_shard_of(k, 8) for k in keys]
    assert got == want
    # every key lands in (and only in) the shard store the routing names
    for k in keys[:400]:
        s.set(k, k.encode())
    shards = [S.Store.open(S.node_shard_name(name, i, S.NODE_SHM)) for i in range(8)]
    try:
        for k in keys[:400]:
            owner = S.node_shard_of(k, 8)
            for i, sh in enumerate(shards):
                assert (sh.get(k) is not None) == (i == owner), (k, i, owner)
        counts = [len(sh.keys()) for sh in shards]
        assert sum(counts) == 400 and min(counts) > 20, counts  # spread over all 8
    finally:
        for sh in shards:
            sh.close()


def test_node_kv_api(shm_node):
    S, s, name = shm_node
    assert s.slots == 8 * 512
    for i in range(200):
        s.set(f"k{i}", f"value-{i}".encode())
    assert s.get("k7") == b"value-7"
    assert sorted(s.keys()) == sorted(f"k{i}" for i in range(200))
    assert s.unset("k7") == len(b"value-7")
    assert s.get("k7") is None
    s.set("n", b"41")
    s.set_type("n", S.SLOT_BIGUINT)
    s.integer_op("n", S.OP_INC, 1)
    assert s.get_u64("n") == 42
    assert s.append("k8", b"+more") == len(b"value-8+more")
    s.set_embedding("k9", [0.5] * 768)
    assert abs(float(s.get_embedding("k9")[3]) - 0.5) < 1e-7
    h = s.header()
    assert h["slots"] == 8 * 512
    # mop replicated to every shard (C6)
    s.set_mop(0)
    assert s.get_mop() == 0
    for i in range(8):
        with S.Store.open(S.node_shard_name(name, i, S.NODE_SHM)) as sh:
            assert sh.get_mop() == 0
    s.set_mop(1)


def test_node_signals_labels_enumerate_and_bus(shm_node):
    S, s, name = shm_node
    keys = [f"doc{i}" for i in range(64)]
    owners = {S.node_shard_of(k, 8) for k in keys}
    assert len(owners) == 8
    for k in keys:
        s.set(k, b"x")
    s.watch_label(0x1, 5)  # label bit 0 -> group 5 on every shard
    fd = -1
    s.event_bus_init()
    fd = s.event_bus_open()
    try:
        before = s.signal_count(5)
        for k in keys:
            assert s.set_label(k, 0x1)
            assert s.bump(k)
        # a pulse on any shard counts for the node's watchers (C2: sum over shards)
        assert s.signal_count(5) - before == len(keys)
        got = s.enumerate(0x1)
        assert sorted(k for k, _ in got) == sorted(keys)
        s.set("late", b"y")
        assert S.Store.event_bus_wait(fd, 2000), "a shard's write must wake the node event bus"
    finally:
        if fd >= 0:
            S.N.core_lib().splinter_event_bus_close(fd)


def test_node_shard_bids_are_node_wide(shm_node):
    S, s, name = shm_node
    s.shard_claim(0x5F10, S.INTENT_WILLNEED, 40, 10 ** 12)
    table = s.shard_table()
    assert any(b["shard_id"] == 0x5F10 for b in table)
    assert s.shard_election()[0] == 0x5F10


def _join_rank(name, rank, world, q):
    try:
        os.environ["SPLINTER_NODE_BACKEND"] = "shm"
        from libsplinter_amd import store as S
        sh = S.Store.create(S.node_shard_name(name, rank, S.NODE_SHM), slots=256, max_val=64, embeddings=False)
        mine = [k for k in (f"r{rank}-{i}" for i in range(400)) if S.node_shard_of(k, world) == rank]
        for k in mine:
            sh.set(k, k.encode())
        S.node_join(name, rank, world, S.NODE_SHM, 256, 64, embeddings=False)
        sh.close()
        q.put((rank, len(mine)))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


def test_node_join_world8_rehearsal():
    """8 ranks (processes) each create their shard and join; a ninth process opens node:NAME
    through the C ABI and sees every rank's keys through one routed store."""
    from libsplinter_amd import store as S
    name = f"nodej{os.getpid()}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_join_rank, args=(name, r, 8, q)) for r in range(8)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert all(isinstance(v, int) for v in res.values()), res
    os.environ["SPLINTER_NODE_BACKEND"] = "shm"
    try:
        s = S.Store.open(f"node:{name}")
        try:
            assert s.nshards == 8
            assert len(s.keys()) == sum(res.values())
            for r in range(8):
                for i in range(0, 400, 37):
                    k = f"r{r}-{i}"
                    if S.node_shard_of(k, 8) == r:
                        assert s.get(k) == k.encode()
        finally:
            s.close()
        # mismatched geometry is refused
        assert S.N.core_lib().spl_node_join(name.encode(), 0, 8, 0, 128, 64, 128) != 0
    finally:
        for r in range(8):
            S.node_leave(name, r)
        for r in range(8):
            S.unlink(S.node_shard_name(name, r, S.NODE_SHM))
        os.environ.pop("SPLINTER_NODE_BACKEND", None)


def test_node_open_waits_for_all_shards():
    from libsplinter_amd import store as S
    name = f"nodep{os.getpid()}"
    os.environ["SPLINTER_NODE_BACKEND"] = "shm"
    try:
        sh = S.Store.create(S.node_shard_name(name, 0, S.NODE_SHM), slots=64, max_val=64, embeddings=False)
        S.node_join(name, 0, 2, S.NODE_SHM, 64, 64, embeddings=False)
        with pytest.raises(S.SplinterBusy):
            S.Store.open(f"node:{name}")
        sh.close()
    finally:
        S.node_leave(name, 0)
        S.unlink(S.node_shard_name(name, 0, S.NODE_SHM))
        os.environ.pop("SPLINTER_NODE_BACKEND", None)


def test_cli_on_node_store():
    from libsplinter_amd import _native as N
    ctl = os.path.join(N.BIN_DIR, "splinterctl")
    name = f"nodecli{os.getpid()}"
    env = dict(os.environ, SPLINTER_NODE_BACKEND="shm", SPLINTER_NODE_SHARDS="4")
    run = lambda *a: subprocess.run([ctl, *a], env=env, capture_output=True, text=True, timeout=60)  # noqa: E731
    try:
        r = run("init", f"node:{name}", "--slots", "4096", "--length", "256")
        assert r.returncode == 0, r.stderr
        for i in range(20):
            assert run("-u", f"node:{name}", "set", f"cli{i}", f"v{i}").returncode == 0
        r = run("-u", f"node:{name}", "get", "cli13")
        assert r.returncode == 0 and "v13" in r.stdout, (r.stdout, r.stderr)
        r = run("-u", f"node:{name}", "list")
        assert r.returncode == 0 and sum(f"cli{i}" in r.stdout for i in range(20)) == 20, r.stdout
        r = run("-u", f"node:{name}", "config")
        assert r.returncode == 0, r.stderr
    finally:
        from libsplinter_amd import store as S
        S.unlink(f"node:{name}")


def test_node_create_failure_rolls_back(monkeypatch):
    """A shard that cannot be created (its name is taken) fails the node create and leaves no
    descriptor or partial shards behind, so the next create with the name free succeeds."""
    monkeypatch.setenv("SPLINTER_NODE_BACKEND", "shm")
    monkeypatch.setenv("SPLINTER_NODE_SHARDS", "6")
    from libsplinter_amd import store as S
    name = f"noderb{os.getpid()}"
    blocker = S.Store.create(S.node_shard_name(name, 3, S.NODE_SHM), slots=64, max_val=64, embeddings=False)
    try:
        with pytest.raises(S.SplinterError):
            S.Store.create(f"node:{name}", slots=6 * 64, max_val=64, embeddings=False)
        for i in range(3):
            assert not os.path.exists(f"/dev/shm/{name}.s{i}"), i
        assert not os.path.exists(f"/dev/shm/{name}.node")
        assert os.path.exists(f"/dev/shm/{name}.s3")  # not ours: the failed create must not remove it
    finally:
        blocker.close()
        S.unlink(S.node_shard_name(name, 3, S.NODE_SHM))
    s = S.Store.create(f"node:{name}", slots=6 * 64, max_val=64, embeddings=False)
    s.set("a", b"b")
    s.close()
    assert S.unlink(f"node:{name}") == 0
    assert not any(os.path.exists(f"/dev/shm/{name}.s{i}") for i in range(6))


def test_node_unlink_without_open(monkeypatch):
    """spl_unlink("node:NAME") cleans up a node that cannot be opened (a joined node whose other
    ranks never attached), reading the shard count from the descriptor."""
    monkeypatch.setenv("SPLINTER_NODE_BACKEND", "shm")
    from libsplinter_amd import store as S
    name = f"nodeun{os.getpid()}"
    sh = S.Store.create(S.node_shard_name(name, 0, S.NODE_SHM), slots=64, max_val=64, embeddings=False)
    S.node_join(name, 0, 3, S.NODE_SHM, 64, 64, embeddings=False)
    sh.close()
    with pytest.raises(S.SplinterBusy):
        S.Store.open(f"node:{name}")
    S.unlink(f"node:{name}")
    assert not os.path.exists(f"/dev/shm/{name}.node") and not os.path.exists(f"/dev/shm/{name}.s0")


def test_node_madvise_forwards_to_host_shards(shm_node):
    """The node election's winner has its advice applied to every host shard (posix_madvise),
    as the reference does for its one mapping (splinter.c:1329-1377): an advice the kernel
    rejects surfaces as an error only if it was forwarded."""
    S, s, name = shm_node
    s.shard_claim(0x77, S.INTENT_WILLNEED, 90, 10 ** 12)
    s.madvise(0x77, 3)  # POSIX_MADV_WILLNEED on every shard
    with pytest.raises(S.SplinterError):
        s.madvise(0x77, 12345)  # invalid advice: posix_madvise -> EINVAL from the shards
    s.shard_release(0x77)


def _race_rank(name, rank, world, go, q):
    try:
        os.environ["SPLINTER_NODE_BACKEND"] = "shm"
        from libsplinter_amd import store as S
        sh = S.Store.create(S.node_shard_name(name, rank, S.NODE_SHM), slots=64, max_val=64, embeddings=False)
        go.wait(30)
        S.node_join(name, rank, world, S.NODE_SHM, 64, 64, embeddings=False)
        sh.close()
        q.put((rank, 0))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("trial", range(3))
def test_node_join_simultaneous(trial):
    """Every rank released at the same instant into spl_node_join (the O_EXCL race of the
    descriptor: a loser must wait for the winner's full-size descriptor, not SIGBUS on it)."""
    from libsplinter_amd import store as S
    name = f"noders{os.getpid()}t{trial}"
    ctx = mp.get_context("fork")
    q, go = ctx.Queue(), ctx.Event()
    ps = [ctx.Process(target=_race_rank, args=(name, r, 8, go, q)) for r in range(8)]
    for p in ps:
        p.start()
    import time
    time.sleep(0.5)
    go.set()
    try:
        res = dict(q.get(timeout=60) for _ in ps)
        for p in ps:
            p.join(30)
        assert res == {r: 0 for r in range(8)}, res
        assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    finally:
        os.environ["SPLINTER_NODE_BACKEND"] = "shm"
        S.unlink(f"node:{name}")
        os.environ.pop("SPLINTER_NODE_BACKEND", None)

"""HBM arena: batched gfx950 kernels vs. a Python-dict reference, the single-op
reference API on an hbm: store, seqlock integrity under concurrent streams,
and checkpoint -> host-backend interop."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def arena(uniq):
    import torch  # noqa: F401
    from libsplinter_amd.ops.arena import HbmArena
    a = HbmArena.create(uniq, slots=4096, max_val=256, embeddings=True)
    yield a
    a.close()


def test_single_op_api_on_hbm_store(arena):
    s = arena.store
    assert s.backend == "hbm" and s.embeddings
    s.set("alpha", b"hello world")
    assert s.get("alpha") == b"hello world"
    s.set("alpha", "updated")
    assert s.get("alpha") == b"updated"
    assert s.get("missing") is None
    e = s.epoch("alpha")
    assert e > 0 and e % 2 == 0
    assert s.set_label("alpha", 1 << 5)
    assert [k for k, _ in s.enumerate(1 << 5)] == ["alpha"]
    s.set("ctr", (41).to_bytes(8, "little"))
    s.set_type("ctr", 1 << 2)  # BIGUINT
    assert s.integer_op("ctr", 4, 1) == 42  # INC
    vec = np.arange(768, dtype=np.float32) * 0.5
    s.set_embedding("alpha", vec)
    np.testing.assert_array_equal(s.get_embedding("alpha"), vec)
    assert s.unset("alpha") == 7
    assert s.get("alpha") is None
    assert sorted(s.list()) == ["ctr"]
    assert s.watch("ctr", 3)
    c0 = s.signal_count(3)
    s.set("ctr", (1).to_bytes(8, "little"))
    assert s.signal_count(3) == c0 + 1


def test_batch_set_get_matches_reference(arena):
    import torch
    from libsplinter_amd.ops.arena import pack_keys, pack_values, unpack
    rng = np.random.default_rng(0)
    n = 3000
    keys = [f"key-{i}-{rng.integers(1 << 30)}" for i in range(n)]
    vals = [bytes(rng.integers(1, 255, size=rng.integers(1, 200), dtype=np.uint8)) for _ in range(n)]
    K = pack_keys(keys, 32)
    V, L = pack_values(vals, 256)
    st = arena.set(K, V, L)
    torch.cuda.synchronize()
    assert (st == 0).all(), st[st != 0][:10]
    st, out, ol = arena.get(K)
    assert (st == 0).all()
    assert unpack(out, ol) == vals
    # host single-op path sees the same data
    for i in range(0, n, 97):
        assert arena.store.get(keys[i]) == vals[i]
    # misses
    st, _, _ = arena.get(pack_keys(["nope-1", "nope-2"], 32))
    assert st.tolist() == [-2, -2]
    # unset half, verify chains survive
    st = arena.unset(K[::2])
    assert (st >= 0).all()
    st, out, ol = arena.get(K)
    got = st.cpu().numpy()
    assert (got[::2] == -2).all() and (got[1::2] == 0).all()
    assert unpack(out[1::2], ol[1::2]) == vals[1::2]
    # full table reports ENOSPC, never duplicates
    idx, _ = arena.scan(0)
    assert idx.numel() == n - (n + 1) // 2


def test_integer_ops_and_meta(arena):
    import torch
    from libsplinter_amd.ops.arena import pack_keys, pack_values
    keys = [f"c{i}" for i in range(64)]
    K = pack_keys(keys, 16)
    V, L = pack_values([(i).to_bytes(8, "little") for i in range(64)], 16)
    assert (arena.set(K, V, L) == 0).all()
    st, _ = arena.meta("type", K, torch.full((64,), 4, dtype=torch.int64, device="cuda"))
    assert (st == 0).all()
    ops = torch.full((64,), 4, dtype=torch.int32, device="cuda")  # INC
    masks = torch.arange(64, dtype=torch.int64, device="cuda")
    st, res = arena.integer_op(K, ops, masks)
    assert (st == 0).all()
    assert res.tolist() == [2 * i for i in range(64)]
    st, _ = arena.meta("set_label", K[:10], torch.full((10,), 1 << 9, dtype=torch.int64, device="cuda"))
    idx, _ = arena.scan(1, 1 << 9)
    assert idx.numel() == 10
    # EPROTOTYPE on non-BIGUINT
    K2 = pack_keys(["txt"], 16)
    V2, L2 = pack_values([b"abc"], 16)
    arena.set(K2, V2, L2)
    st, _ = arena.integer_op(K2, torch.tensor([4], dtype=torch.int32, device="cuda"))
    assert st.item() == -91


def test_embeddings_batch(arena):
    import torch
    from libsplinter_amd.ops.arena import pack_keys, pack_values
    keys = [f"doc{i}" for i in range(200)]
    K = pack_keys(keys, 16)
    V, L = pack_values([b"text"] * 200, 16)
    arena.set(K, V, L)
    vecs = torch.randn(200, 768, device="cuda")
    st = arena.set_embeddings(K, vecs)
    assert (st == 0).all()
    st, back = arena.get_embeddings(K)
    assert (st == 0).all()
    assert torch.equal(back, vecs)
    m = arena.embedding_matrix()
    slot0 = arena.store.find_slot("doc0") if arena.store.backend != "hbm" else None
    assert m.shape == (4096, 768)
    idx, _ = arena.scan(2)
    assert idx.numel() == 200


def test_concurrent_streams_integrity(uniq):
    """Writers and readers on different HIP streams race on the same keys;
    every successful read must be an intact value written by some writer."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values
    a = HbmArena.create(uniq, slots=1 << 16, max_val=256, embeddings=False)
    try:
        n = 20000
        K = format_keys(n, "k", 9, 16)
        V0, L0 = format_values(n, 1, 150, 256)
        assert (a.set(K, V0, L0) == 0).all()
        torch.cuda.synchronize()
        sw, sr = torch.cuda.Stream(), torch.cuda.Stream()
        outs = []
        for ver in range(2, 8):
            V, L = format_values(n, ver, 150, 256)
            torch.cuda.synchronize()
            with torch.cuda.stream(sw):
                a.set(K, V, L)
            with torch.cuda.stream(sr):
                outs.append(a.get(K, retries=1000))
        torch.cuda.synchronize()
        for st, out, ol in outs:
            assert (st == 0).all()
            o = out.cpu().numpy()
            ln = ol.cpu().numpy()
            for i in range(0, n, 37):
                s = bytes(o[i, : ln[i]])
                head, _, rest = s.partition(b"|id:")
                ver = int(head[4:])
                ident = int(rest.split(b"|")[0])
                assert ident == i
                fill = s[s.index(b"data:") + 5:]
                assert fill == bytes([65 + ver % 26]) * len(fill), "torn value"
    finally:
        a.close()


def test_checkpoint_roundtrip_to_host_backend(arena, uniq, tmp_path):
    from libsplinter_amd import Store
    s = arena.store
    for i in range(50):
        s.set(f"p{i}", f"value-{i}")
    s.set_label("p3", 1 << 7)
    path = str(tmp_path / "ckpt.spl")
    arena.checkpoint(path)
    h = Store.open(path)
    try:
        assert h.backend == "file" and h.stride == 3200 and h.slots == 4096
        assert h.get("p7") == b"value-7"
        assert [k for k, _ in h.enumerate(1 << 7)] == ["p3"]
        h.set("p8", "changed")
    finally:
        h.close()
    arena.restore(path)
    assert s.get("p8") == b"changed"


def test_watchdog_finds_stuck_writer_and_retrain_recovers(arena):
    """A slot left odd (writer died mid-write) is reported by the odd-epoch scan
    watchdog, and retrain (epoch -> 4) makes it readable again."""
    import torch
    from libsplinter_amd.ops.arena import pack_keys, pack_values
    K = pack_keys([f"w{i}" for i in range(100)], 16)
    V, L = pack_values([b"v"] * 100, 16)
    assert (arena.set(K, V, L) == 0).all()
    st, idx = arena.meta("find", K[7:8])
    slot = int(idx[0])
    sv = arena.slot_view()
    ep = sv[slot, 8:16].clone().view(torch.int64)
    sv[slot, 8:16] = (ep | 1).view(torch.uint8)  # simulate a crashed writer
    torch.cuda.synchronize()
    stuck, eps = arena.stuck_slots(hold_ms=20)
    assert stuck.tolist() == [slot] and int(eps[0]) & 1
    st, _, _ = arena.get(K[7:8], retries=4)
    assert int(st[0]) == -11  # EAGAIN while the writer "holds" the slot
    assert int(arena.meta("retrain", K[7:8])[0][0]) == 0
    assert arena.stuck_slots(hold_ms=1)[0].numel() == 0
    assert int(arena.get(K[7:8])[0][0]) == 0


def test_cross_process_attach_ipc(arena, uniq):
    """Another process attaches the same HBM arena through the hbm: descriptor
    (hipIpcOpenMemHandle): the C CLI reads what this process wrote, a child Python
    process writes a key this process then reads."""
    import subprocess
    import sys
    import torch
    from libsplinter_amd.ops.arena import pack_keys, pack_values
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    K = pack_keys(["ipc_a", "ipc_b"], 16)
    V, L = pack_values([b"from parent", b"second"], 16)
    assert (arena.set(K, V, L) == 0).all()
    torch.cuda.synchronize()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cli = os.path.join(root, "libsplinter_amd", "bin", "splinterctl")
    r = subprocess.run([cli, "-u", f"hbm:{uniq}", "get", "ipc_a"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and r.stdout.startswith("from parent"), r.stderr
    code = ("import torch; from libsplinter_amd import Store; "
            f"s = Store.open('hbm:{uniq}'); assert s.get('ipc_b') == b'second'; s.set('ipc_child', 'hello from child')")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    st, out, ol = arena.get(pack_keys(["ipc_child"], 16))
    assert int(st[0]) == 0 and bytes(out[0, : int(ol[0])].cpu().numpy()) == b"hello from child"


def test_racing_inserts_no_duplicates(uniq):
    """Many lanes / two streams insert the same 512 keys concurrently (each key 128x per
    batch): every key ends up in exactly one slot (the insert re-validation protocol)."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values
    from libsplinter_amd.parallel.sharded import GpuShard
    a = HbmArena.create(uniq + "r", slots=4096, max_val=64, embeddings=False)
    try:
        ids = torch.arange(512, device="cuda").repeat(128)
        ids = ids[torch.randperm(ids.numel(), device="cuda")]
        K = format_keys(ids.numel(), "race", 6, 16, ids=ids)
        V, L = format_values(ids.numel(), 1, 24, 64, ids=ids)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for _ in range(3):
            with torch.cuda.stream(s1):
                a.set(K, V, L)
            with torch.cuda.stream(s2):
                a.set(K.flip(0).contiguous(), V.flip(0).contiguous(), L.flip(0).contiguous())
            torch.cuda.synchronize()
        idx, _ = a.scan(0)
        rows = GpuShard(a).key_rows(idx).cpu().numpy()
        keys = [bytes(r).split(b"\0", 1)[0] for r in rows]
        assert len(keys) == 512 and len(set(keys)) == 512
    finally:
        a.close()


def test_hot_keys_carried_retries(uniq):
    """64 hot keys, 40k sets racing 40k gets on two streams: contended ops are carried into
    later rounds (k_set_carry / k_get_carry); every op ends ok or EAGAIN after its bounded
    attempts, the stats add up, every successful read is an intact value of its key, and the
    final value of each key is one of the versions written to it."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values
    a = HbmArena.create(uniq + "h", slots=4096, max_val=256, embeddings=False)
    try:
        n, hot = 40000, 64
        ids = torch.arange(n, device="cuda") % hot
        K = format_keys(n, "hot", 4, 16, ids=ids)
        V0, L0 = format_values(hot, 1, 150, 256, ids=torch.arange(hot, device="cuda"))
        assert (a.set(K[:hot], V0, L0) == 0).all()
        torch.cuda.synchronize()
        a.reset_stats()
        V, L = format_values(n, 5, 150, 256, ids=ids)
        sw, sr = torch.cuda.Stream(), torch.cuda.Stream()
        with torch.cuda.stream(sw):
            sst = a.set(K, V, L, retries=64)
        with torch.cuda.stream(sr):
            gst, out, ol = a.get(K, retries=64)
        torch.cuda.synchronize()
        sst, gst = sst.cpu(), gst.cpu()
        assert bool(((sst == 0) | (sst == -11)).all()) and bool(((gst == 0) | (gst == -11)).all())
        # 625 racing sets per key: a bounded attempt budget leaves many EAGAIN (the reference's
        # "retry" status) -- readers of a key that is being rewritten all the time may starve
        # inside one batch -- but the writers make progress
        assert int((sst == 0).sum()) >= hot
        attempts, ok, again, miss = [int(x) for x in a.stats.tolist()]
        assert ok == int((sst == 0).sum()) + int((gst == 0).sum()) and miss == 0
        assert attempts == ok + again  # every attempt ends ok or EAGAIN here (no misses)
        o, ln, idh = out.cpu().numpy(), ol.cpu().numpy(), ids.cpu().numpy()
        for i in np.nonzero(gst.numpy() == 0)[0][::97]:
            s = bytes(o[i, : ln[i]])
            head, _, rest = s.partition(b"|id:")
            ver = int(head[4:])
            assert int(rest.split(b"|")[0]) == idh[i] and ver in (1, 5)
            fill = s[s.index(b"data:") + 5:]
            assert fill == bytes([65 + ver % 26]) * len(fill), "torn value"
        # a client that resubmits its EAGAIN ops gets them all through
        pend = torch.nonzero(sst.cuda() != 0).squeeze(1)
        for _ in range(200):
            if pend.numel() == 0:
                break
            r = a.set(K[pend].contiguous(), V[pend].contiguous(), L[pend].contiguous(), retries=64)
            pend = pend[r != 0]
        assert pend.numel() == 0
        st, out2, ol2 = a.get(K[:hot])
        assert (st == 0).all()
        for i in range(hot):
            s = bytes(out2[i, : ol2[i]].cpu().numpy())
            assert s.startswith(b"ver:5|")
        # the starved reads go through once the writers are done
        gpend = torch.nonzero(gst.cuda() != 0).squeeze(1)
        if gpend.numel():
            st3, _, _ = a.get(K[gpend].contiguous())
            assert (st3 == 0).all()
    finally:
        a.close()


def test_unaligned_value_rows_do_not_spill(uniq):
    """max_val = 100 (value rows 4-B aligned, last 16-B chunk partial): full-length values in
    neighbouring slots survive each other's sets (set rounds, cooperative copy, single-op path),
    and integer ops work on rows that are not 8-B aligned."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena, pack_keys, pack_values, unpack
    a = HbmArena.create(uniq + "u", slots=2048, max_val=100, embeddings=False)
    try:
        keys = [f"u{i:05d}" for i in range(1500)]
        vals = [bytes([65 + (i % 26)]) * (100 if i % 3 else 37 + i % 50) for i in range(len(keys))]
        K = pack_keys(keys, 16)
        V, L = pack_values(vals, 112)
        for _ in range(2):  # insert, then update in place
            assert (a.set(K, V, L) == 0).all()
        st, out, ol = a.get(K)
        torch.cuda.synchronize()
        assert (st == 0).all()
        assert unpack(out, ol) == vals
        s = a.store
        s.set("ctr", (7).to_bytes(8, "little"))
        s.set_type("ctr", 1 << 2)  # BIGUINT
        assert s.integer_op("ctr", 4, 5) == 12  # INC
        st, out, ol = a.get(K)
        assert unpack(out, ol) == vals
    finally:
        a.close()


_RACE_READER = r"""
import json, sys, time
import numpy as np
import torch
sys.path.insert(0, sys.argv[3])
from libsplinter_amd import Store
from libsplinter_amd.ops.arena import HbmArena, format_keys
n, secs = int(sys.argv[2]), float(sys.argv[4])
a = HbmArena(Store.open(sys.argv[1]))


def check(v, want_id):
    try:
        head, rest = v.split(b"|id:", 1)
        ver = int(head[4:])
        ident = int(rest.split(b"|", 1)[0])
        fill = v[v.index(b"data:") + 5:]
        return ident == want_id and len(fill) > 0 and fill == bytes([65 + ver % 26]) * len(fill)
    except Exception:
        return False


g = torch.Generator(device="cuda")
g.manual_seed(7)
checked = torn = again = calls = 0
print("ready", flush=True)
t0 = time.time()
while time.time() - t0 < secs:
    ids = torch.randint(0, n, (4096,), device="cuda", generator=g)
    K = format_keys(4096, "race", 8, 16, ids=ids)
    st, out, ln = a.get(K, retries=0)
    st, out, ln, ids = st.cpu().numpy(), out.cpu().numpy(), ln.cpu().numpy(), ids.cpu().numpy()
    for i in range(4096):
        if st[i] == -11:
            again += 1
            continue
        checked += 1
        if st[i] != 0 or not check(bytes(out[i, : ln[i]]), int(ids[i])):
            torn += 1
    for i in range(0, 64):  # the per-call path (device command ring) on the same slots
        k = int(np.random.randint(n))
        try:
            v = a.store.get(f"race{k:08d}")
            calls += 1
            if v is None or not check(v, k):
                torn += 1
        except OSError:
            again += 1
print(json.dumps({"checked": checked, "calls": calls, "torn": torn, "eagain": again}), flush=True)
"""


def test_cross_process_reader_races_gpu_writers(uniq):
    """A separate process attaches the arena and reads (batched kernels with no retries, plus
    per-call gets through its own command ring) while THIS process's writer kernels keep
    rewriting the same keys with new versions: every value read that is not EAGAIN must be a
    whole, self-consistent record (ver / id / fill bytes) -- the seqlock across processes."""
    import json
    import subprocess
    import sys
    import time
    import torch
    from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values
    n = 20000
    a = HbmArena.create(uniq, slots=1 << 16, max_val=256, embeddings=False)
    try:
        K = format_keys(n, "race", 8, 16)
        V, L = format_values(n, 1, 200, 256)
        assert (a.set(K, V, L) == 0).all()
        torch.cuda.synchronize()
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        p = subprocess.Popen([sys.executable, "-u", "-c", _RACE_READER, f"hbm:{uniq}", str(n), root, "4"],
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
        assert p.stdout.readline().strip() == "ready"
        ver, t0 = 2, time.time()
        while p.poll() is None and time.time() - t0 < 60:
            V, L = format_values(n, ver, 120 + 20 * (ver % 5), 256)  # lengths change too
            st = a.set(K, V, L)
            ver += 1
            if ver % 16 == 0:
                torch.cuda.synchronize()
        out, err = p.communicate(timeout=120)
        assert p.returncode == 0, err[-2000:]
        res = json.loads(out.strip().splitlines()[-1])
        print(res, "writer versions", ver)
        assert res["torn"] == 0, res
        assert res["checked"] > 10000 and res["calls"] > 100 and ver > 10
        del st
    finally:
        a.close()


def test_acquire_free_get_cross_xcd_hot_keys(uniq):
    """Pins the coherence assumption of the default acquire-free get (SPLINTER_ARENA_COOP_GET=2,
    arena_kernels.hip k_get_carry FAST): writer and reader workgroups of large grids are dealt
    round-robin over all 8 XCDs, so every hot key below is written and read from different XCDs
    at once.  Every returned row (not a sample) must be one intact version: the 'ver:<v>' header,
    the id and the fill byte 'A' + v % 26 all agree."""
    import numpy as np
    import torch
    from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values
    a = HbmArena.create(uniq, slots=1 << 14, max_val=256, embeddings=False)
    try:
        hot, rep = 256, 64  # 256 keys, each repeated 64 times per batch: 16384 ops over ~64 workgroups
        ids = torch.arange(hot, device="cuda").repeat(rep)
        K = format_keys(hot * rep, "hx", 6, 16, ids=ids)
        V0, L0 = format_values(hot, 1, 150, 256, ids=torch.arange(hot, device="cuda"))
        assert (a.set(K[:hot], V0, L0) == 0).all()
        torch.cuda.synchronize()
        ws = [torch.cuda.Stream() for _ in range(4)]
        rs = [torch.cuda.Stream() for _ in range(4)]
        vals = [format_values(hot * rep, v, 150, 256, ids=ids) for v in range(2, 14)]
        outs = []
        torch.cuda.synchronize()
        for j, (V, L) in enumerate(vals):
            with torch.cuda.stream(ws[j % 4]):
                a.set(K, V, L, retries=10000)
            with torch.cuda.stream(rs[j % 4]):
                outs.append(a.get(K, retries=10000))
        torch.cuda.synchronize()
        want_id = ids.cpu().numpy()
        checked = 0
        for st, out, ol in outs:
            s_ = st.cpu().numpy()
            o = out.cpu().numpy()
            ln = ol.cpu().numpy()
            assert (s_ == 0).all(), np.unique(s_, return_counts=True)
            for i in range(o.shape[0]):
                row = bytes(o[i, : ln[i]])
                head, _, rest = row.partition(b"|id:")
                ver = int(head[4:])
                assert int(rest.split(b"|")[0]) == want_id[i]
                fill = row[row.index(b"data:") + 5:]
                assert fill == bytes([65 + ver % 26]) * len(fill), f"torn value at row {i}: {row[:40]!r}"
                checked += 1
        assert checked == len(outs) * hot * rep
    finally:
        a.close()


@pytest.mark.parametrize("kstride", [16, 32])
@pytest.mark.parametrize("mode", [0, 1, 2, 3, "2s0", "2s1"])
def test_kvs_step_modes_match_plain_kernels(uniq, kstride, mode):
    """One KV step of 8 + 8 client streams (spl_kvs_step) -- per-slice launches (0), one fused
    grid (1, 2: the default; "2s0" / "2s1": its workgroup-barrier and chunk-claim schedules) or
    stream-posted slices on a server grid (3; 32-B keys take the fused grid) -- sets new and
    existing keys and gets present and missing ones with the same results as the plain batch
    kernels."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena, KvStreams, pack_keys, pack_values, unpack
    sched = -1
    if isinstance(mode, str):
        mode, sched = int(mode[0]), int(mode[2:])
    rng = np.random.default_rng(kstride + mode + 7 * sched)
    a = HbmArena.create(uniq, slots=1 << 16, max_val=256, embeddings=False)
    kvs = KvStreams(8, 8)
    try:
        kvs.set_fused(mode)
        kvs.set_sched(sched)
        n = 20000
        w = kstride - 1
        keys = [f"k{i:0{min(w - 1, 12)}d}"[:w] for i in range(n)]
        vals = [bytes(rng.integers(1, 255, size=int(rng.integers(1, 200)), dtype=np.uint8)) for _ in range(n)]
        K = pack_keys(keys, kstride)
        V, L = pack_values(vals, 256)
        half = n // 2
        assert (a.set(K[:half], V[:half], L[:half]) == 0).all()
        # step: set the second half (new) and rewrite the first quarter; get the first half + misses
        sidx = np.r_[np.arange(half, n), np.arange(0, half // 2)]
        new_vals = {int(i): vals[int(i)][::-1] for i in sidx}
        SV, SL = pack_values([new_vals[int(i)] for i in sidx], 256)
        SK = K[torch.as_tensor(sidx, device=K.device)]
        GK = torch.cat([K[:half], pack_keys([f"zz{i}"[:w] for i in range(500)], kstride)])
        sst = torch.full((len(sidx),), 99, dtype=torch.int32, device="cuda")
        gst = torch.full((GK.shape[0],), 99, dtype=torch.int32, device="cuda")
        gout = torch.zeros((GK.shape[0], 256), dtype=torch.uint8, device="cuda")
        glen = torch.zeros(GK.shape[0], dtype=torch.int32, device="cuda")
        kvs.step(a, SK, SV, SL, sst, GK, gout, glen, gst)
        torch.cuda.synchronize()
        assert (sst == 0).all()
        g = gst.cpu().numpy()
        assert (g[half:] == -2).all()
        assert (g[:half] == 0).all(), np.unique(g[:half])
        got = unpack(gout[:half], glen[:half])
        for i in range(half):  # a get racing a set of the same key sees the old or the new value
            assert got[i] in (vals[i], new_vals.get(i, vals[i])), i
        st, out, ol = a.get(K)
        assert (st == 0).all()
        final = unpack(out, ol)
        assert all(final[i] == new_vals.get(i, vals[i]) for i in range(n))
    finally:
        kvs.close()
        a.close()


def test_kvs_async_server_reads_producer_kernel_output(uniq):
    """Mode 3 (stream-posted server): every step's set keys / values and get keys are rewritten by
    device kernels on the origin stream immediately before the step is posted -- no host
    synchronisation in between -- into the SAME buffers each step, so a server CU that kept a stale
    L1 copy of the previous step's rows (no acquire after the post) would store or fetch the
    previous step's keys / data (verdict round 5, item 6: k_kv_server's agent acquire)."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena, KvStreams, format_keys, format_values
    a = HbmArena.create(uniq, slots=1 << 17, max_val=256, embeddings=False)
    kvs = KvStreams(32, 32)
    try:
        kvs.set_fused(3)
        n, ns, ng = 40000, 12000, 12000
        ids = torch.arange(n, device="cuda")
        V0, L0 = format_values(n, 1, 100, 256, ids=ids)
        assert (a.set(format_keys(n, "p", 9, 16, ids=ids), V0, L0) == 0).all()
        ver = np.ones(n, dtype=np.int64)
        SK = torch.empty((ns, 16), dtype=torch.uint8, device="cuda")
        SV = torch.empty((ns, 256), dtype=torch.uint8, device="cuda")
        SL = torch.empty(ns, dtype=torch.int32, device="cuda")
        GK = torch.empty((ng, 16), dtype=torch.uint8, device="cuda")
        sst = torch.empty(ns, dtype=torch.int32, device="cuda")
        gst = torch.empty(ng, dtype=torch.int32, device="cuda")
        gout = torch.empty((ng, 256), dtype=torch.uint8, device="cuda")
        glen = torch.empty(ng, dtype=torch.int32, device="cuda")
        for step in range(8):
            perm = torch.randperm(n, device="cuda")
            sidx, gidx = perm[:ns], perm[ns:ns + ng]
            SK.copy_(format_keys(ns, "p", 9, 16, ids=sidx))
            v, ln = format_values(ns, step + 2, 60 + 10 * step, 256, ids=sidx)
            SV.copy_(v)
            SL.copy_(ln)
            GK.copy_(format_keys(ng, "p", 9, 16, ids=gidx))
            kvs.step(a, SK, SV, SL, sst, GK, gout, glen, gst)  # posted right behind the producers
            torch.cuda.synchronize()
            assert kvs.async_error() == 0
            assert (sst == 0).all(), np.unique(sst.cpu().numpy(), return_counts=True)
            assert (gst == 0).all(), np.unique(gst.cpu().numpy(), return_counts=True)
            gh, o, lh = gidx.cpu().numpy(), gout.cpu().numpy(), glen.cpu().numpy()
            for j in range(0, ng, 7):
                val = bytes(o[j, : lh[j]])
                assert val.startswith(b"ver:%d|id:" % ver[gh[j]]), (step, j, val[:24], ver[gh[j]])
                assert int(val.split(b"|id:", 1)[1].split(b"|", 1)[0]) == gh[j]
            ver[sidx.cpu().numpy()] = step + 2
        st, out, ol = a.get(format_keys(n, "p", 9, 16, ids=ids))
        assert (st == 0).all()
        o, lh = out.cpu().numpy(), ol.cpu().numpy()
        for i in range(0, n, 13):
            assert bytes(o[i, : lh[i]]).startswith(b"ver:%d|id:%d|" % (ver[i], i))
    finally:
        kvs.close()
        a.close()


def test_kvs_async_server_steps(uniq):
    """Stream-posted server (mode 3) over 32 + 32 client streams for several steps in a row: slices
    of every size (empty ones included: fewer rows than streams x 128-row alignment) all run, each
    step's sets land and its gets return the previous step's values, and no server gives up."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena, KvStreams, pack_keys, pack_values, unpack
    rng = np.random.default_rng(7)
    a = HbmArena.create(uniq, slots=1 << 17, max_val=256, embeddings=False)
    kvs = KvStreams(32, 32)
    try:
        kvs.set_fused(3)
        n = 30000
        keys = [f"a{i:012d}" for i in range(n)]
        K = pack_keys(keys, 16)
        cur = [bytes([65 + i % 26]) * int(rng.integers(1, 150)) for i in range(n)]
        V, L = pack_values(cur, 256)
        assert (a.set(K, V, L) == 0).all()
        for step, (ns, ng) in enumerate([(12000, 9000), (1000, 30000), (28000, 2000), (77, 4000)]):
            sidx = rng.choice(n, ns, replace=False)
            gidx = rng.choice(n, ng, replace=False)
            gset = set(int(i) for i in sidx)
            gidx = np.array([i for i in gidx if int(i) not in gset])
            new = {int(i): bytes([97 + (int(i) + step) % 26]) * int(rng.integers(1, 200)) for i in sidx}
            SV, SL = pack_values([new[int(i)] for i in sidx], 256)
            SK = K[torch.as_tensor(sidx, device=K.device)]
            GK = K[torch.as_tensor(gidx, device=K.device)]
            sst = torch.full((len(sidx),), 99, dtype=torch.int32, device="cuda")
            gst = torch.full((len(gidx),), 99, dtype=torch.int32, device="cuda")
            gout = torch.zeros((len(gidx), 256), dtype=torch.uint8, device="cuda")
            glen = torch.zeros(len(gidx), dtype=torch.int32, device="cuda")
            kvs.step(a, SK, SV, SL, sst, GK, gout, glen, gst)
            torch.cuda.synchronize()
            assert kvs.async_error() == 0
            assert (sst == 0).all(), np.unique(sst.cpu().numpy(), return_counts=True)
            assert (gst == 0).all(), np.unique(gst.cpu().numpy(), return_counts=True)
            got = unpack(gout, glen)
            assert all(got[j] == cur[int(i)] for j, i in enumerate(gidx))
            for i in sidx:
                cur[int(i)] = new[int(i)]
        st, out, ol = a.get(K)
        assert (st == 0).all()
        assert unpack(out, ol) == cur
    finally:
        kvs.close()
        a.close()

"""Maintenance passes of an HBM arena (csrc/hip/arena_maint.hip) and the side region's bf16 vector
copy: probe-chain statistics against a host recomputation from the raw slot words, the online
tombstone compaction under insert / unset churn at 50 % and 90 % load (every live key still found
with its vector, bf16 copy and norm, absent keys still missing, no key duplicated, misses shorter
after), the same pass running beside live fused KV steps, the exclusive full rebuild, and the bf16
copy kept in step by every embedding writer."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _host_stats(ar):
    """Probe statistics from the slot words (hash, epoch) on the host, as k_probe_stats defines them."""
    import torch
    sv = ar.slot_view()[:, :16].contiguous().cpu().numpy()
    h = sv[:, :8].copy().view(np.uint64).ravel()
    e = sv[:, 8:16].copy().view(np.uint64).ravel()
    n = h.size
    busy = (e & 1) == 1
    live = (~busy) & (h != 0)
    virgin = (h == 0) & (e == 0)
    tomb = (~busy) & (h == 0) & (e != 0)
    idx = np.arange(n, dtype=np.uint64)
    home = h[live] % np.uint64(n)
    disp = (idx[live] - home) % np.uint64(n) + 1
    miss_sum = 0
    vpos = np.nonzero(virgin)[0]
    if vpos.size:
        prev = np.roll(vpos, 1)
        L = (vpos - prev - 1) % n
        if vpos.size == 1:
            L = np.array([n - 1])
        miss_sum = int(((L + 1) * (L + 2) // 2).sum())
    del torch
    return dict(live=int(live.sum()), tombstones=int(tomb.sum()), virgin=int(virgin.sum()), busy=int(busy.sum()),
                disp_sum=int(disp.sum()), disp_max=int(disp.max()) if disp.size else 0, miss_sum=miss_sum)


def _keys(ids):
    from libsplinter_amd.ops.arena import format_keys
    import torch
    return format_keys(len(ids), "c", 9, 16, ids=torch.as_tensor(ids, device="cuda"))


def _churn(ar, slots, load, rng, vlen=32, vstride=64):
    """Fill to `load`, then 8 cycles of unsetting 30 % of the live keys and inserting as many new
    ones; returns (live ids, next id)."""
    import torch
    from libsplinter_amd.ops.arena import format_values
    n = int(slots * load)
    live = np.arange(n)
    nxt = n
    V, Lv = format_values(n, 1, vlen, vstride, ids=torch.as_tensor(live, device="cuda"))
    assert int((ar.set(_keys(live), V, Lv) != 0).sum()) == 0
    for cyc in range(8):
        kill = rng.choice(live.size, size=int(0.3 * live.size), replace=False)
        gone = live[kill]
        assert int((ar.unset(_keys(gone)) < 0).sum()) == 0
        live = np.delete(live, kill)
        new = np.arange(nxt, nxt + gone.size)
        nxt += gone.size
        V, Lv = format_values(new.size, 1, vlen, vstride, ids=torch.as_tensor(new, device="cuda"))
        assert int((ar.set(_keys(new), V, Lv) != 0).sum()) == 0
        live = np.concatenate([live, new])
    return live, nxt


def _check_values(ar, live, ver=None):
    sts, out, lens = ar.get(_keys(live))
    assert int((sts != 0).sum()) == 0, np.unique(sts.cpu().numpy(), return_counts=True)
    o, ln = out.cpu().numpy(), lens.cpu().numpy()
    for i in range(0, live.size, max(1, live.size // 2000)):
        v = bytes(o[i, : ln[i]])
        assert int(v.split(b"|id:", 1)[1].split(b"|", 1)[0]) == live[i]
        if ver is not None:
            assert v.startswith(b"ver:%d|" % ver[i]), (v[:12], ver[i])


def _no_duplicates(ar, n_live):
    """Every key lives in exactly one slot (no insert duplicated a key that was mid-move)."""
    sv = ar.slot_view().cpu().numpy()
    h = sv[:, :8].copy().view(np.uint64).ravel()
    e = sv[:, 8:16].copy().view(np.uint64).ravel()
    live = (h != 0) & ((e & 1) == 0)
    keys = sv[live, 64:128]
    uk = np.unique(keys, axis=0)
    assert uk.shape[0] == keys.shape[0] == n_live, (uk.shape[0], keys.shape[0], n_live)


@pytest.mark.parametrize("emb", [False, True])
@pytest.mark.parametrize("load", [0.5, 0.9])
def test_probe_stats_and_rehash_under_churn(uniq, load, emb):
    import torch
    from libsplinter_amd.ops.arena import HbmArena, format_values
    slots = 1 << 16 if not emb else 1 << 13
    ar = HbmArena.create(f"{uniq}", slots=slots, max_val=64, embeddings=emb)
    try:
        rng = np.random.default_rng(7)
        st0 = ar.store.probe_stats()
        live, nxt = _churn(ar, slots, load, rng)
        vec = None
        if emb:  # every live key carries a vector: moves must carry it, its bf16 copy and its norm
            vec = torch.randn(live.size, 768, device="cuda")
            assert int((ar.set_embeddings(_keys(live), vec) != 0).sum()) == 0
        torch.cuda.synchronize()
        st1 = ar.store.probe_stats()
        host = _host_stats(ar)
        for k, v in host.items():
            assert st1[k] == v, (k, st1[k], v)
        assert st1["live"] == live.size and st1["tombstones"] > 0
        assert st1["miss_mean"] > st0["miss_mean"] or st0["virgin"] == 0
        r = ar.store.rehash()  # online compaction
        torch.cuda.synchronize()
        st2 = ar.store.probe_stats()
        host2 = _host_stats(ar)
        for k, v in host2.items():
            assert st2[k] == v, (k, st2[k], v)
        print(dict(load=load, emb=emb, before=(st1["hit_mean"], st1["miss_mean"], st1["tombstones"]),
                   after=(st2["hit_mean"], st2["miss_mean"], st2["tombstones"]), rehash=r))
        assert st2["live"] == live.size and st2["busy"] == 0
        assert r["moved"] > 0 or r["reclaimed"] > 0
        assert st2["tombstones"] < st1["tombstones"]
        assert st2["miss_mean"] < st1["miss_mean"] or st1["virgin"] == 0  # no cluster end: nothing to reclaim
        assert st2["hit_mean"] <= st1["hit_mean"] + 1e-9
        assert st2["rebuilds"] == 1 and st2["moved"] == r["moved"] and st2["reclaimed"] == r["reclaimed"]
        assert ar.store.maint_seq() == 2  # one pass opened and closed
        _check_values(ar, live)
        _no_duplicates(ar, live.size)
        dead = np.setdiff1d(np.arange(nxt), live)[:5000]
        sd, _, _ = ar.get(_keys(dead))
        assert bool((sd == -2).all())
        if emb:
            _check_vectors(ar, live, vec)
        # the exclusive full rebuild: no tombstone left at all
        r2 = ar.store.rehash(full=True)
        torch.cuda.synchronize()
        st3 = ar.store.probe_stats()
        assert st3["tombstones"] == 0 and r2["moved"] == live.size and r2["skipped"] == 0
        _check_values(ar, live)
        if emb:
            _check_vectors(ar, live, vec)
        # the store keeps working: inserts after the passes
        new = np.arange(nxt, nxt + 100)
        V, Lv = format_values(100, 1, 32, 64, ids=torch.as_tensor(new, device="cuda"))
        assert int((ar.set(_keys(new), V, Lv) != 0).sum()) == 0
    finally:
        ar.close()


def _check_vectors(ar, live, vec):
    """fp32 vectors, the side region's bf16 copy and norms at each key's (new) slot, and the batched
    search ABI against a float64 brute force over the same vectors."""
    import torch
    st, got = ar.get_embeddings(_keys(live))
    assert int((st != 0).sum()) == 0
    assert torch.equal(got, vec)
    st, idx = ar.meta("find", _keys(live))
    torch.cuda.synchronize()
    nrm2, v16 = ar.vec16_view()
    sl = idx.long()
    assert torch.equal(v16[sl], vec.bfloat16())
    assert torch.allclose(nrm2[sl], (vec * vec).sum(1), rtol=1e-5)
    occ = torch.zeros(ar.slots, dtype=torch.bool, device="cuda")
    occ[sl] = True
    assert bool((nrm2[~occ] == 0).all())  # vacated slots are never search candidates
    from test_search_gpu import _c_search_batch
    q = vec[:16].cpu().numpy().astype(np.float32) + 0.01
    hits = _c_search_batch(ar.store, q, 5)
    v64 = vec.cpu().numpy().astype(np.float64)
    vn = np.linalg.norm(v64, axis=1)
    for i in range(q.shape[0]):
        sims = v64 @ q[i].astype(np.float64) / (vn * np.linalg.norm(q[i]))
        want = live[int(np.argmax(sims))]
        assert hits[i][0] is not None and hits[i][0][0] == "c%09d" % want, (hits[i][0], want)


@pytest.mark.parametrize("emb", [False, True])
def test_rehash_online_beside_live_kv_steps(uniq, emb):
    """The online compaction runs while fused KV steps (updates + gets of live keys, gets of removed
    keys) keep running on another stream: 0 false misses, 0 duplicate keys, every value intact (the
    last version written), and the probe chains shorter afterwards (verdict round 5, item 2)."""
    import threading
    import torch
    from libsplinter_amd.ops.arena import HbmArena, KvStreams, format_values
    slots = 1 << 22 if not emb else 1 << 17
    ar = HbmArena.create(f"{uniq}", slots=slots, max_val=64, embeddings=emb)
    kv = KvStreams(4, 4)
    try:
        rng = np.random.default_rng(11)
        live, nxt = _churn(ar, slots, 0.9, rng)
        vec = None
        if emb:
            vec = torch.randn(live.size, 768, device="cuda")
            assert int((ar.set_embeddings(_keys(live), vec) != 0).sum()) == 0
        torch.cuda.synchronize()
        st1 = ar.store.probe_stats()
        dead = np.setdiff1d(np.arange(nxt), live)[:2048]
        ver = np.ones(live.size, dtype=np.int64)
        res, err = [], []

        passes = 6

        def worker():
            try:
                for _ in range(passes):
                    res.append(ar.store.rehash())
            except Exception as e:  # noqa: BLE001
                err.append(e)

        from libsplinter_amd.ops.arena import _device_view
        seqv = _device_view(ar._side_base() + 256, 8, dtype=torch.int64)  # MaintRec::seq
        seqs = []

        n_set = n_get = min(131072, live.size // 8)
        # the ops of every step come from one permutation, and a batch's inputs are built before any
        # of its steps is queued: the fused KV grid fills every CU while it runs, so a pass's kernels
        # interleave with KV steps only at kernel boundaries -- many steps must be queued back to back
        # when the pass opens
        perm = rng.permutation(live.size)
        # the removed keys' gets are spread through every step's get batch, so every workgroup of
        # the fused grid has some (a miss is where an open pass shows: EAGAIN)
        nd = 512
        dmask = np.zeros(n_get + nd, dtype=bool)
        dmask[np.linspace(0, n_get + nd - 1, nd).astype(np.int64)] = True
        dmask_d = torch.as_tensor(dmask, device="cuda")
        steps, false_miss, live_again, dead_seen = 0, 0, 0, {}
        t = threading.Thread(target=worker)
        t_started = False
        per_batch = 24
        while (not t_started or t.is_alive() or steps < 2 * per_batch) and steps < 4000:
            inputs = []
            for b in range(per_batch):
                st_i = steps + b
                off = (st_i * (n_set + n_get)) % (live.size - n_set - n_get)
                pick = perm[off:off + n_set + n_get]
                si, gi = pick[:n_set], pick[n_set:]
                V, Lv = format_values(n_set, st_i + 2, 40, 64, ids=torch.as_tensor(live[si], device="cuda"))
                sk = _keys(live[si])
                gk = torch.empty((n_get + nd, 16), dtype=torch.uint8, device="cuda")
                gk[~dmask_d] = _keys(live[gi])
                gk[dmask_d] = _keys(dead[:nd])
                inputs.append((si, gi, sk, V, Lv, gk))
            torch.cuda.synchronize()
            if not t_started:  # the first batch is queued behind the first pass's opening
                import time
                seq0 = ar.store.maint_seq()
                t.start()
                t_started = True
                t_end = time.time() + 10
                while ar.store.maint_seq() == seq0 and t.is_alive() and time.time() < t_end:
                    pass
            batch = []
            for si, gi, sk, V, Lv, gk in inputs:
                sst = torch.empty(n_set, dtype=torch.int32, device="cuda")
                go = torch.empty(gk.shape[0], 64, dtype=torch.uint8, device="cuda")
                gl = torch.empty(gk.shape[0], dtype=torch.int32, device="cuda")
                gst = torch.empty(gk.shape[0], dtype=torch.int32, device="cuda")
                kv.step(ar, sk, V, Lv, sst, gk, go, gl, gst)
                seqs.append(seqv.clone())  # the seq as the stream passes this step: odd = a pass was running
                batch.append((si, gi, sst, go, gl, gst, ver[gi].copy()))
                ver[si] = steps + 2
                steps += 1
            torch.cuda.synchronize()
            for si, gi, sst, go, gl, gst, gv in batch:
                s_set, s_get = sst.cpu().numpy(), gst.cpu().numpy()
                assert int((s_set != 0).sum()) == 0, np.unique(s_set, return_counts=True)
                live_st, dead_st = s_get[~dmask], s_get[dmask]
                false_miss += int((live_st == -2).sum())
                live_again += int((live_st == -11).sum())
                for v, c in zip(*np.unique(dead_st, return_counts=True)):
                    dead_seen[int(v)] = dead_seen.get(int(v), 0) + int(c)
                o, ln = go.cpu().numpy()[~dmask], gl.cpu().numpy()[~dmask]
                for i in range(0, n_get, 61):
                    if live_st[i] == 0:
                        v = bytes(o[i, : ln[i]])
                        assert v.startswith(b"ver:%d|id:%d|" % (gv[i], live[gi[i]])), (v[:20], gv[i], live[gi[i]])
        t.join()
        assert not err, err
        assert len(res) == passes
        overlapped = int(sum(int(x.item()) & 1 for x in seqs))
        st2 = ar.store.probe_stats()
        print(dict(emb=emb, steps=steps, overlapped_steps=overlapped, rehash=res, dead_status=dead_seen,
                   live_again=live_again,
                   before=(st1["miss_mean"], st1["tombstones"]), after=(st2["miss_mean"], st2["tombstones"])))
        assert false_miss == 0 and live_again == 0, (false_miss, live_again)
        assert set(dead_seen) <= {-2, -11}
        assert st2["live"] == live.size and st2["busy"] == 0
        assert st2["tombstones"] < st1["tombstones"]
        assert st2["miss_mean"] < st1["miss_mean"] or st1["virgin"] == 0
        assert ar.store.maint_seq() == 2 * passes
        # (whether a step's kernels ran inside a pass depends on the queue scheduler: reported, and
        # pinned deterministically by test_kv_step_inside_an_open_maintenance_window)
        _check_values(ar, live, ver)
        _no_duplicates(ar, live.size)
        sd, _, _ = ar.get(_keys(dead))
        assert bool((sd == -2).all())
        if emb:
            _check_vectors(ar, live, vec)
    finally:
        kv.close()
        ar.close()


def test_vec16_copy_follows_every_vector_writer(uniq):
    import torch
    from libsplinter_amd.ops.arena import HbmArena, format_values
    from libsplinter_amd import Store
    ar = HbmArena.create(f"{uniq}", slots=4096, max_val=64, embeddings=True)
    try:
        assert ar.has_vec16
        ids = np.arange(300)
        K = _keys(ids)
        V, Lv = format_values(300, 1, 32, 64, ids=torch.as_tensor(ids, device="cuda"))
        assert int((ar.set(K, V, Lv) != 0).sum()) == 0
        vec = torch.randn(300, 768, device="cuda")
        assert int((ar.set_embeddings(K, vec) != 0).sum()) == 0  # batched writer (k_embed_set)
        st, idx = ar.meta("find", K)
        torch.cuda.synchronize()
        nrm2, v16 = ar.vec16_view()
        sl = idx.long()
        assert torch.equal(v16[sl], vec.bfloat16())
        assert torch.allclose(nrm2[sl], (vec * vec).sum(1), rtol=1e-5)
        # per-call writer (the ring worker) through the Store API
        s = ar.store
        one = np.random.default_rng(1).standard_normal(768).astype(np.float32)
        key = bytes(K[7].cpu().numpy()).split(b"\0", 1)[0].decode()
        s.set_embedding(key, one)
        torch.cuda.synchronize()
        assert torch.equal(v16[sl[7]], torch.from_numpy(one).cuda().bfloat16())
        assert abs(nrm2[sl[7]].item() - float((one.astype(np.float64) ** 2).sum())) < 1e-3
        # unset and retrain clear the copy (norm 0: never a search candidate)
        assert int((ar.unset(K[:5]) < 0).sum()) == 0
        key9 = bytes(K[9].cpu().numpy()).split(b"\0", 1)[0].decode()
        assert s.retrain(key9)
        torch.cuda.synchronize()
        assert bool((nrm2[sl[:5]] == 0).all()) and nrm2[sl[9]].item() == 0.0
        # checkpoint / restore rebuilds the copy from the restored vectors
        import os
        import tempfile
        path = os.path.join(tempfile.mkdtemp(), "ck.spl")
        ar.checkpoint(path)
        nrm2.zero_()
        ar.restore(path)
        torch.cuda.synchronize()
        assert torch.equal(v16[sl[20:]], vec[20:].bfloat16())
        assert bool((nrm2[sl[20:]] > 0).all()) and bool((nrm2[sl[:5]] == 0).all())
        del Store
    finally:
        ar.close()


def test_vec16_written_by_the_encoder_pool(uniq):
    """The encoder's fused mean-pool write-back (nomic_kernels.hip k_pool) fills the copy too."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena
    from libsplinter_amd.models.nomic import smoke_embed
    ar = HbmArena.create(f"{uniq}", slots=1024, max_val=256, embeddings=True)
    try:
        from libsplinter_amd.ops.arena import pack_keys, pack_values
        keys = [f"doc-{i}" for i in range(4)]
        K = pack_keys(keys, 16)
        V, L = pack_values([b"x"] * 4, 256)
        assert (ar.set(K, V, L) == 0).all()
        smoke_embed(ar, K)
        st, idx = ar.meta("find", K)
        _, vecs = ar.get_embeddings(K)
        torch.cuda.synchronize()
        nrm2, v16 = ar.vec16_view()
        sl = idx.long()
        assert torch.equal(v16[sl], vecs.bfloat16())
        assert torch.allclose(nrm2[sl], (vecs * vecs).sum(1), rtol=1e-4)
    finally:
        ar.close()


def test_kv_step_inside_an_open_maintenance_window(uniq):
    """While a maintenance pass is open (the side header's seq odd), a fused KV step keeps serving
    hits -- gets and updates of live keys -- and answers every ABSENT outcome (a miss, the insert of
    a new key) with EAGAIN instead of "missing" or a possibly duplicate insert; once the pass closes
    the same ops resolve (arena_dev.hpp online maintenance; reference splinter.c:431-464: a miss
    only after the whole chain was seen)."""
    import ctypes
    import os
    import torch
    from libsplinter_amd import _native as N
    from libsplinter_amd.ops.arena import HbmArena, KvStreams, _stream, format_values
    ar = HbmArena.create(f"{uniq}", slots=1 << 20, max_val=64, embeddings=False)
    kv = KvStreams(2, 2)
    L = N.hip_lib()
    L.spl_arena_maint_mark.argtypes = [N.Arena, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                       ctypes.c_void_p]
    L.spl_arena_maint_mark.restype = ctypes.c_int
    ok = torch.zeros(1, dtype=torch.int64, device="cuda")
    opened = False
    try:
        live = np.arange(200_000)
        V, Lv = format_values(live.size, 1, 40, 64, ids=torch.as_tensor(live, device="cuda"))
        assert int((ar.set(_keys(live), V, Lv) != 0).sum()) == 0
        new = np.arange(300_000, 300_000 + 4096)  # never inserted
        upd, hit = live[:8192], live[10_000:18_192]

        def step(set_ids, get_ids, ver, retries=8):
            sk = _keys(set_ids) if set_ids is not None else None
            Vs, Ls = (format_values(set_ids.size, ver, 40, 64, ids=torch.as_tensor(set_ids, device="cuda"))
                      if set_ids is not None else (None, None))
            gk = _keys(get_ids) if get_ids is not None else None
            n_g = get_ids.size if get_ids is not None else 0
            sst = torch.full((max(set_ids.size if set_ids is not None else 0, 1),), 99, dtype=torch.int32,
                             device="cuda")
            go = torch.zeros(max(n_g, 1), 64, dtype=torch.uint8, device="cuda")
            gl = torch.zeros(max(n_g, 1), dtype=torch.int32, device="cuda")
            gst = torch.full((max(n_g, 1),), 99, dtype=torch.int32, device="cuda")
            kv.step(ar, sk, Vs, Ls, sst if sk is not None else None, gk, go if gk is not None else None,
                    gl if gk is not None else None, gst if gk is not None else None, retries=retries)
            torch.cuda.synchronize()
            return sst.cpu().numpy(), gst.cpu().numpy(), go.cpu().numpy(), gl.cpu().numpy()

        assert L.spl_arena_maint_mark(ar.desc, 1, os.getpid(), 0, ok.data_ptr(), _stream()) == 0
        torch.cuda.synchronize()
        assert int(ok.item()) == 1
        opened = True
        assert ar.store.maint_seq() & 1
        sst, gst, go, gl = step(np.concatenate([upd, new]), np.concatenate([hit, new]), 2)
        assert (sst[:upd.size] == 0).all()           # updates of present keys go through
        assert (sst[upd.size:] == -11).all()         # inserts wait for the pass (never a duplicate)
        assert (gst[:hit.size] == 0).all()           # hits are served
        assert (gst[hit.size:] == -11).all()         # misses are EAGAIN, never "missing"
        for i in range(0, hit.size, 97):
            assert bytes(go[i, :gl[i]]).startswith(b"ver:1|id:%d|" % hit[i])
        assert L.spl_arena_maint_mark(ar.desc, 0, 0, 0, ok.data_ptr(), _stream()) == 0
        torch.cuda.synchronize()
        opened = False
        assert ar.store.maint_seq() % 2 == 0
        _, gst, _, _ = step(None, new, 0)
        assert (gst == -2).all()                     # closed: the absent keys are absent
        sst, _, _, _ = step(new, None, 3)
        assert (sst == 0).all()                      # and insert once
        sst2, gst, go, gl = step(None, np.concatenate([upd, new]), 0)
        assert (gst == 0).all()
        for i in range(0, gst.size, 97):
            want = b"ver:2|" if i < upd.size else b"ver:3|"
            assert bytes(go[i, :gl[i]]).startswith(want)
        _no_duplicates(ar, live.size + new.size)
    finally:
        if opened:
            L.spl_arena_maint_mark(ar.desc, 0, 0, 0, ok.data_ptr(), _stream())
            torch.cuda.synchronize()
        kv.close()
        ar.close()

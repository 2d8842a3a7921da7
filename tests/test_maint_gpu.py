"""Maintenance passes of an HBM arena (csrc/hip/arena_maint.hip) and the side region's bf16 vector
copy: probe-chain statistics against a host recomputation from the raw slot words, the tombstone
rebuild under insert / unset churn at 50 % and 90 % load (every live key still found, absent keys
still missing, misses shorter after), and the bf16 copy kept in step by every embedding writer."""
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


@pytest.mark.parametrize("load", [0.5, 0.9])
def test_probe_stats_and_rehash_under_churn(uniq, load):
    import torch
    from libsplinter_amd.ops.arena import HbmArena, format_values
    slots = 1 << 16
    ar = HbmArena.create(f"{uniq}", slots=slots, max_val=64, embeddings=False)
    try:
        rng = np.random.default_rng(7)
        n = int(slots * load)
        live = np.arange(n)
        nxt = n
        V, Lv = format_values(n, 1, 32, 64, ids=torch.as_tensor(live, device="cuda"))
        assert int((ar.set(_keys(live), V, Lv) != 0).sum()) == 0
        st0 = ar.store.probe_stats()
        for cyc in range(8):  # unset 30 % of the live keys, insert as many new ones
            kill = rng.choice(live.size, size=int(0.3 * live.size), replace=False)
            gone = live[kill]
            assert int((ar.unset(_keys(gone)) < 0).sum()) == 0
            live = np.delete(live, kill)
            new = np.arange(nxt, nxt + gone.size)
            nxt += gone.size
            V, Lv = format_values(new.size, 1, 32, 64, ids=torch.as_tensor(new, device="cuda"))
            assert int((ar.set(_keys(new), V, Lv) != 0).sum()) == 0
            live = np.concatenate([live, new])
        torch.cuda.synchronize()
        st1 = ar.store.probe_stats()
        host = _host_stats(ar)
        for k, v in host.items():
            assert st1[k] == v, (k, st1[k], v)
        assert st1["live"] == live.size and st1["tombstones"] > 0
        assert st1["miss_mean"] > st0["miss_mean"]  # tombstones lengthen misses
        r = ar.store.rehash()
        torch.cuda.synchronize()
        st2 = ar.store.probe_stats()
        host2 = _host_stats(ar)
        for k, v in host2.items():
            assert st2[k] == v, (k, st2[k], v)
        print(dict(load=load, before=(st1["hit_mean"], st1["miss_mean"], st1["tombstones"]),
                   after=(st2["hit_mean"], st2["miss_mean"], st2["tombstones"]), rehash=r))
        assert st2["live"] == live.size
        assert r["moved"] > 0 or r["reclaimed"] > 0
        if st1["virgin"] * 20 < slots:  # merged clusters: the full rebuild (no tombstone left)
            assert st2["tombstones"] == 0 and r["moved"] == live.size and r["skipped"] == 0
        assert st2["tombstones"] < st1["tombstones"] and st2["miss_mean"] < st1["miss_mean"]
        assert st2["hit_mean"] <= st1["hit_mean"] + 1e-9
        assert st2["rebuilds"] == 1 and st2["moved"] == r["moved"] and st2["reclaimed"] == r["reclaimed"]
        # every live key still found with its own value; removed keys still missing
        sts, out, lens = ar.get(_keys(live))
        assert int((sts != 0).sum()) == 0
        o, ln = out.cpu().numpy(), lens.cpu().numpy()
        for i in range(0, live.size, max(1, live.size // 2000)):
            v = bytes(o[i, : ln[i]])
            assert int(v.split(b"|id:", 1)[1].split(b"|", 1)[0]) == live[i]
        dead = np.setdiff1d(np.arange(nxt), live)[:5000]
        sd, _, _ = ar.get(_keys(dead))
        assert bool((sd == -2).all())
        # the store keeps working: inserts after the rebuild
        new = np.arange(nxt, nxt + 100)
        V, Lv = format_values(100, 1, 32, 64, ids=torch.as_tensor(new, device="cuda"))
        assert int((ar.set(_keys(new), V, Lv) != 0).sum()) == 0
    finally:
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

"""Fused GPU top-k search vs the scalar reference ranking; daemon end to end."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_search_matches_reference(uniq):
    import torch
    from libsplinter_amd.ops.arena import HbmArena, pack_keys, pack_values
    from libsplinter_amd.ops.search import VectorSearch, search_reference
    a = HbmArena.create(uniq, slots=8192, max_val=64, embeddings=True)
    try:
        n = 5000
        K = pack_keys([f"v{i}" for i in range(n)], 16)
        V, L = pack_values([b"x"] * n, 16)
        assert (a.set(K, V, L) == 0).all()
        g = torch.Generator().manual_seed(0)
        vecs = torch.randn(n, 768, generator=g)
        vecs[7] = 0  # an un-embedded slot must be skipped
        assert (a.set_embeddings(K, vecs.cuda()) == 0).all()
        a.meta("set_label", K[:100], torch.full((100,), 1 << 4, dtype=torch.int64, device="cuda"))
        mat = a.embedding_matrix().cpu().numpy()
        occ = np.zeros(a.slots, bool)
        idx, _ = a.scan(3)
        occ[idx.cpu().numpy()] = True
        q = torch.randn(5, 768, generator=g)
        q[1] = vecs[42] * 2.0  # exact direction match -> sim 1
        vs = VectorSearch(a, grid=64)
        sidx, sim, dist = vs.search(q, k=10)
        for j in range(5):
            ref = search_reference(mat, occ, q[j].numpy(), 10)
            assert sidx[j].tolist() == [r[0] for r in ref]
            np.testing.assert_allclose(sim[j].cpu().numpy(), [r[1] for r in ref], rtol=1e-4, atol=1e-5)
            np.testing.assert_allclose(dist[j].cpu().numpy(), [r[2] for r in ref], rtol=1e-4, atol=1e-3)
        assert vs.keys_of(sidx[1:2])[0][0] == "v42"
        # label filter + min-sim filter
        li, ls, _ = vs.search(q[:1], k=5, label_mask=1 << 4)
        lab = {vs.keys_of(li)[0][t] for t in range(5)}
        assert all(int(x[1:]) < 100 for x in lab)
        fi, fs, _ = vs.search(q[1:2], k=5, min_sim=0.99)
        assert fi[0, 0].item() >= 0 and (fi[0, 1:] == -1).all()
    finally:
        a.close()


def test_splinference_daemon_oneshot(uniq):
    """Reference daemon contract on a host store: label-bound keys get vectors,
    WAITING cleared, oversize input flagged CONTEXT_EXCEEDED."""
    from libsplinter_amd import Store, unlink
    s = Store.create(uniq, slots=256, max_val=8192, embeddings=True)
    try:
        for i in range(20):
            s.set(f"doc{i}", f"the vector store document number {i} about search")
            s.set_type(f"doc{i}", 1 << 7)
            s.set_label(f"doc{i}", 0x1 | 0x40)
        s.set("huge", "a " * 2000)  # ~2000 tokens > 0.9 * n_ctx (2048)
        r = subprocess.run([sys.executable, "-m", "libsplinter_amd.daemons.splinference", "--oneshot",
                            "--random-init", "--layers", "2", uniq, "none.gguf", "3"],
                           cwd=ROOT, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        for i in range(20):
            v = s.get_embedding(f"doc{i}")
            assert v is not None and np.linalg.norm(v) > 0
            assert not (s.snapshot(f"doc{i}")["bloom"] & 0x40)
        assert s.snapshot("huge")["bloom"] & 0x80
        assert s.get("huge").startswith(b"CONTEXT_EXCEEDED")
    finally:
        s.close()
        unlink(uniq)


def _clustered(n, g, centers=64, noise=0.35):
    import torch
    c = torch.randn(centers, 768, generator=g)
    lab = torch.randint(0, centers, (n,), generator=g)
    return c[lab] + noise * torch.randn(n, 768, generator=g)


@pytest.mark.parametrize("nq", [40, 300])
def test_search_batch_matches_exact(uniq, nq):
    """MFMA batched search (bf16 threshold passes + fp32 re-score) == exact fp32 kernel,
    including a partial last tile, un-embedded slots, label mask, min-sim and max-dist."""
    import torch
    from libsplinter_amd.ops.arena import HbmArena, pack_keys, pack_values
    from libsplinter_amd.ops.search import VectorSearch
    a = HbmArena.create(uniq, slots=20011, max_val=32, embeddings=True)
    try:
        n = 15000
        K = pack_keys([f"e{i}" for i in range(n)], 16)
        V, L = pack_values([b"x"] * n, 16)
        assert (a.set(K, V, L) == 0).all()
        g = torch.Generator().manual_seed(1)
        vecs = _clustered(n, g)
        vecs[11] = 0
        vecs[12] = 1e-8  # below the exact kernel's norm floor
        assert (a.set_embeddings(K, vecs.cuda()) == 0).all()
        a.meta("set_label", K[::3], torch.full((len(range(0, n, 3)),), 1 << 5, dtype=torch.int64, device="cuda"))
        q = _clustered(nq, g) * 3.0
        q[0] = vecs[100]
        vs = VectorSearch(a, grid=128)
        st = {}
        for kw in ({}, {"label_mask": 1 << 5}, {"min_sim": 0.6}, {"max_dist": 30.0}):
            i1, s1, d1 = vs.search_batch(q, k=10, stats=st, **kw)
            i0, s0, d0 = vs.search(q, k=10, **kw)
            assert torch.equal(i1, i0), kw
            assert torch.equal(s1, s0) and torch.equal(d1, d0), kw
            if "max_dist" not in kw:  # bounded distance: no sample threshold, every slot is a candidate
                assert st["overflow"] == 0 and st["candidates"] < nq * 2000, (kw, st)
        # tiny candidate cap: every query overflows and falls back to the exact kernel
        i2, _, _ = vs.search_batch(q, k=10, capb=1, stats=st)
        assert torch.equal(i2, vs.search(q, k=10)[0]) and st["overflow"] > 0
    finally:
        a.close()

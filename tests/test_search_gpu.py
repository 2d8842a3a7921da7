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

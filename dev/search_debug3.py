"""Debug: tests/test_search_gpu.py::test_search_batch_matches_exact[40] step by step."""
import os
import sys
import uuid

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from libsplinter_amd.ops.arena import HbmArena, pack_keys, pack_values  # noqa: E402
from libsplinter_amd.ops import search as S  # noqa: E402


def clustered(n, g, centers=64, noise=0.35):
    c = torch.randn(centers, 768, generator=g)
    lab = torch.randint(0, centers, (n,), generator=g)
    return c[lab] + noise * torch.randn(n, 768, generator=g)


name = "sd" + uuid.uuid4().hex[:8]
a = HbmArena.create(name, slots=20011, max_val=32, embeddings=True)
try:
    n = 15000
    K = pack_keys([f"e{i}" for i in range(n)], 16)
    V, L = pack_values([b"x"] * n, 16)
    assert (a.set(K, V, L) == 0).all()
    g = torch.Generator().manual_seed(1)
    vecs = clustered(n, g)
    vecs[11] = 0
    vecs[12] = 1e-8
    assert (a.set_embeddings(K, vecs.cuda()) == 0).all()
    a.meta("set_label", K[::3], torch.full((len(range(0, n, 3)),), 1 << 5, dtype=torch.int64, device="cuda"))
    nq = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    q = clustered(nq, g) * 3.0
    q[0] = vecs[100]
    vs = S.VectorSearch(a, grid=128)
    for capb in (64, 4096):
        st = {}
        i1, s1, d1 = vs.search_batch(q, k=10, stats=st, capb=capb)
        i0, s0, d0 = vs.search(q, k=10)
        bad = (i1 != i0).any(dim=1)
        print("capb", capb, "stats", st, "queries differing", int(bad.sum()), "of", nq)
        if bad.any():
            qq = int(bad.nonzero()[0])
            print("  q", qq, "batch", i1[qq].tolist(), s1[qq].tolist())
            print("  q", qq, "exact", i0[qq].tolist(), s0[qq].tolist())
finally:
    a.close()
    from libsplinter_amd import store as ST
    ST.unlink("hbm:" + name)

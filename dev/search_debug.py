"""Debug: MODE 0 per-tile max of the MFMA search pass vs a torch fp32 reference (small arena)."""
import os
import sys
import uuid

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from libsplinter_amd.ops.arena import HbmArena, pack_keys, pack_values  # noqa: E402
from libsplinter_amd.ops import search as S  # noqa: E402

name = "sd" + uuid.uuid4().hex[:8]
a = HbmArena.create(name, slots=4096, max_val=32, embeddings=True)
try:
    n = 4096
    K = pack_keys([f"e{i}" for i in range(n)], 16)
    V, L = pack_values([b"x"] * n, 16)
    assert (a.set(K, V, L) == 0).all()
    g = torch.Generator().manual_seed(1)
    vecs = torch.randn(n, 768, generator=g)
    assert (a.set_embeddings(K, vecs.cuda()) == 0).all()
    # slot index of each key
    idx, _, _ = S.VectorSearch(a).search(vecs[:4].cuda(), k=1)
    print("self-search slots", idx.flatten().tolist())
    vs = S.VectorSearch(a)
    L_ = vs.L
    nq = 40
    q = torch.randn(nq, 768, generator=g).cuda()
    qb = torch.zeros(256, 768, dtype=torch.bfloat16, device="cuda")
    qb[:nq] = (q / q.norm(dim=1, keepdim=True)).to(torch.bfloat16)
    qf = qb.view(16, 16, 24, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
    T = S.TILE
    tiles = 4096 // T
    bmax = torch.full((tiles, nq), -7.0, dtype=torch.float32, device="cuda")
    rc = L_.spl_search_mma_pass(a.desc, qf.data_ptr(), nq, 0, 4096, 0, 0, None, bmax.data_ptr(), None, None, 0, 64,
                                torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    print("rc", rc)
    # reference: vectors read back from the arena slots (slot order)
    emb = a.embedding_matrix()
    print("have view", emb is not None)
    if emb is not None:
        E = emb.float()
        E = E / E.norm(dim=1, keepdim=True).clamp_min(1e-30)
        Qn = qb[:nq].float()
        sc = E @ Qn.T  # [slots, nq]
        ref = sc.view(tiles, T, nq).max(dim=1).values
        d = (bmax - ref).abs()
        print("max |bmax - ref|", float(d.max()), "tiles bad", int((d > 0.02).any(dim=1).sum()), "of", tiles)
        bad = (d > 0.02).nonzero()[:10].tolist()
        print("bad (tile, q)", bad)
        for t, qq in bad[:3]:
            print(t, qq, float(bmax[t, qq]), float(ref[t, qq]), int(sc[t * T:(t + 1) * T, qq].argmax()))
finally:
    a.close()
    from libsplinter_amd import store as ST
    ST.unlink("hbm:" + name) if not name.startswith("hbm:") else None

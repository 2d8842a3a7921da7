"""Debug: the failing batch-search case -- MODE 0 bmax and MODE 1 candidates vs torch fp32."""
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
slots = int(sys.argv[1]) if len(sys.argv) > 1 else 20011
grid = int(sys.argv[2]) if len(sys.argv) > 2 else 256
a = HbmArena.create(name, slots=slots, max_val=32, embeddings=True)
st = torch.cuda.current_stream().cuda_stream
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
    nq = 40
    q = clustered(nq, g) * 3.0
    q[0] = vecs[100]
    q = q.cuda()
    vs = S.VectorSearch(a, grid=128)
    Lb = vs.L
    qb = torch.zeros(256, 768, dtype=torch.bfloat16, device="cuda")
    qb[:nq] = (q / q.norm(dim=1, keepdim=True)).to(torch.bfloat16)
    qf = qb.view(16, 16, 24, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
    T = S.TILE
    E = a.embedding_matrix().float()
    nrm = E.norm(dim=1, keepdim=True)
    live = (nrm.flatten() > 0)
    En = E / nrm.clamp_min(1e-30)
    sc = En @ qb[:nq].float().T
    sc[~live] = -9
    sample = slots // T * T
    tiles = sample // T
    bmax = torch.full((tiles, nq), -7.0, device="cuda")
    assert Lb.spl_search_mma_pass(a.desc, qf.data_ptr(), nq, 0, sample, 0, 0, None, bmax.data_ptr(), None, None, 0,
                                  grid, st) == 0
    ref = sc[:sample].view(tiles, T, nq).max(dim=1).values
    ref[ref < -8] = -3.0e38
    d = (bmax - ref).abs()
    bad = (d > 0.02)
    print("MODE0 bad tile/q", int(bad.sum()), "of", bad.numel(), "tiles with a bad q", int(bad.any(dim=1).sum()))
    if bad.any():
        t, qq = bad.nonzero()[0].tolist()
        print("  e.g.", t, qq, float(bmax[t, qq]), float(ref[t, qq]), "rows", sc[t * T:(t + 1) * T, qq].topk(3))
    thr = (bmax.topk(10, dim=0).values[-1] - 2 * S.DELTA).contiguous()
    capb = 4096
    cnt = torch.zeros(nq, grid, dtype=torch.int32, device="cuda")
    cand = torch.full((nq * grid * capb,), -1, dtype=torch.int32, device="cuda")
    assert Lb.spl_search_mma_pass(a.desc, qf.data_ptr(), nq, 0, slots, 0, 1, thr.data_ptr(), None, cnt.data_ptr(),
                                  cand.data_ptr(), capb, grid, st) == 0
    torch.cuda.synchronize()
    cv = cand.view(nq, grid, capb)
    miss = extra = 0
    for qq in range(nq):
        got = set()
        for b in range(grid):
            c = int(cnt[qq, b])
            got |= set(cv[qq, b, :c].tolist())
        want = set((sc[:, qq] >= thr[qq] + 0.01).nonzero().flatten().tolist())
        if qq == 0:
            for x in (19262, 2029, 7040, 14234):
                print('slot', x, 'in cand', x in got, 'score', float(sc[x, 0]), 'thr', float(thr[0]), 'bmax tile', float(bmax[x // T, 0]) if x // T < tiles else None, 'ref tile', float(ref[x // T, 0]) if x // T < tiles else None)
        m = want - got
        miss += len(m)
        if m and qq < 3:
            r = sorted(m)[:8]
            print("q", qq, "missing", r, "tiles", [x // T for x in r], "rows", [x % T for x in r],
                  "scores", [round(float(sc[x, qq]), 3) for x in r], "thr", float(thr[qq]))
    print("MODE1 missing candidates", miss)
    i0, s0, _ = vs.search(q, k=10)
    got0 = set()
    for b in range(grid):
        got0 |= set(cv[0, b, :int(cnt[0, b])].tolist())
    print("exact top10 q0", i0[0].tolist(), [round(x, 4) for x in s0[0].tolist()])
    print("in cand", [int(x) in got0 for x in i0[0].tolist()])
    tv, ti = sc[:, 0].topk(10)
    print("torch top10 q0", ti.tolist(), [round(float(x), 4) for x in tv])
    lv = a.slot_view()
    for x in (19262, int(ti[3])):
        print("slot", x, "hash", int(lv[x, :8].view(torch.int64)), "norm", float(E[x].norm()))
finally:
    a.close()
    from libsplinter_amd import store as ST
    ST.unlink("hbm:" + name)

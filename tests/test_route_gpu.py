"""Routed exchange (route_kernels.hip spl_xr_pack / spl_xr_gather, arena_kernels.hip
spl_kvs_step_xr, parallel/xroute.py) and segmented set/get (arena_kernels.hip Seg) on the GPU."""
import os
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(n, world, vstride=256, vlen=150, seed=0):
    from libsplinter_amd.ops.arena import format_keys, format_values
    g = torch.Generator(device="cuda").manual_seed(seed)
    ids = torch.randint(0, 1 << 40, (n,), device="cuda", generator=g)
    K = format_keys(n, "rk", 12, 32, ids=ids)
    V, L = format_values(n, 3, vlen, vstride, ids=ids)
    return K, V, L


def _pack(K, V, L, world, rank, cap, vw):
    """spl_xr_pack into local staging blocks (the rccl transport's layout) -> (geom, buf, counts, lidx, pos)."""
    from libsplinter_amd import _native as N
    from libsplinter_amd.parallel.xroute import XGeom
    n, ks = K.shape[0], K.shape[1]
    g = XGeom(world, cap, cap, ks, vw)
    buf = torch.zeros(g.par_b, dtype=torch.uint8, device="cuda")
    tab = torch.tensor([buf.data_ptr() + g.req(0, d) for d in range(world)], dtype=torch.int64, device="cuda")
    counts = torch.empty(world, dtype=torch.int32, device="cuda")
    lidx = torch.full((cap,), -7, dtype=torch.int32, device="cuda")
    pos = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    vp = V.data_ptr() if V is not None else None
    lp = L.data_ptr() if L is not None else None
    rc = N.hip_lib().spl_xr_pack(K.data_ptr(), ks, vp, V.shape[1] if V is not None else 0, lp, n, world, rank, cap,
                                 tab.data_ptr(), g.off_sk if V is not None else g.off_gk, g.off_sl, g.off_sv,
                                 vw if V is not None else 0, counts.data_ptr(), lidx.data_ptr(), pos.data_ptr(), -1,
                                 None, None, s)
    assert rc == 0
    torch.cuda.synchronize()
    return g, buf, counts, lidx, pos


@pytest.mark.parametrize("world,rank,capmode", [(8, 3, "auto"), (3, 0, "auto"), (8, 5, "tight"), (2, 1, "auto")])
def test_xr_pack_matches_reference(world, rank, capmode):
    """Every remote op's record lands in row j of its owner's block (pos = d*cap + j, each row used
    once), own ops are listed in lidx and never copied, counts are the per-destination totals, and
    with a tight capacity exactly the excess ops of each destination come back pos = -1."""
    from libsplinter_amd.parallel.sharded import GpuShard, shard_of
    from libsplinter_amd.parallel.xroute import route_capacity
    n = 40000
    K, V, L = _setup(n, world)
    dest = shard_of(GpuShard(None).hash_keys(K), world)
    want = torch.bincount(dest, minlength=world)
    cap = route_capacity(n, world) if capmode == "auto" else int(want.min()) - 50
    g, buf, counts, lidx, pos = _pack(K, V, L, world, rank, cap, 160)
    assert torch.equal(counts.long(), want)
    full = pos == -1
    own = pos == -2
    rem = pos >= 0
    assert int(full.sum()) == int((want - cap).clamp(min=0).sum())
    assert torch.equal(own | full, (dest == rank) | full)
    assert int(own.sum()) == min(int(want[rank]), cap)
    ol = lidx[: int(own.sum())].long()
    assert torch.equal(torch.sort(ol).values, torch.nonzero(own).squeeze(1))
    p = pos[rem].long()
    assert torch.equal(p // cap, dest[rem]) and p.unique().numel() == p.numel()
    d, j = p // cap, p % cap
    for dd in range(world):
        if dd == rank:
            continue
        sel = d == dd
        if not sel.any():
            continue
        o = g.req(0, dd)
        keys = buf[o + g.off_sk: o + g.off_sk + cap * K.shape[1]].view(cap, K.shape[1])
        lens = buf[o + g.off_sl: o + g.off_sl + cap * 4].view(torch.int32)
        vals = buf[o + g.off_sv: o + g.off_sv + cap * 160].view(cap, 160)
        idx = torch.nonzero(rem).squeeze(1)[sel]
        assert torch.equal(keys[j[sel]], K[idx])
        assert torch.equal(lens[j[sel]], L[idx])
        assert torch.equal(vals[j[sel]], V[idx, :160])
    # gets: keys only
    g2, buf2, c2, l2, pos2 = _pack(K, None, None, world, rank, cap, 160)
    assert torch.equal(c2, counts) and int((pos2 >= 0).sum()) == int(rem.sum())
    if capmode == "auto":  # no block full: the same ops are remote (with a full one, which excess ops
        assert torch.equal(pos2 >= 0, rem)  # overflow depends on the order of the block atomics)


def test_xr_gather_matches_reference():
    """Remote ops read status / len / value row j of owner d's response block; full ops -> EAGAIN;
    own ops are left untouched (their results were written in place)."""
    from libsplinter_amd import _native as N
    from libsplinter_amd.parallel.xroute import XGeom
    world, cap, vw, n = 4, 500, 160, 3000
    g = XGeom(world, cap, cap, 16, vw)
    win = torch.zeros(g.par_b, dtype=torch.uint8, device="cuda")
    gen = torch.Generator(device="cuda").manual_seed(5)
    for o in range(world):
        b = g.resp(0, o)
        win[b + g.off_gs: b + g.off_gs + cap * 4].view(torch.int32).copy_(
            torch.where(torch.rand(cap, device="cuda", generator=gen) < 0.9, 0, -2).to(torch.int32))
        win[b + g.off_gl: b + g.off_gl + cap * 4].view(torch.int32).copy_(
            torch.randint(1, vw, (cap,), device="cuda", generator=gen, dtype=torch.int32))
        win[b + g.off_gv: b + g.off_gv + cap * vw].copy_(
            torch.randint(0, 256, (cap * vw,), device="cuda", generator=gen, dtype=torch.uint8))
    pos = torch.randint(0, world * cap, (n,), device="cuda", generator=gen, dtype=torch.int32)
    pos[::7] = -2
    pos[::11] = -1
    tab = torch.tensor([win.data_ptr() + g.resp(0, o) for o in range(world)], dtype=torch.int64, device="cuda")
    st = torch.full((n,), 99, dtype=torch.int32, device="cuda")
    ln = torch.full((n,), 77, dtype=torch.int32, device="cuda")
    out = torch.full((n, 256), 0xAB, dtype=torch.uint8, device="cuda")
    rc = N.hip_lib().spl_xr_gather(pos.data_ptr(), n, cap, tab.data_ptr(), g.off_gs, g.off_gl, g.off_gv, vw,
                                   st.data_ptr(), ln.data_ptr(), out.data_ptr(), 256,
                                   torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    for i in range(0, n, 13):
        p = int(pos[i])
        if p == -2:
            assert int(st[i]) == 99 and int(ln[i]) == 77 and (out[i] == 0xAB).all()
            continue
        if p == -1:
            assert int(st[i]) == -11 and int(ln[i]) == 0
            continue
        d, j = divmod(p, cap)
        b = g.resp(0, d)
        s_ = int(win[b + g.off_gs: b + g.off_gs + cap * 4].view(torch.int32)[j])
        assert int(st[i]) == s_
        if s_ == 0:
            assert int(ln[i]) == int(win[b + g.off_gl: b + g.off_gl + cap * 4].view(torch.int32)[j])
            assert torch.equal(out[i, :vw], win[b + g.off_gv + j * vw: b + g.off_gv + (j + 1) * vw])
        else:
            assert int(ln[i]) == 0


def test_xroute_world1_runs_in_place(uniq):
    """At world 1 every op is the rank's own: the routed step is the in-place fan-out on the client
    arrays (spl_kvs_step_xr, identity rows), with the same results as the plain batch kernels."""
    from libsplinter_amd.ops.arena import HbmArena, KvStreams
    from libsplinter_amd.parallel.sharded import GpuShard
    from libsplinter_amd.parallel.xroute import XRoute
    a = HbmArena.create(uniq, slots=1 << 16, max_val=256, embeddings=False)
    try:
        n = 20000
        K, V, L = _setup(n, 1)
        kvs = KvStreams(4, 4)
        xr = XRoute(GpuShard(a), n, n, 160, ks=32)
        assert xr.transport == "local"
        st, _, _, _ = xr.step(0, kvs, K, V, L, None)
        torch.cuda.synchronize()
        assert (st == 0).all()
        _, gs, gv, gl = xr.step(1, kvs, None, None, None, K)
        torch.cuda.synchronize()
        assert (gs == 0).all() and (gl == 150).all() and torch.equal(gv, V[:, :160])
        kvs.close()
    finally:
        a.close()


_PEER_WORKER = r"""
import os, sys, json, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
rank, world, transport = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
dist.init_process_group("gloo", rank=rank, world_size=world)
torch.cuda.set_device(0)
from libsplinter_amd.ops.arena import HbmArena, KvStreams, format_keys, format_values
from libsplinter_amd.parallel.sharded import GpuShard, ShardedKV
from libsplinter_amd.parallel.xroute import XRoute
a = HbmArena.create(f"xrp{os.environ['TAG']}r{rank}", slots=1 << 18, max_val=256, embeddings=False)
kvs = KvStreams(4, 4)
n, steps = 30000, 6
xr = XRoute(GpuShard(a), n, n, 160, ks=16, resp_group=dist.new_group(backend="gloo"), transport=transport)
res = {"transport": xr.transport, "direct": xr.direct}
outs = ([xr.outputs(p) for p in range(2)] if xr.direct else
        [(torch.empty(n, dtype=torch.int32, device="cuda"), torch.zeros((n, 160), dtype=torch.uint8, device="cuda"),
          torch.empty(n, dtype=torch.int32, device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"))
         for _ in range(2)])
bad = checked = setbad = 0
pend = None
batches = []
for i in range(steps + 1):
    cur = None
    if i < steps:
        ids = torch.arange(n, device="cuda") + (i * world + rank) * n   # this rank's keys of step i
        K = format_keys(n, "pk", 10, 16, ids=ids)
        V, L = format_values(n, 5 + i, 150, 256, ids=ids)
        gk = None
        if i >= 2:  # keys another rank set two steps ago
            src = (rank + 1) % world
            gids = torch.arange(n, device="cuda") + ((i - 2) * world + src) * n
            gk = format_keys(n, "pk", 10, 16, ids=gids)
            GV, GL = format_values(n, 5 + i - 2, 150, 256, ids=gids)
        batches.append((K, V, L, gk))
        xr.request(i, K, V, L, gk)
        o = outs[i & 1]
        xr.execute(i, kvs, *o)
        cur = (i, o, gk, (GV, GL) if gk is not None else None)
    if pend is not None:
        pi, (ss, gv, gl, gs), pgk, want = pend
        xr.respond(pi)
        xr.finish(pi, ss, gv, gl, gs)
        torch.cuda.synchronize()
        setbad += int((ss != 0).sum())
        if pgk is not None:
            ok = (gs == 0) & (gl == want[1]) & (gv == want[0][:, :160]).all(1)
            bad += int((~ok).sum())
            checked += n
    pend = cur
    dist.barrier()
# the API path over the same stores (rccl transport through gloo staging)
kv = ShardedKV(GpuShard(a))
allids = torch.arange(n * world * steps, device="cuda")[::97]
s_, v_, l_ = kv.get(format_keys(allids.numel(), "pk", 10, 16, ids=allids), width=160)
res.update(checked=checked, bad=bad, setbad=setbad, api_bad=int((s_ != 0).sum()), sync=xr.sync,
           sync_err=xr.sync_error())
print("RES " + json.dumps(res), flush=True)
xr.close()
kvs.close()
dist.barrier()
a.close()
dist.destroy_process_group()
"""


@pytest.mark.parametrize("transport,sync,direct", [("peer", "flags", "1"), ("peer", "coll", "1"), ("peer", "coll", "0"),
                                                   ("rccl", "coll", "0")])
def test_xroute_two_ranks_one_gpu(tmp_path, transport, sync, direct):
    """Two ranks (processes) on device 0 run the pipelined routed step through the exchange: the
    peer transport maps each other's windows (VMM dmabuf) and stores request rows directly, and
    either the owners write every result straight into the requester's client arrays (direct
    responses, no gather) or into response blocks the requester gathers; its steps are ordered by
    device-side posts into the windows (flags) or by the count / response collectives (coll); the
    rccl transport moves the blocks with collectives (gloo-staged here).  Gets of the keys another
    rank set two steps earlier must all return their values (integrity 0), and no device-side wait
    may give up."""
    import json
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    w = tmp_path / "w.py"
    w.write_text(_PEER_WORKER)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               REPO=root, TAG=str(os.getpid()), SPLINTER_XR_SYNC=sync, SPLINTER_XR_DIRECT=direct)
    ps = [subprocess.Popen([sys.executable, str(w), str(r), "2", transport], env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = []
    try:
        for p in ps:
            o, e = p.communicate(timeout=240)
            outs.append((p.returncode, o, e))
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
    for rc, o, e in outs:
        assert rc == 0, (o + e)[-3000:]
        line = [x for x in o.splitlines() if x.startswith("RES ")][-1]
        res = json.loads(line[4:])
        assert res["transport"] == transport and res["sync"] == sync and not res["sync_err"], res
        assert res["direct"] == (transport == "peer" and direct == "1"), res
        assert res["checked"] == 4 * 30000 and res["bad"] == 0 and res["setbad"] == 0 and res["api_bad"] == 0, res


def test_segmented_set_get_skip_dead_rows(uniq):
    from libsplinter_amd.ops.arena import HbmArena
    a = HbmArena.create(uniq, slots=1 << 16, max_val=256, embeddings=False)
    try:
        world, cap = 3, 1000
        K, V, L = _setup(world * cap, world)
        counts = torch.tensor([1000, 0, 371], dtype=torch.int32, device="cuda")
        live = (torch.arange(world * cap, device="cuda") % cap) < counts.repeat_interleave(cap)
        a.reset_stats()
        st = a.set_seg(K, V, L, counts, cap)
        torch.cuda.synchronize()
        assert (st[live] == 0).all() and (st[~live] == -22).all()
        # attempts count EAGAIN retries of racing inserts (stats[2]); dead rows count nowhere
        assert int(a.stats[1]) == int(live.sum()) and int(a.stats[0]) - int(a.stats[2]) == int(live.sum())
        # dead rows were not inserted; live rows read back through the plain and segmented gets
        s2, out, ln = a.get(K)
        assert (s2[live] == 0).all() and (s2[~live] == -2).all()
        assert torch.equal(out[live, :160], V[live, :160])
        s3, o3, l3 = a.get_seg(K, counts, cap, 160)
        assert (s3[live] == 0).all() and (s3[~live] == -22).all()
        assert torch.equal(o3[live], V[live, :160]) and (l3[live] == 150).all() and (l3[~live] == 0).all()
        # values longer than the response row: EMSGSIZE
        s4, _, _ = a.get_seg(K, counts, cap, 128)
        assert (s4[live] == -90).all()
    finally:
        a.close()


def test_chunked_all_to_all_rccl():
    """Equal-split all-to-alls above SPLINTER_A2A_CHUNK_BYTES go out in parts (an RCCL
    all_to_all_single of 1.5 GiB returned wrong bytes past 768 MiB): byte-exact up to 2.5 GiB."""
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "dev/debug/a2a_check.py", "--chunked"],
                       cwd=root, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "chunked 2560 MiB: mismatching bytes 0" in r.stdout

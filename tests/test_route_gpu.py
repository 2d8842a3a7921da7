"""C1 routing kernels (route_kernels.hip) and segmented set/get (arena_kernels.hip
Seg) against the torch references in parallel/routed.py."""
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


@pytest.mark.parametrize("world,capmode", [(8, "auto"), (3, "auto"), (8, "tight"), (1, "auto")])
def test_route_pack_matches_reference(world, capmode):
    from libsplinter_amd.parallel.routed import pack_ref, route_capacity
    from libsplinter_amd.parallel.sharded import GpuShard
    n = 100_003
    K, V, L = _setup(n, world)
    cap = route_capacity(n, world) if capmode == "auto" else n // world - 200
    sh = GpuShard(None)
    h = sh.hash_keys(K)
    c, pos, ko, lo, vo = sh.route_pack(K, V, L, 160, world, cap)
    rc, rpos, rko, rlo, rvo = pack_ref(h, K, V, L, 160, world, cap)
    torch.cuda.synchronize()
    assert torch.equal(c, rc)
    over = int((rc.to(torch.int64) - cap).clamp(min=0).sum())
    assert int((pos < 0).sum()) == over == int((rpos < 0).sum())
    if capmode == "auto":
        assert over == 0
    ok = pos >= 0
    # every placed op sits in its destination segment, exactly once
    assert torch.unique(pos[ok]).numel() == int(ok.sum())
    assert torch.equal(ko[pos[ok]], K[ok])
    assert torch.equal(lo[pos[ok]], L[ok])
    assert torch.equal(vo[pos[ok]], V[ok, :160])
    dest = torch.div(pos[ok], cap, rounding_mode="floor")
    from libsplinter_amd.parallel.sharded import shard_of
    assert torch.equal(dest, shard_of(h[ok], world))
    # key-only pack (get requests)
    c2, pos2, ko2, lo2, vo2 = sh.route_pack(K, None, None, 0, world, cap)
    assert lo2 is None and vo2 is None and torch.equal(c2, rc)
    assert torch.equal(ko2[pos2[pos2 >= 0]], K[pos2 >= 0])


def test_route_gather_matches_reference():
    from libsplinter_amd.parallel.routed import gather_ref
    from libsplinter_amd.parallel.sharded import GpuShard
    n, rows, w = 50_001, 60_000, 160
    g = torch.Generator(device="cuda").manual_seed(1)
    pos = torch.randperm(rows, device="cuda", generator=g)[:n].to(torch.int64)
    pos[::97] = -1
    rst = torch.randint(-100, 5, (rows,), device="cuda", generator=g, dtype=torch.int32)
    rl = torch.randint(0, 200, (rows,), device="cuda", generator=g, dtype=torch.int32)
    rv = torch.randint(0, 256, (rows, w), device="cuda", generator=g, dtype=torch.int32).to(torch.uint8)
    sh = GpuShard(None)
    st, v, ln = sh.route_gather(pos, rst, rl, rv, w)
    est, ev, eln = gather_ref(pos, rst, rl, rv, w)
    torch.cuda.synchronize()
    assert torch.equal(st, est) and torch.equal(ln, eln)
    ok = pos >= 0
    assert torch.equal(v[ok], ev[ok])
    st2 = sh.route_gather(pos, rst)[0]
    assert torch.equal(st2, est)
    # narrower client rows: only the first ostride bytes are copied
    out = torch.zeros((n, 64), dtype=torch.uint8, device="cuda")
    sh.route_gather(pos, rst, rl, rv, w, out=out)
    assert torch.equal(out[ok], ev[ok, :64])


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

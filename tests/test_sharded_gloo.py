"""Cross-shard collectives C1-C6 (parallel/sharded.py) on gloo, world_size 2 and 3.

Same code path as the RCCL run in bench.py, with HostShard (a host store per
rank, CPU tensors) standing in for the HBM arena.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _keys(names, width=32):
    out = torch.zeros((len(names), width), dtype=torch.uint8)
    for i, n in enumerate(names):
        b = n.encode()
        out[i, : len(b)] = torch.tensor(list(b), dtype=torch.uint8)
    return out


def _vals(vals, width=64):
    out = torch.zeros((len(vals), width), dtype=torch.uint8)
    for i, v in enumerate(vals):
        out[i, : len(v)] = torch.tensor(list(v), dtype=torch.uint8)
    return out, torch.tensor([len(v) for v in vals], dtype=torch.int32)


def _worker(rank, world, port, base, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from libsplinter_amd import Store, unlink
        from libsplinter_amd.parallel.sharded import HostShard, ShardedKV, decode_keys
        name = f"{base}_r{rank}"
        st = Store.create(name, slots=1024, max_val=128, embeddings=True)
        kv = ShardedKV(HostShard(st))
        # ---- C1 set/get across shards: every rank writes its own 60 keys
        mine = [f"r{rank}_k{i}" for i in range(60)]
        K = _keys(mine)
        V, L = _vals([f"val-{n}".encode() for n in mine])
        assert (kv.set(K, V, L) == 0).all()
        dist.barrier()
        # each key landed only on its owner shard
        own = kv.owned_mask(K)
        local = set(st.list())
        for n, o in zip(mine, own.tolist()):
            assert (n in local) == o or not o, n
        allk = [f"r{r}_k{i}" for r in range(world) for i in range(60)]
        s_, v_, l_ = kv.get(_keys(allk))
        assert (s_ == 0).all()
        for i, n in enumerate(allk):
            assert bytes(v_[i, : l_[i]].numpy()) == f"val-{n}".encode()
        # local store holds exactly the keys this rank owns
        owned_all = kv.owned_mask(_keys(allk))
        assert sorted(st.list()) == sorted(n for n, o in zip(allk, owned_all.tolist()) if o)
        # ---- integer_op routed: everyone increments the same counter
        ctr = _keys(["counter"])
        # collectives need every rank: non-zero ranks contribute empty batches
        cv, cl = _vals([(0).to_bytes(8, "little")] if rank == 0 else [])
        assert (kv.set(ctr[: 1 if rank == 0 else 0], cv, cl) == 0).all()
        es_, ep_ = kv.meta("epoch", ctr)
        assert int(es_[0]) == 0 and int(ep_[0]) >= 2
        # BIGUINT typing is done by the owner locally (no routed set_type op in the reference API batch)
        if kv.owned_mask(ctr)[0]:
            st.set_type("counter", 1 << 2)
        dist.barrier()
        stt, res = kv.integer_op(ctr.repeat(5, 1), torch.full((5,), 4, dtype=torch.int32),
                                 torch.ones(5, dtype=torch.int64))  # SPL_OP_INC = 4
        assert (stt == 0).all(), stt
        dist.barrier()
        s_, v_, l_ = kv.get(ctr)
        assert int.from_bytes(bytes(v_[0, :8].numpy()), "little") == 5 * world
        # ---- meta: labels routed to owners, then C5 enumerate sees them globally
        lab = _keys([f"r{rank}_k{i}" for i in range(10)])
        ms, _ = kv.meta("set_label", lab, torch.full((10,), 0x8, dtype=torch.int64))
        assert (ms == 0).all()
        dist.barrier()
        rows, eps = kv.enumerate(0x8)
        got = sorted(decode_keys(rows))
        assert got == sorted(f"r{r}_k{i}" for r in range(world) for i in range(10)), got
        assert len(eps) == 10 * world
        rows, _ = kv.enumerate(0)
        assert len(rows) == 60 * world + 1
        # ---- C1 unset routed
        us = kv.unset(_keys([f"r{rank}_k59"]))
        assert (us == 0).all()
        dist.barrier()
        s_, _, _ = kv.get(_keys([f"r{r}_k59" for r in range(world)]))
        assert (s_ == -2).all()
        # ---- C3/C4 search: embeddings set through routed set_embeddings
        g = torch.Generator().manual_seed(7)
        allv = torch.randn(60 * world, 768, generator=g)
        myidx = [r * 60 + i for r in [rank] for i in range(50)]
        es = kv.set_embeddings(_keys([allk[i] for i in myidx]), allv[myidx])
        assert (es == 0).all()
        dist.barrier()
        qv = allv[[3, 60 * (world - 1) + 17]].clone()
        qv[1] *= 3.0
        own, sim, dd, krows = kv.search(qv if rank == 0 else None, k=5)
        names = [decode_keys(krows[j]) for j in range(2)]
        assert names[0][0] == "r0_k3" and names[1][0] == f"r{world - 1}_k17"
        assert abs(float(sim[0, 0]) - 1.0) < 1e-5
        # reference ranking over the union
        M = allv[[r * 60 + i for r in range(world) for i in range(50)]].double().numpy()
        names_all = [f"r{r}_k{i}" for r in range(world) for i in range(50)]
        for j in range(2):
            qq = qv[j].double().numpy()
            s = M @ qq / (np.linalg.norm(M, axis=1) * np.linalg.norm(qq))
            top = [names_all[i] for i in np.argsort(-s, kind="stable")[:5]]
            assert names[j] == top
            np.testing.assert_allclose(sim[j].numpy(), np.sort(s)[::-1][:5], rtol=1e-5, atol=1e-6)
        # ---- C2 signal counts: bind label 0x8 -> group 3 on every shard via C6, bump labelled keys
        if rank == 0:
            st.watch_label(0x8, 3)
            st.set_mop(0)
        mop, watches = kv.sync_config()
        assert mop == 0 and watches[3] == 3
        assert st.get_mop() == 0
        kv.meta("bump", _keys([f"r{rank}_k{i}" for i in range(4)]))
        dist.barrier()
        sc = kv.signal_counts()
        assert int(sc[3]) >= 4 * world
        q.put((rank, "ok"))
        st.close()
        unlink(name)
        dist.destroy_process_group()
    except Exception as e:  # report to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_collectives_gloo(world, uniq):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, uniq, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, msg = q.get(timeout=240)
            res[r] = msg
            if msg != "ok":
                break  # peers are blocked in a collective; fail fast
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res.get(r) == "ok", res.get(r)


def _xroute_worker(rank, world, port, base, q):
    """XRoute (parallel/xroute.py) on the host transport: one request / one response exchange,
    own-shard ops in place, full blocks -> EAGAIN, narrow response rows -> EMSGSIZE."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from libsplinter_amd import Store, unlink
        from libsplinter_amd.parallel.sharded import HostShard, shard_of
        from libsplinter_amd.parallel.xroute import XRoute
        name = f"{base}_q{rank}"
        st = Store.create(name, slots=2048, max_val=128, embeddings=False)
        sh = HostShard(st)
        n = 120
        mine = [f"q{rank}_k{i}" for i in range(n)]
        K = _keys(mine)
        V, L = _vals([f"value-{m}-padding".encode() for m in mine])
        xr = XRoute(sh, n, 0, 32, ks=32, resp_group=dist.new_group(backend="gloo"))
        assert xr.transport == "host"
        s, _, _, _ = xr.step(0, None, K, V, L, None)
        assert (s == 0).all(), s
        # own-shard ops never entered the exchange: they sit only in this rank's store
        own = shard_of(sh.hash_keys(K), world) == rank
        assert int(xr.scnt[0][rank, 0]) == int(own.sum())
        dist.barrier()
        allk = [f"q{r}_k{i}" for r in range(world) for i in range(n)]
        xg = XRoute(sh, 0, len(allk), 32, ks=32)
        _, sts, vs, ls = xg.step(1, None, None, None, None, _keys(allk))
        assert (sts == 0).all()
        for i, k in enumerate(allk):
            assert bytes(vs[i, : ls[i]].numpy()) == f"value-{k}-padding".encode()
        # response rows narrower than the values: EMSGSIZE, no bytes
        xn = XRoute(sh, 0, 10, 16, ks=32)
        _, s_, v_, l_ = xn.step(0, None, None, None, None, _keys(allk[:10]))
        assert (s_ == -90).all() and (l_ == 0).all(), (s_, l_)
        # tight capacity: the excess ops of a full block come back EAGAIN, the rest land
        ex = [f"x{rank}_{i}" for i in range(60)]
        KX = _keys(ex)
        VX, LX = _vals([b"x" * 8] * 60)
        tight = 60 // world - 3
        xt = XRoute(sh, 60, 0, 16, ks=32, cap_s=tight, cap_g=0)
        sx, _, _, _ = xt.step(0, None, KX, VX, LX, None)
        dest = shard_of(sh.hash_keys(KX), world)
        over = int((torch.bincount(dest, minlength=world) - tight).clamp(min=0).sum())
        assert int((sx == -11).sum()) == over and int((sx == 0).sum()) == 60 - over
        dist.barrier()
        q.put((rank, "ok"))
        st.close()
        unlink(name)
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_xroute_gloo(world, uniq):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_xroute_worker, args=(r, world, port, uniq, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, msg = q.get(timeout=240)
            res[r] = msg
            if msg != "ok":
                break
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res.get(r) == "ok", res.get(r)


def _a2a_worker(rank, world, port, q):
    """_Coll._all_to_all_uneven (the RCCL path's chunked uneven all-to-all) on gloo CPU tensors
    with a tiny chunk size: every part boundary case (empty segments, segments shorter / longer
    than a part) against one all_to_all_single."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import libsplinter_amd.parallel.sharded as S
        S.A2A_CHUNK_BYTES = 3 * 40 * world  # 3 rows of 40 B per destination per part
        rng = np.random.default_rng(rank)
        # send splits: row counts per destination; rank r sends (r + d) % 4 * 3 + d rows to d
        send = [((rank + d) % 4) * 3 + d for d in range(world)]
        allsend = [[((r + d) % 4) * 3 + d for d in range(world)] for r in range(world)]
        recv = [allsend[r][rank] for r in range(world)]
        inp = torch.from_numpy(rng.integers(0, 256, size=(sum(send), 40), dtype=np.uint8))
        ref = torch.empty((sum(recv), 40), dtype=torch.uint8)
        dist.all_to_all_single(ref, inp, recv, send)
        c = S._Coll(None)
        out = torch.full((sum(recv), 40), 7, dtype=torch.uint8)
        c._all_to_all_uneven(out, inp, recv, send)
        assert torch.equal(out, ref), "chunked uneven all-to-all differs"
        # an idle rank (rank 0 sends and receives no rows) must still take part in every part: the
        # part count is agreed from the shape, not from rows this rank happens to hold
        allsend = [[0 if (r == 0 or d == 0) else ((r + d) % 3) * 4 + 1 for d in range(world)] for r in range(world)]
        send = allsend[rank]
        recv = [allsend[r][rank] for r in range(world)]
        inp = torch.from_numpy(rng.integers(0, 256, size=(sum(send), 40), dtype=np.uint8))
        ref = torch.empty((sum(recv), 40), dtype=torch.uint8)
        dist.all_to_all_single(ref, inp, recv, send)
        out = torch.full((sum(recv), 40), 7, dtype=torch.uint8)
        c._all_to_all_uneven(out, inp, recv, send)
        assert torch.equal(out, ref), "chunked uneven all-to-all with an idle rank differs"
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_chunked_uneven_all_to_all_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_a2a_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, msg = q.get(timeout=120)
            res[r] = msg
            if msg != "ok":
                break
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res.get(r) == "ok", res.get(r)


def _routed_step_worker(rank, world, port, base, q, steps, n):
    """The routed step of bench.py at N > 1 (XRoute: pack -> count exchange -> owner runs ->
    response exchange -> gather), software-pipelined as there: step i's request is issued before
    step i-1's responses are gathered, and the two parities' blocks are both live.  Each step sets
    n new keys and gets n keys set by OTHER ranks two steps earlier; every get must return its
    key's value (integrity 0)."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from libsplinter_amd import Store, unlink
        from libsplinter_amd.parallel.sharded import HostShard
        from libsplinter_amd.parallel.xroute import XRoute
        name = f"{base}_w{rank}"
        st = Store.create(name, slots=8192, max_val=64, embeddings=False)
        xr = XRoute(HostShard(st), n, n, 32, ks=32, resp_group=dist.new_group(backend="gloo"))

        def val(k):
            return f"v:{k}".encode()

        pending, checked, bad = None, 0, 0
        for i in range(steps + 1):
            cur = None
            if i < steps:
                sk = [f"s{i}_r{rank}_{j}" for j in range(n)]
                K = _keys(sk)
                V, L = _vals([val(k) for k in sk])
                gk = None
                GK = None
                if i >= 2:  # keys another rank set two steps ago: already finished everywhere
                    src = (rank + 1 + i) % world
                    gk = [f"s{i - 2}_r{src}_{j}" for j in range(n)]
                    GK = _keys(gk)
                outs = (torch.empty(n, dtype=torch.int32), torch.zeros((n, 32), dtype=torch.uint8),
                        torch.empty(n, dtype=torch.int32), torch.empty(n, dtype=torch.int32))
                xr.request(i, K, V, L, GK)
                xr.execute(i, None, *outs)
                cur = (i, outs, gk)
            if pending is not None:  # the previous step's responses, after this step's requests
                pi, (ss, gv, gl, gs), pgk = pending
                xr.respond(pi)
                xr.finish(pi, ss, gv, gl, gs)
                bad += int((ss != 0).sum())
                if pgk is not None:
                    for j, k in enumerate(pgk):
                        ok = int(gs[j]) == 0 and bytes(gv[j, : gl[j]].numpy()) == val(k)
                        bad += 0 if ok else 1
                        checked += 1
            pending = cur
            dist.barrier()
        q.put((rank, f"ok {checked} {bad}"))
        st.close()
        unlink(name)
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def test_routed_step_world8_rehearsal(uniq):
    """World-8 CPU rehearsal of bench.py's routed step (one process per 'GPU', gloo over 127.0.0.1)."""
    world, steps, n = 8, 6, 150
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_routed_step_worker, args=(r, world, port, uniq, q, steps, n)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, msg = q.get(timeout=400)
            res[r] = msg
            if not msg.startswith("ok"):
                break
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res.get(r, "").startswith("ok"), res.get(r)
        _, checked, bad = res[r].split()
        assert int(checked) == (steps - 2) * n and int(bad) == 0, res[r]

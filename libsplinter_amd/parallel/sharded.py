"""Hash-sharded KV arena across the GPUs of a node (one process per GPU).

The reference is single-host shared memory (no collectives);
its closest scale-out idea is the disjoint key lanes of splinter_chi_sao
(/root/reference/splinter_chi_sao.c:400-418).  Here the key space is sharded:
shard(key) = (fnv1a(key) >> 40) % world, so a shard's in-arena probe (which
uses fnv1a % slots, the low bits) stays well spread.  Each rank owns one HBM
arena; a batch of client ops is routed to owners with RCCL all-to-all over
xGMI, executed by the owner's kernels, and the results are routed back.

Collectives, all over the default (RCCL) group:

  C1  routed set/get: parallel/xroute.py -- one request and one response
      exchange per batch, own-shard ops executed in place, the blocks moved by
      xGMI stores into peer-mapped windows (bench) or one all-to-all each (API).
      unset/integer_op/meta/set_embeddings: ONE all-to-all-v of packed request
      rows (key | args | value) and ONE of packed response rows per batch,
      after a count exchange.
  C2  node-wide signal-group counters: all-reduce(sum) of the 64 u64 counters.
  C3  search query broadcast from rank 0.
  C4  search top-k merge: all-gather of each shard's local top-k (sim, dist,
      key bytes), merged identically on every rank.
  C5  cross-shard enumerate/list: all-gather of counts, then of padded
      key rows + epochs.
  C6  config replication (mop + label->group map) broadcast from rank 0.

The local shard is pluggable (GpuShard = HBM arena kernels, HostShard = a
host store on CPU tensors), so every collective path is tested with gloo on
CPU (tests/test_sharded_gloo.py) and runs unchanged on RCCL.
"""
from __future__ import annotations

import itertools

import os

from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

SHARD_SHIFT = 40
KEY_BYTES = 64


def shard_of(hashes: torch.Tensor, world: int) -> torch.Tensor:
    """Owner rank for each 64-bit FNV-1a hash (int64 bit pattern)."""
    hi = (hashes >> SHARD_SHIFT) & 0xFFFFFF  # arithmetic shift of int64: mask the sign-extended bits
    return torch.remainder(hi, world)


def _u8(t: torch.Tensor) -> torch.Tensor:
    """Byte view [n, bytes] of a [n, ...] tensor (for packing rows)."""
    t = t.contiguous()
    row = int(np.prod(t.shape[1:])) * t.element_size() if t.dim() > 1 else t.element_size()
    return t.view(torch.uint8).reshape(t.shape[0], row)  # explicit width: batches may be empty


def _unpack(rows: torch.Tensor, spec: List[Tuple[torch.dtype, Tuple[int, ...]]]) -> List[torch.Tensor]:
    """Split packed uint8 rows back into typed columns (inverse of cat(_u8(...)))."""
    out, off = [], 0
    n = rows.shape[0]
    for dt, shape in spec:
        isz = torch.empty((), dtype=dt).element_size()
        nb = int(np.prod(shape)) * isz if shape else isz
        col = torch.empty((n, nb), dtype=torch.uint8, device=rows.device)  # fresh storage: aligned dtype view
        col.copy_(rows[:, off:off + nb])
        col = col.view(dt)
        out.append(col.reshape((n,) + tuple(shape)) if shape else col.reshape(n))
        off += nb
    return out


def decode_keys(rows: torch.Tensor) -> List[str]:
    return [bytes(r).split(b"\0", 1)[0].decode("utf-8", "replace") for r in rows.cpu().numpy()]


# bytes per RCCL all-to-all call (SPLINTER_A2A_CHUNK_BYTES); see _Coll.all_to_all
A2A_CHUNK_BYTES = int(os.environ.get("SPLINTER_A2A_CHUNK_BYTES", str(256 << 20)))


class _Coll:
    """Collective calls of one group.  RCCL takes device tensors directly; with the
    gloo backend (CPU tests, or several ranks sharing one GPU to rehearse the
    multi-GPU path) device tensors are staged through host copies."""

    def __init__(self, group):
        self.group = group
        self.stage = dist.get_backend(group) == "gloo"

    def _h(self, t):
        return t.cpu() if self.stage and t.is_cuda else t

    def all_to_all(self, out, inp, out_splits=None, in_splits=None):
        if self.stage and out.is_cuda:
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(o)
        elif out_splits is None and in_splits is None and out.is_cuda and \
                inp.numel() * inp.element_size() > A2A_CHUNK_BYTES:
            # Large equal-split all-to-alls go out in parts of <= A2A_CHUNK_BYTES per call: one
            # RCCL all_to_all_single of 1.5 GiB returned wrong bytes past 768 MiB on MI355X
            # (dev/debug/a2a_check.py, profiles/r1_routed_integrity.md).  Each part is one
            # contiguous byte range of every destination segment, sent as a grouped send/recv.
            w = dist.get_world_size(self.group)
            ib = inp.contiguous().view(torch.uint8).view(w, -1)
            ob = out.view(torch.uint8).view(w, -1)
            step = max(A2A_CHUNK_BYTES // w, 1)
            for p0 in range(0, ib.shape[1], step):
                p1 = min(ib.shape[1], p0 + step)
                dist.all_to_all([ob[d, p0:p1] for d in range(w)], [ib[d, p0:p1] for d in range(w)], group=self.group)
        elif out_splits is not None and out.is_cuda and inp.dim() >= 1:
            self._all_to_all_uneven(out, inp, list(out_splits), list(in_splits))
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def _all_to_all_uneven(self, out, inp, out_splits, in_splits):
        """Uneven all-to-all (the _route path) in parts of <= A2A_CHUNK_BYTES per call, like the
        equal-split case.  Whether to split must be decided identically on every rank (each call
        is a collective), so the largest segment of any rank is agreed with one small all-reduce;
        part p moves rows [p*step, (p+1)*step) of every segment."""
        w = dist.get_world_size(self.group)
        # row bytes from the shape (identical on every rank, also on one that sends and receives no
        # rows), and agreed in the same all-reduce as the segment maxima: every rank then computes the
        # same part count, so the collective sequences match
        row = int(np.prod(inp.shape[1:])) * inp.element_size()
        m = torch.tensor([max(in_splits + [0]), max(out_splits + [0]), row], dtype=torch.int64, device=out.device)
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
        mx = int(m[:2].max().item())
        row = max(int(m[2].item()), 1)
        if mx * row * w <= A2A_CHUNK_BYTES:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)
            return
        step = max(1, A2A_CHUNK_BYTES // (w * row))
        ioff = [0] + list(itertools.accumulate(in_splits))
        ooff = [0] + list(itertools.accumulate(out_splits))
        for p0 in range(0, mx, step):
            ins = [inp[ioff[d] + min(p0, in_splits[d]): ioff[d] + min(p0 + step, in_splits[d])] for d in range(w)]
            outs = [out[ooff[d] + min(p0, out_splits[d]): ooff[d] + min(p0 + step, out_splits[d])] for d in range(w)]
            # one all_to_all_single per part on packed copies (<= A2A_CHUNK_BYTES each)
            pout = torch.empty((sum(o.shape[0] for o in outs),) + tuple(out.shape[1:]), dtype=out.dtype,
                               device=out.device)
            dist.all_to_all_single(pout, torch.cat(ins), [o.shape[0] for o in outs], [i.shape[0] for i in ins],
                                   group=self.group)
            for o, part in zip(outs, pout.split([o.shape[0] for o in outs])):
                o.copy_(part)

    def all_reduce(self, t, op=dist.ReduceOp.SUM):
        h = self._h(t)
        dist.all_reduce(h, op=op, group=self.group)
        if h is not t:
            t.copy_(h)

    def broadcast(self, t, src):
        h = self._h(t)
        dist.broadcast(h, src, group=self.group)
        if h is not t:
            t.copy_(h)

    def all_gather(self, outs, t):
        if self.stage and t.is_cuda:
            ho = [torch.empty(o.shape, dtype=o.dtype) for o in outs]
            dist.all_gather(ho, t.cpu(), group=self.group)
            for o, h in zip(outs, ho):
                o.copy_(h)
        else:
            dist.all_gather(outs, t, group=self.group)


class ShardedKV:
    def __init__(self, local, group: Optional[dist.ProcessGroup] = None):
        self.local = local
        self.group = group
        self._kvstreams = None
        if dist.is_available() and dist.is_initialized():
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
            self._c = _Coll(group)
        else:
            self.world, self.rank = 1, 0
            self._c = None

    # ----------------------------------------------------------- routing --
    def _plan(self, keys: torch.Tensor):
        h = self.local.hash_keys(keys)
        dest = shard_of(h, self.world)
        order = torch.argsort(dest, stable=True)
        send = torch.bincount(dest, minlength=self.world)
        recv = torch.empty_like(send)
        self._c.all_to_all(recv, send)
        s, r = send.tolist(), recv.tolist()
        return order, s, r

    def _route(self, x: torch.Tensor, send_splits, recv_splits) -> torch.Tensor:
        out = torch.empty((sum(recv_splits),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        self._c.all_to_all(out, x.contiguous(), recv_splits, send_splits)
        return out

    def _roundtrip(self, keys: torch.Tensor, cols: List[torch.Tensor], execute, resp_spec):
        """C1 skeleton: pack (keys | cols) rows -> owners, execute, pack responses -> back.

        ``execute(keys, *cols) -> list of response tensors`` runs on the owner;
        responses are returned in the caller's original order.
        """
        order, s, r = self._plan(keys)
        req_spec = [(keys.dtype, tuple(keys.shape[1:]))] + [(c.dtype, tuple(c.shape[1:])) for c in cols]
        packed = torch.cat([_u8(keys[order])] + [_u8(c[order]) for c in cols], dim=1)
        got = _unpack(self._route(packed, s, r), req_spec)
        resp = execute(got[0], *got[1:])
        rspec = [(t.dtype, tuple(t.shape[1:])) for t in resp]
        back = _unpack(self._route(torch.cat([_u8(t) for t in resp], dim=1), r, s), rspec)
        outs = []
        for b in back:
            o = torch.empty_like(b)
            o[order] = b
            outs.append(o)
        return outs

    def owned_mask(self, keys: torch.Tensor) -> torch.Tensor:
        return shard_of(self.local.hash_keys(keys), self.world) == self.rank

    # -------------------------------------------------------- C1: ops ----
    def _exact_cap(self, keys: torch.Tensor) -> int:
        """Largest per-destination count of this batch over all ranks (one host sync):
        the API path never returns EAGAIN for a full request block."""
        dest = shard_of(self.local.hash_keys(keys), self.world)
        c = torch.bincount(dest, minlength=self.world).max().reshape(1).to(torch.int64)
        self._c.all_reduce(c, op=dist.ReduceOp.MAX)
        return max(1, int(c.item()))

    def _kvs(self):
        if self._kvstreams is None:
            from ..ops.arena import KvStreams
            self._kvstreams = KvStreams(1, 1)
        return self._kvstreams

    def _xroute(self, keys, n_set, n_get, vw, cap, set_kind):
        """A one-shot routed exchange (parallel/xroute.py) sized for this batch; the API path moves
        the blocks with the collectives (rccl / host transport), bench.py keeps a persistent peer one."""
        from .xroute import XRoute
        # the block geometry must be identical on every rank: caps, key and value widths are agreed
        # (a rank with an empty batch still takes part in the exchange)
        return XRoute(self.local, n_set, n_get, vw, ks=keys.shape[1], group=self.group,
                      transport="rccl" if self.local.device == "cuda" else "host",
                      cap_s=cap if set_kind else 0, cap_g=0 if set_kind else cap)

    def _agree_keys(self, keys: torch.Tensor) -> torch.Tensor:
        """Key records widened to the widest of any rank's batch (16-B multiple)."""
        m = torch.tensor([keys.shape[1]], dtype=torch.int64, device=keys.device)
        self._c.all_reduce(m, op=dist.ReduceOp.MAX)
        w = int(m.item())
        if w != keys.shape[1]:
            k2 = torch.zeros((keys.shape[0], w), dtype=torch.uint8, device=keys.device)
            k2[:, : keys.shape[1]] = keys
            keys = k2
        return keys.contiguous()

    def set(self, keys: torch.Tensor, vals: torch.Tensor, lens: torch.Tensor, vwidth: Optional[int] = None,
            **kw) -> torch.Tensor:
        """Routed set (C1): one request and one response exchange; only the used 16-B prefix of
        the value rows travels (``vwidth``, measured on this batch when not given)."""
        if self.world == 1:
            return self.local.set(keys, vals, lens, **kw)
        if vwidth is None:
            m = torch.tensor([int(lens.max().item()) if lens.numel() else 1], dtype=torch.int64, device=keys.device)
            self._c.all_reduce(m, op=dist.ReduceOp.MAX)
            vwidth = (int(m.item()) + 15) // 16 * 16
        vwidth = max(16, min(vwidth, (vals.shape[1] + 15) // 16 * 16))
        if vals.shape[1] % 16 or vals.shape[1] < vwidth:
            v2 = torch.zeros((vals.shape[0], max(vwidth, (vals.shape[1] + 15) // 16 * 16)), dtype=torch.uint8,
                             device=vals.device)
            v2[:, : vals.shape[1]] = vals
            vals = v2
        keys = self._agree_keys(keys)
        xr = self._xroute(keys, keys.shape[0], 0, vwidth, self._exact_cap(keys), True)
        try:
            st, _, _, _ = xr.step(0, self._kvs() if self.local.device == "cuda" else None, keys.contiguous(),
                                  vals.contiguous(), lens.to(torch.int32).contiguous(), None)
        finally:
            xr.close()
        return st

    def get(self, keys: torch.Tensor, width: Optional[int] = None,
            **kw) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Routed get (C1) -> (status, vals, lens).  Response rows carry ``width`` value bytes
        (default: the shard's max_val); a longer value returns EMSGSIZE (-90)."""
        if self.world == 1:
            return self.local.get(keys, **kw)
        width = width or (self.local.max_val + 15) // 16 * 16
        keys = self._agree_keys(keys)
        xr = self._xroute(keys, 0, keys.shape[0], width, self._exact_cap(keys), False)
        try:
            _, st, out, ln = xr.step(0, self._kvs() if self.local.device == "cuda" else None, None, None, None,
                                     keys.contiguous())
        finally:
            xr.close()
        return st, out, ln

    def unset(self, keys: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return self.local.unset(keys)
        return self._roundtrip(keys, [], lambda k: [self.local.unset(k).to(torch.int32)], None)[0]

    def integer_op(self, keys: torch.Tensor, ops: torch.Tensor, masks: Optional[torch.Tensor] = None):
        ops = ops.to(torch.int32)
        masks = torch.zeros(keys.shape[0], dtype=torch.int64, device=keys.device) if masks is None \
            else masks.to(torch.int64)
        if self.world == 1:
            return self.local.integer_op(keys, ops, masks)

        def ex(k, o, m):
            st, res = self.local.integer_op(k, o, m)
            return [st.to(torch.int32), res.to(torch.int64)]
        st, res = self._roundtrip(keys, [ops, masks], ex, None)
        return st, res

    def meta(self, op: str, keys: torch.Tensor, args: Optional[torch.Tensor] = None):
        args = torch.zeros(keys.shape[0], dtype=torch.int64, device=keys.device) if args is None \
            else args.to(torch.int64)
        if self.world == 1:
            return self.local.meta(op, keys, args)

        def ex(k, a):
            st, out = self.local.meta(op, k, a)
            return [st.to(torch.int32), out.to(torch.int64)]
        st, out = self._roundtrip(keys, [args], ex, None)
        return st, out

    def set_embeddings(self, keys: torch.Tensor, vecs: torch.Tensor) -> torch.Tensor:
        vecs = vecs.to(torch.float32)
        if self.world == 1:
            return self.local.set_embeddings(keys, vecs)
        return self._roundtrip(keys, [vecs], lambda k, v: [self.local.set_embeddings(k, v).to(torch.int32)],
                               None)[0]

    # -------------------------------------------------- C2: signals -------
    def signal_counts(self, local_counts: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Node-wide signal-group counters: sum of per-shard counters (64 x u64)."""
        t = (self.local.signal_counts() if local_counts is None else local_counts).clone()
        if self.world > 1:
            self._c.all_reduce(t)
        return t

    # ------------------------------------------- C3 + C4: vector search ----
    def search(self, queries: Optional[torch.Tensor], k: int = 10, min_sim: float = -2.0,
               max_dist: float = 3.4e38, label_mask: int = 0, nq: Optional[int] = None):
        """Global top-k over every shard.  Rank 0's queries are broadcast (C3);
        each shard scores its own slots, local top-k lists are all-gathered
        (C4) and merged (sim desc, dist asc) identically on every rank.

        Returns (owner_rank int64 [nq,k], sim, dist, key_rows uint8 [nq,k,64]);
        owner -1 marks an empty position."""
        dev = self.local.device
        if self.world > 1:
            n = torch.tensor([0 if queries is None else queries.shape[0]], dtype=torch.int64, device=dev)
            self._c.broadcast(n, 0)
            q = torch.empty((int(n.item()), 768), dtype=torch.float32, device=dev)
            if self.rank == 0:
                q.copy_(queries.reshape(-1, 768))
            self._c.broadcast(q, 0)
        else:
            q = queries.reshape(-1, 768).to(device=dev, dtype=torch.float32)
        sim, dst, krows = self.local.search(q, k, min_sim, max_dist, label_mask)
        valid = torch.isfinite(sim) & (sim > -3.0)
        sim = torch.where(valid, sim, torch.full_like(sim, -1e30))
        if self.world > 1:
            gs = [torch.empty_like(sim) for _ in range(self.world)]
            gd = [torch.empty_like(dst) for _ in range(self.world)]
            gk = [torch.empty_like(krows) for _ in range(self.world)]
            self._c.all_gather(gs, sim)
            self._c.all_gather(gd, dst)
            self._c.all_gather(gk, krows)
            sim, dst, krows = torch.cat(gs, 1), torch.cat(gd, 1), torch.cat(gk, 1)
        nqq, tot = sim.shape
        owner = torch.arange(tot, device=dev).div(k, rounding_mode="floor").expand(nqq, tot)
        # lexicographic (sim desc, dist asc): stable sort by dist, then stable sort by -sim
        o1 = torch.argsort(dst, dim=1, stable=True)
        s1 = torch.gather(sim, 1, o1)
        o2 = torch.argsort(-s1, dim=1, stable=True)
        order = torch.gather(o1, 1, o2)[:, :k]
        sim_k = torch.gather(sim, 1, order)
        dist_k = torch.gather(dst, 1, order)
        own_k = torch.gather(owner, 1, order)
        key_k = torch.gather(krows, 1, order.unsqueeze(-1).expand(-1, -1, KEY_BYTES))
        empty = sim_k < -1e29
        own_k = torch.where(empty, torch.full_like(own_k, -1), own_k)
        return own_k, sim_k, dist_k, key_k

    # ----------------------------------------------------- C5: enumerate ---
    def _all_gather_var(self, t: torch.Tensor) -> torch.Tensor:
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        counts = [torch.empty_like(n) for _ in range(self.world)]
        self._c.all_gather(counts, n)
        cs = [int(c.item()) for c in counts]
        mx = max(cs) if cs else 0
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        self._c.all_gather(parts, pad)
        return torch.cat([p[:c] for p, c in zip(parts, cs)])

    def enumerate(self, mask: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
        """Every key (on any shard) whose bloom contains ``mask`` (0 = all keys):
        (key rows uint8 [m, 64], epochs int64 [m]), identical on every rank."""
        rows, ep = self.local.enumerate(mask)
        if self.world == 1:
            return rows, ep
        packed = torch.cat([rows, _u8(ep.to(torch.int64))], dim=1)
        allp = self._all_gather_var(packed)
        krows, eps = _unpack(allp, [(torch.uint8, (KEY_BYTES,)), (torch.int64, ())])
        return krows, eps

    # --------------------------------------------------- C6: config -----
    def sync_config(self) -> Tuple[int, List[int]]:
        """Replicate rank 0's mop mode and label->group map to every shard."""
        cfg = self.local.get_config().to(self.local.device)  # uint8[65]: mop, bloom_watches[64]
        if self.world > 1:
            self._c.broadcast(cfg, 0)
            if self.rank != 0:
                self.local.apply_config(cfg)
        c = cfg.cpu().tolist()
        return c[0], c[1:]


class GpuShard:
    """Local shard = an HBM arena driven by the gfx950 kernels."""

    device = "cuda"

    def __init__(self, arena, search_grid: int = 512):
        self.arena = arena
        self._search = None
        self._grid = search_grid

    def hash_keys(self, keys: torch.Tensor) -> torch.Tensor:
        from .. import _native as N
        from ..ops.arena import _check, _keys, _stream
        keys = _keys(keys)
        out = torch.empty(keys.shape[0], dtype=torch.int64, device=keys.device)
        _check(N.hip_lib().spl_hash_keys(keys.data_ptr(), keys.shape[1], keys.shape[0], out.data_ptr(), _stream()),
               "hash_keys")
        return out

    def set(self, keys, vals, lens, **kw):
        return self.arena.set(keys, vals, lens, **kw)

    def get(self, keys, **kw):
        return self.arena.get(keys, **kw)

    def unset(self, keys):
        return self.arena.unset(keys)

    @property
    def max_val(self):
        return self.arena.max_val

    def integer_op(self, keys, ops, masks):
        return self.arena.integer_op(keys, ops, masks)

    def meta(self, op, keys, args):
        return self.arena.meta(op, keys, args)

    def set_embeddings(self, keys, vecs):
        return self.arena.set_embeddings(keys, vecs.contiguous())

    def key_rows(self, slots: torch.Tensor) -> torch.Tensor:
        from .. import _native as N
        from ..ops.arena import _stream
        sel = slots.to(torch.int32).contiguous()
        core = torch.empty((sel.numel(), 128), dtype=torch.uint8, device="cuda")
        if sel.numel():
            N.hip_lib().spl_arena_gather_slots(self.arena.desc, sel.data_ptr(), sel.numel(), core.data_ptr(),
                                               _stream())
        return core[:, KEY_BYTES:]

    def search(self, q, k, min_sim, max_dist, label_mask):
        if q.shape[0] >= 32 and self.capi_search:
            return self._search_capi(q, k, min_sim, max_dist, label_mask)
        from ..ops.search import VectorSearch
        if self._search is None:
            self._search = VectorSearch(self.arena, grid=self._grid)
        # many queries: the batched MFMA path (bf16 threshold passes + exact fp32 re-score,
        # same ranking); a handful: the exact fp32 kernel
        fn = self._search.search_batch if q.shape[0] >= 32 else self._search.search
        idx, sim, dst = fn(q, k, min_sim, max_dist, label_mask)
        valid = idx >= 0
        rows = self.key_rows(torch.where(valid, idx, torch.zeros_like(idx)).reshape(-1))
        rows = rows.reshape(idx.shape[0], idx.shape[1], KEY_BYTES) * valid.unsqueeze(-1).to(torch.uint8)
        sim = torch.where(valid, sim, torch.full_like(sim, -1e30))
        dst = torch.where(valid, dst, torch.full_like(dst, 3.4e38))
        return sim, dst, rows

    # many-query searches go through the product C ABI (spl_search_batch on this shard's store: device
    # query prep, MFMA candidate passes, fp32 re-score, keys fetched with the hits); False: the
    # Python driver of the same kernels (ops/search.py VectorSearch.search_batch)
    capi_search = os.environ.get("SPLINTER_SEARCH_CAPI", "1") != "0"

    def _search_capi(self, q, k, min_sim, max_dist, label_mask):
        hits = self.arena.store.search_batch(q.detach().float().cpu().numpy(), k, min_sim, max_dist, label_mask)
        valid = hits["emb"] != 0
        sim = np.where(valid, hits["sim"], np.float32(-1e30)).astype(np.float32)
        dst = np.where(valid, hits["dist"], np.float32(3.4e38)).astype(np.float32)
        rows = np.zeros((hits.shape[0], hits.shape[1], KEY_BYTES), dtype=np.uint8)
        rows[...] = np.frombuffer(hits["key"].tobytes(), dtype=np.uint8).reshape(hits.shape[0], hits.shape[1], 64)
        rows *= valid[..., None].astype(np.uint8)
        dev = q.device
        return (torch.from_numpy(sim).to(dev), torch.from_numpy(dst).to(dev), torch.from_numpy(rows).to(dev))

    def enumerate(self, mask):
        from ..ops.arena import SCAN_LABELS, SCAN_LIST
        idx, ep = self.arena.scan(SCAN_LABELS if mask else SCAN_LIST, mask)
        return self.key_rows(idx), ep

    def signal_counts(self):
        h = self.arena.header_view()[128:128 + 64 * 64]
        return h.view(torch.int64).view(64, 8)[:, 0].clone()

    def get_config(self):
        s = self.arena.store
        cfg = torch.empty(65, dtype=torch.uint8, device="cuda")
        cfg[0] = s.get_mop()
        cfg[1:] = self.arena.header_view()[56:120]
        return cfg

    def apply_config(self, cfg):
        _apply_config(self.arena.store, cfg)


def _apply_config(store, cfg: torch.Tensor) -> None:
    c = cfg.cpu().tolist()
    store.set_mop(int(c[0]))
    for bit, g in enumerate(c[1:]):
        if g != 0xFF:
            store.watch_label(1 << bit, int(g))


class HostShard:
    """Local shard = a host (shm) store; CPU tensors; used for gloo tests."""

    device = "cpu"

    def __init__(self, store):
        from .. import _native as N
        self.store = store
        self._L = N.core_lib()

    @staticmethod
    def _key(row) -> bytes:
        return bytes(row).split(b"\0", 1)[0]

    def hash_keys(self, keys: torch.Tensor) -> torch.Tensor:
        k = keys.cpu().numpy()
        hs = [self._L.spl_hash_key(self._key(row)) for row in k]
        return torch.tensor([h - (1 << 64) if h >= (1 << 63) else h for h in hs], dtype=torch.int64)

    def set(self, keys, vals, lens, **kw):
        k, v, ln = keys.numpy(), vals.numpy(), lens.numpy()
        st = []
        for i in range(k.shape[0]):
            rc = self._L.spl_set(self.store.handle, self._key(k[i]), bytes(v[i, : ln[i]]), int(ln[i]))
            st.append(0 if rc == 0 else -11)
        return torch.tensor(st, dtype=torch.int32)

    def get(self, keys, **kw):
        k = keys.numpy()
        width = (self.store.max_val + 15) // 16 * 16
        out = torch.zeros((k.shape[0], width), dtype=torch.uint8)
        lens = torch.zeros(k.shape[0], dtype=torch.int32)
        st = torch.zeros(k.shape[0], dtype=torch.int32)
        for i in range(k.shape[0]):
            v = self.store.get(self._key(k[i]))
            if v is None:
                st[i] = -2
            else:
                out[i, : len(v)] = torch.frombuffer(bytearray(v), dtype=torch.uint8)
                lens[i] = len(v)
        return st, out, lens

    def unset(self, keys):
        return torch.tensor([0 if self.store.unset(self._key(r)) >= 0 else -2 for r in keys.numpy()],
                            dtype=torch.int32)

    @property
    def max_val(self):
        return self.store.max_val

    def integer_op(self, keys, ops, masks):
        st, res = [], []
        for r, o, m in zip(keys.numpy(), ops.tolist(), masks.tolist()):
            try:
                res.append(self.store.integer_op(self._key(r), int(o), int(m) & 0xFFFFFFFFFFFFFFFF))
                st.append(0)
            except OSError:
                res.append(0)
                st.append(-22)
        res = [x - (1 << 64) if x >= (1 << 63) else x for x in res]
        return torch.tensor(st, dtype=torch.int32), torch.tensor(res, dtype=torch.int64)

    def meta(self, op, keys, args):
        fns = {"set_label": self.store.set_label, "unset_label": self.store.unset_label,
               "bump": lambda k, a: self.store.bump(k), "epoch": lambda k, a: self.store.epoch(k),
               "watch": self.store.watch, "unwatch": self.store.unwatch, "pulse": lambda k, a: self.store.pulse(k),
               "find": lambda k, a: self.store.find_slot(k)}
        st, out = [], []
        for r, a in zip(keys.numpy(), args.tolist()):
            v = fns[op](self._key(r), int(a))
            ok = v is not False and not (isinstance(v, int) and not isinstance(v, bool) and v < 0)
            st.append(0 if ok else -2)
            out.append(int(v) if isinstance(v, (int, bool)) else 0)
        return torch.tensor(st, dtype=torch.int32), torch.tensor(out, dtype=torch.int64)

    def set_embeddings(self, keys, vecs):
        st = []
        for r, v in zip(keys.numpy(), vecs.numpy()):
            try:
                self.store.set_embedding(self._key(r), v)
                st.append(0)
            except OSError:
                st.append(-2)
        return torch.tensor(st, dtype=torch.int32)

    def search(self, q, k, min_sim, max_dist, label_mask):
        names = [n for n, _ in self.store.enumerate(label_mask)] if label_mask else self.store.list()
        nq = q.shape[0]
        sim = torch.full((nq, k), -1e30)
        dst = torch.full((nq, k), 3.4e38)
        rows = torch.zeros((nq, k, KEY_BYTES), dtype=torch.uint8)
        vecs, keys = [], []
        for n in names:
            v = self.store.get_embedding(n)
            if v is not None and float(np.sqrt((v.astype(np.float64) ** 2).sum())) >= 1e-6:
                vecs.append(v)
                keys.append(n)
        if not vecs:
            return sim, dst, rows
        M = np.stack(vecs).astype(np.float64)
        mn = np.sqrt((M ** 2).sum(1))
        for j in range(nq):
            qq = q[j].numpy().astype(np.float64)
            s = M @ qq / (mn * np.sqrt((qq ** 2).sum()))
            d = np.sqrt(((M - qq) ** 2).sum(1))
            cand = [(-s[i], d[i], i) for i in range(len(keys)) if s[i] >= min_sim and d[i] <= max_dist]
            cand.sort()
            for t, (ns, dd, i) in enumerate(cand[:k]):
                sim[j, t], dst[j, t] = float(-ns), float(dd)
                kb = keys[i].encode()[:KEY_BYTES]
                rows[j, t, : len(kb)] = torch.tensor(list(kb), dtype=torch.uint8)
        return sim, dst, rows

    def enumerate(self, mask):
        items = self.store.enumerate(mask) if mask else [(n, self.store.epoch(n)) for n in self.store.list()]
        rows = torch.zeros((len(items), KEY_BYTES), dtype=torch.uint8)
        for i, (n, _) in enumerate(items):
            kb = n.encode()[:KEY_BYTES]
            rows[i, : len(kb)] = torch.tensor(list(kb), dtype=torch.uint8)
        return rows, torch.tensor([e for _, e in items], dtype=torch.int64)

    def signal_counts(self):
        return torch.tensor([self.store.signal_count(g) for g in range(64)], dtype=torch.int64)

    def get_config(self):
        reg = self.store.region()
        cfg = torch.empty(65, dtype=torch.uint8)
        cfg[0] = self.store.get_mop()
        cfg[1:] = torch.tensor(list(bytes(reg[56:120])), dtype=torch.uint8)
        return cfg

    def apply_config(self, cfg):
        _apply_config(self.store, cfg)

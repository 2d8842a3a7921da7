"""Host-sync-free C1 routing for batched set/get across the shards of a node.

SURVEY §2.10 C1: a batch of client ops is routed to the owning shards, run by
the owners' kernels and the results routed back.  The generic path in
``sharded.ShardedKV._roundtrip`` exchanges per-destination counts through the
host (``.tolist()``) before every all-to-all; this path removes every host
synchronisation so that a routed step can be queued ahead and its RCCL
transfers overlap compute that is queued on other streams (bench.py overlaps
them with the embed phase).

How: a batch is packed on the device into ``world x cap`` fixed-capacity
destination segments (``route_kernels.hip``), so every all-to-all has EQUAL
splits.  The owner learns the live rows of each segment from a device-side
count all-to-all, and its seqlock kernels skip the dead rows
(``spl_arena_set_seg`` / ``spl_arena_get_seg``).  Ops beyond a full segment
come back as EAGAIN, the reference's "retry" status (splinter.h:398-412).
``cap`` must be the same on every rank: ``route_capacity`` of a common batch
size leaves overflow at < 1e-15 per segment for hashed keys.

xGMI is point-to-point (7 links per MI355X), so one large all-to-all per
column drives every link at once; values travel as their used 16-B prefix
(``vwidth``), not the arena's full ``max_val`` row.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.distributed as dist

from .sharded import _Coll, shard_of


def route_capacity(n: int, world: int) -> int:
    """Rows per destination segment for a batch of ``n`` hashed keys: the mean
    n/world plus 8 standard deviations of the binomial spread (+64).  At
    n = 8M, world = 8 that is 0.8 % above the mean."""
    mean = n / world
    sd = math.sqrt(max(mean * (1.0 - 1.0 / world), 1.0))
    return max(1, int(math.ceil(mean + 8.0 * sd)) + 64)


def pack_ref(hashes, keys, vals, lens, vwidth, world, cap):
    """Torch reference of ``spl_route_pack`` (CPU shards, and the oracle of the
    kernel test).  Rows keep client order inside a destination segment."""
    n, dev = keys.shape[0], keys.device
    dest = shard_of(hashes, world)
    counts = torch.bincount(dest, minlength=world).to(torch.int32)
    order = torch.argsort(dest, stable=True)
    starts = torch.cumsum(counts.to(torch.int64), 0) - counts.to(torch.int64)
    slot = torch.empty(n, dtype=torch.int64, device=dev)
    slot[order] = torch.arange(n, device=dev) - starts[dest[order]]
    pos = torch.where(slot < cap, dest * cap + slot, torch.full_like(slot, -1))
    ok = pos >= 0
    kout = torch.zeros((world * cap, keys.shape[1]), dtype=torch.uint8, device=dev)
    kout[pos[ok]] = keys[ok]
    lout = vout = None
    if vals is not None:
        lout = torch.zeros(world * cap, dtype=torch.int32, device=dev)
        lout[pos[ok]] = lens[ok].to(torch.int32)
        vout = torch.zeros((world * cap, vwidth), dtype=torch.uint8, device=dev)
        vout[pos[ok]] = vals[ok, :vwidth]
    return counts, pos, kout, lout, vout


def gather_ref(pos, rstatus, rlens=None, rvals=None, width=None):
    """Torch reference of ``spl_route_gather``."""
    ok = pos >= 0
    p = pos.clamp(min=0)
    status = torch.where(ok, rstatus[p], torch.full_like(rstatus[p], -11))
    if rlens is None:
        return status, None, None
    lens = torch.where(ok, rlens[p], torch.zeros_like(rlens[p]))
    vals = rvals[p][:, :width] * ok.unsqueeze(1).to(torch.uint8)
    return status, vals, lens


class RoutedOp:
    """One routed batch in flight.  Every phase runs on the caller's CURRENT
    stream, so a pipeline can put the request all-to-all, the owner kernels
    and the response all-to-all on different streams; each tensor of the op
    is recorded on every stream that touches it (caching-allocator safety)."""

    def __init__(self, kind: str, n: int, cap: int, width: int):
        self.kind, self.n, self.cap, self.width = kind, n, cap, width
        self.t = {}

    def touch(self):
        vs = [v for v in self.t.values() if v is not None]
        if vs and vs[0].is_cuda:
            s = torch.cuda.current_stream()
            for v in vs:
                v.record_stream(s)


class RoutedKV:
    """Phases: ``begin_set`` / ``begin_get`` (pack + request all-to-all on
    ``group``), ``execute`` (owner kernels), ``respond`` (response all-to-all
    on ``resp_group``), ``finish`` (gather into client order).  Requests and
    responses use separate communicators, so step i's responses and step
    i+1's requests can be in flight at the same time."""

    def __init__(self, local, group=None, resp_group=None):
        self.local = local
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._c = _Coll(group)
        self._cr = _Coll(resp_group if resp_group is not None else group)

    def _native(self, t: torch.Tensor) -> bool:
        return t.is_cuda and hasattr(self.local, "route_pack")

    def _requests(self, op, keys, vals, lens, vwidth, cap):
        if self._native(keys):
            counts, pos, kout, lout, vout = self.local.route_pack(keys, vals, lens, vwidth, self.world, cap)
        else:
            counts, pos, kout, lout, vout = pack_ref(self.local.hash_keys(keys), keys, vals, lens, vwidth,
                                                     self.world, cap)
        rc = torch.empty_like(counts)
        self._c.all_to_all(rc, counts)
        kr = torch.empty_like(kout)
        self._c.all_to_all(kr, kout)
        op.t.update(pos=pos, counts=counts, kout=kout, rcounts=rc, krecv=kr)
        if vout is not None:
            lr, vr = torch.empty_like(lout), torch.empty_like(vout)
            self._c.all_to_all(lr, lout)
            self._c.all_to_all(vr, vout)
            op.t.update(lout=lout, vout=vout, lrecv=lr, vrecv=vr)
        op.touch()
        return op

    def begin_set(self, keys, vals, lens, cap: int, vwidth: Optional[int] = None) -> RoutedOp:
        vwidth = vals.shape[1] if vwidth is None else vwidth
        assert vwidth % 16 == 0 and 0 < vwidth <= vals.shape[1]
        return self._requests(RoutedOp("set", keys.shape[0], cap, vwidth), keys, vals, lens, vwidth, cap)

    def begin_get(self, keys, cap: int, width: int) -> RoutedOp:
        assert width % 16 == 0 and width > 0
        return self._requests(RoutedOp("get", keys.shape[0], cap, width), keys, None, None, 0, cap)

    def execute(self, op: RoutedOp, **kw) -> None:
        t = op.t
        if op.kind == "set":
            t["rstatus"] = self.local.set_seg(t["krecv"], t["vrecv"], t["lrecv"], t["rcounts"], op.cap, **kw)
        else:
            t["rstatus"], t["rvals"], t["rlens"] = self.local.get_seg(t["krecv"], t["rcounts"], op.cap, op.width,
                                                                      **kw)
        op.touch()

    def execute_fanout(self, sop: Optional[RoutedOp], gop: Optional[RoutedOp], kvs) -> None:
        """Owner kernels of a set and a get batch fanned out over ``kvs``'s writer / reader streams
        (ops/arena.py KvStreams.step_seg): the routed step runs the same client-stream configuration as
        a local step, each stream a slice of the received segments."""
        sargs = gargs = None
        if sop is not None:
            t = sop.t
            t["rstatus"] = torch.empty(t["krecv"].shape[0], dtype=torch.int32, device=t["krecv"].device)
            sargs = (t["krecv"], t["vrecv"], t["lrecv"], t["rcounts"], sop.cap, t["rstatus"])
        if gop is not None:
            t = gop.t
            n = t["krecv"].shape[0]
            dev = t["krecv"].device
            t["rvals"] = torch.empty((n, gop.width), dtype=torch.uint8, device=dev)
            t["rlens"] = torch.empty(n, dtype=torch.int32, device=dev)
            t["rstatus"] = torch.empty(n, dtype=torch.int32, device=dev)
            gargs = (t["krecv"], t["rcounts"], gop.cap, t["rvals"], t["rlens"], t["rstatus"])
        kvs.step_seg(self.local.arena, sargs, gargs)
        for op in (sop, gop):
            if op is not None:
                op.touch()

    def respond(self, op: RoutedOp) -> None:
        t = op.t
        b = torch.empty_like(t["rstatus"])
        self._cr.all_to_all(b, t["rstatus"])
        t["bstatus"] = b
        if op.kind == "get":
            bl, bv = torch.empty_like(t["rlens"]), torch.empty_like(t["rvals"])
            self._cr.all_to_all(bl, t["rlens"])
            self._cr.all_to_all(bv, t["rvals"])
            t["blens"], t["bvals"] = bl, bv
        op.touch()

    def finish(self, op: RoutedOp, out: Optional[torch.Tensor] = None, out_lens: Optional[torch.Tensor] = None,
               status: Optional[torch.Tensor] = None):
        """Client-order results: set -> status; get -> (status, vals [n, width], lens)."""
        t = op.t
        native = self._native(t["pos"])
        if op.kind == "set":
            if native:
                res = self.local.route_gather(t["pos"], t["bstatus"], status=status)[0]
            else:
                res = gather_ref(t["pos"], t["bstatus"])[0]
                if status is not None:
                    status.copy_(res)
                    res = status
        elif native:
            res = self.local.route_gather(t["pos"], t["bstatus"], t["blens"], t["bvals"], op.width, out=out,
                                          out_lens=out_lens, status=status)
        else:
            st, v, ln = gather_ref(t["pos"], t["bstatus"], t["blens"], t["bvals"], op.width)
            if out is not None:
                w = min(out.shape[1], op.width)
                out[:, :w] = v[:, :w]
                v = out
            res = (st, v, ln)
        op.touch()
        op.t = {}
        return res

    # --------------------------------------------------------- one-shot --
    def set(self, keys, vals, lens, cap: int, vwidth: Optional[int] = None, **kw):
        op = self.begin_set(keys, vals, lens, cap, vwidth)
        self.execute(op, **kw)
        self.respond(op)
        return self.finish(op)

    def get(self, keys, cap: int, width: int, **kw):
        op = self.begin_get(keys, cap, width)
        self.execute(op, **kw)
        self.respond(op)
        return self.finish(op)

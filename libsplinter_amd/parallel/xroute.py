"""Routed KV step across the shards of a node: one request and one response exchange per step.

SURVEY §2.10 C1 / §2.13.  Every rank owns the hash-shard ``((fnv1a >> 40) & 0xFFFFFF) % world``
of the key space (parallel/sharded.py ``shard_of``); a client batch of sets and gets is executed
by the owners' seqlock kernels and the results come back in client order.  The reference has no
multi-device path at all -- its only scale-out is disjoint key lanes on one mapping
(/root/reference/splinter_chi_sao.c:400-418); per-op semantics are those of
/root/reference/splinter.c:365-464.

Per step, per direction, ONE exchange:

* Every (requester r, owner o) pair has one request block in o's window -- [set keys | set lens |
  set value prefixes | get keys], ``cap`` rows per kind -- and one response block in r's window
  -- [set status | get status | get lens | get values] (``XGeom``).
* ``request``: the pack kernel (route_kernels.hip ``spl_xr_pack``) writes every remote op's record
  straight into its owner's request block.  Ops this rank owns never enter the exchange: the pack
  only lists their client indices.  The per-(kind, destination) row counts are the only thing a
  collective carries (one all-to-all of 2 x world int32); it is also the step's ordering point:
  an owner starts after every requester's pack of the step has completed.
* ``execute``: the owner kernels (arena_kernels.hip ``spl_kvs_step_xr``) run the own ops in place
  on the client arrays and every peer's request block, fanned out over the same 32 + 32 client
  streams as a local step, and write each peer's results into that peer's response block.
* ``respond`` / ``finish``: one collective marks the responses complete, then the gather kernel
  (``spl_xr_gather``) copies the remote ops' results into client order.

Transports for the bytes (the collectives above are the same for both):

* ``peer`` (default on GPUs): every rank's window is device memory exported as dmabuf VMM chunks
  (``spl_xw_create``) and mapped by every other rank (``spl_xw_attach``; on another GPU an xGMI
  peer mapping, ``hipDeviceEnablePeerAccess``).  The pack kernel stores request rows and the owner
  kernels store response rows directly into the destination rank's HBM over xGMI: no collective
  and no copy kernel moves them, every link of the point-to-point fabric carries its own pair's
  traffic, and nothing of the exchange competes with the encoder except those stores.  Set-up
  validates every mapping with a marker round trip and falls back to ``rccl`` if any fails.
* ``rccl``: the pack writes into local send staging blocks and ONE equal-split all-to-all per
  direction moves them (chunked at A2A_CHUNK_BYTES, parallel/sharded.py ``_Coll``).
* ``host``: the same protocol on CPU tensors with torch reference kernels (HostShard, gloo), so
  the exchange logic runs in the CPU test suite at world 8.

Step ordering (``sync``): ``coll`` -- the count all-to-all and the response all-to-all above (RCCL
takes device tensors, so on GPUs of their own the ranks never wait on the host); ``flags`` (peer
transport, SPLINTER_XR_SYNC=flags) -- no collective per step: each rank posts its counts and a
step sequence into its peers' windows from the device (route_kernels.hip ``spl_xr_post``) and
waits for theirs with a one-workgroup bounded wait kernel (``spl_xr_wait``) in stream order, so
no host sync is left in the step even where the collectives are gloo's (ranks sharing a GPU).
Measured on that one-GPU rehearsal it is slower than the gloo-staged collectives (0.62-0.63 vs
0.68 of the 1-rank step, profiles/r5/exchange_sync.md), so ``coll`` is the default.

At world 1 every op is its own shard's: the step is the in-place execution alone.

Fixed capacity per block (``route_capacity``: mean + 8 sigma + 64): an op whose block is full
returns EAGAIN, the reference's retry status (splinter.h:398-412).

Buffer reuse is double-buffered by step parity; ``request(i)`` waits (stream-wise) for
``finish(i - 2)``, which in turn follows every rank's ``execute(i - 2)`` through the response
collective, so no block is overwritten while anyone still reads it.
"""
from __future__ import annotations

import ctypes
import math
import os
import time
import secrets
from typing import Optional

import torch
import torch.distributed as dist

from .sharded import _Coll, shard_of

ALIGN = 256
FLAG_BYTES = 2 * 2 * 64 * 8 + 2 * 64 * 2 * 4  # == spl_xr_flag_bytes()
OWN, FULL = -2, -1
EAGAIN, EMSGSIZE = -11, -90


def route_capacity(n: int, world: int) -> int:
    """Rows per request block for a batch of ``n`` hashed keys: the mean n/world plus 8 standard
    deviations of the binomial spread (+64).  At n = 8M, world = 8: 0.8 % above the mean."""
    if n <= 0:
        return 0
    mean = n / world
    sd = math.sqrt(max(mean * (1.0 - 1.0 / world), 1.0))
    return max(1, int(math.ceil(mean + 8.0 * sd)) + 64)


def _al(x: int) -> int:
    return (x + ALIGN - 1) // ALIGN * ALIGN


class XGeom:
    """Byte layout of the exchange blocks and windows.

    window (per rank) = 2 parities x [REQ block from source 0..W-1 | RESP block from owner 0..W-1]
      REQ  = set keys cap_s x ks | set lens cap_s x 4 | set values cap_s x vw | get keys cap_g x ks
      RESP = set status cap_s x 4 | get status cap_g x 4 | get lens cap_g x 4 | get values cap_g x vw
    direct responses (peer transport): REQ also carries the ops' client indices (set cap_s x 4 | get
    cap_g x 4) and the RESP blocks are replaced by this rank's client output arrays, which the owners
    write in client order:
      OUT  = set status n_set x 4 | get status n_get x 4 | get lens n_get x 4 | get values n_get x vw
    """

    def __init__(self, world: int, cap_s: int, cap_g: int, ks: int, vw: int, n_set: int = 0, n_get: int = 0,
                 direct: bool = False):
        self.world, self.cap_s, self.cap_g, self.ks, self.vw = world, cap_s, cap_g, ks, vw
        self.direct = direct
        self.off_sk = 0
        self.off_sl = _al(cap_s * ks)
        self.off_sv = self.off_sl + _al(cap_s * 4)
        self.off_gk = self.off_sv + _al(cap_s * vw)
        self.req_b = self.off_gk + _al(cap_g * ks)
        self.off_sp = self.off_gp = -1
        if direct:
            self.off_sp = self.req_b
            self.off_gp = self.off_sp + _al(cap_s * 4)
            self.req_b = self.off_gp + _al(cap_g * 4)
            rs, rg = n_set, n_get  # the OUT area: client order
        else:
            rs, rg = cap_s, cap_g  # a response block per owner
        self.off_ss = 0
        self.off_gs = _al(rs * 4)
        self.off_gl = self.off_gs + _al(rg * 4)
        self.off_gv = self.off_gl + _al(rg * 4)
        self.resp_b = self.off_gv + _al(rg * vw)
        self.par_b = world * self.req_b + (self.resp_b if direct else world * self.resp_b)
        # device-side ordering (sync "flags"): [parity][dir][source] u64 step sequences, then
        # [parity][source][kind] i32 row counts, 64 sources (route_kernels.hip kMaxWorld)
        self.off_flag = 2 * self.par_b
        self.flag_b = FLAG_BYTES
        self.off_fcnt = self.off_flag + 2 * 2 * 64 * 8
        self.window_b = self.off_flag + _al(self.flag_b)

    def req(self, p: int, s: int) -> int:
        """Offset of the request block from source s, parity p."""
        return p * self.par_b + s * self.req_b

    def resp(self, p: int, o: int) -> int:
        """Offset of the response block from owner o, parity p (the OUT area when direct)."""
        return p * self.par_b + self.world * self.req_b + (0 if self.direct else o * self.resp_b)

    def wire_bytes(self, n_set_remote: float, n_get_remote: float) -> float:
        """Bytes a rank stores into its peers per step: request rows + response rows."""
        extra = 4 if self.direct else 0
        return (n_set_remote * (self.ks + 4 + self.vw + 4 + extra)
                + n_get_remote * (self.ks + 4 + 4 + self.vw + extra))


def _view(t: torch.Tensor, off: int, rows: int, width: int, dtype=torch.uint8) -> torch.Tensor:
    """[rows, width] (or [rows] for width 0) typed view of a flat uint8 window at byte offset off."""
    isz = torch.empty((), dtype=dtype).element_size()
    n = rows * max(width, 1) * isz
    v = t[off: off + n].view(dtype)
    return v.view(rows, width) if width else v


class XRoute:
    """A routed step pipeline of fixed batch geometry (n_set sets + n_get gets per step per rank).

    Phases run on the caller's CURRENT stream (so a pipeline can put them on different streams):
    ``request(i, ...)`` -> ``execute(i, kvs)`` -> ``respond(i)`` -> ``finish(i)``.  The client arrays
    passed to ``request`` (keys, values, lens) and ``execute`` (status / output arrays) must stay
    alive until ``finish(i)`` has run on the device."""

    def __init__(self, local, n_set: int, n_get: int, vw: int, ks: int = 16, group=None, resp_group=None,
                 transport: Optional[str] = None, cap_s: Optional[int] = None, cap_g: Optional[int] = None):
        self.local = local
        if dist.is_available() and dist.is_initialized():
            self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        else:
            self.world, self.rank = 1, 0
        W = self.world
        self.group = group
        self._c = _Coll(group) if W > 1 else None
        self._cr = _Coll(resp_group if resp_group is not None else group) if W > 1 else None
        self.n_set, self.n_get, self.ks, self.vw = n_set, n_get, ks, vw
        assert ks % 16 == 0 and 0 < ks <= 64 and vw % 16 == 0 and vw > 0
        if W == 1:
            cap_s, cap_g = n_set, n_get
        self.cap_s = route_capacity(n_set, W) if cap_s is None else cap_s
        self.cap_g = route_capacity(n_get, W) if cap_g is None else cap_g
        self.g = XGeom(W, self.cap_s, self.cap_g, ks, vw)
        self.cuda = getattr(local, "device", "cpu") == "cuda"
        dev = "cuda" if self.cuda else "cpu"
        self.dev = dev
        self._win = self._send = None
        self._xw = []
        self._ev_done = [None, None]
        self._batch = [None, None]
        if transport is None:
            transport = os.environ.get("SPLINTER_XR_TRANSPORT", "peer") if self.cuda else "host"
        if W == 1:
            transport = "local"
        self.transport = transport
        # direct responses (peer transport, fused owner grid): owners write results straight into the
        # requester's client output arrays (outputs(p)) -- no response blocks, no gather kernel
        # (profiles/r6/README.md: the gather was 0.38 of the 2-rank step's 2.79 ms)
        self.direct = (transport == "peer" and self.cuda and W > 1
                       and os.environ.get("SPLINTER_XR_DIRECT", "1") != "0"
                       and os.environ.get("SPL_KVS_FUSED", "2") != "0")
        if self.direct:
            self.g = XGeom(W, self.cap_s, self.cap_g, ks, vw, n_set, n_get, direct=True)
        self.fallback_reason = None  # why a requested peer transport fell back to rccl (None: it did not)
        self.sync = "coll"
        self.wait_ms = int(os.environ.get("SPLINTER_XR_WAIT_MS", "20000"))
        i32 = dict(dtype=torch.int32, device=dev)
        # per parity: pack counts [kind][dest], sent counts [dest][kind], received [src][kind]
        self.cnt = [torch.zeros((2, W), **i32) for _ in range(2)]
        self.scnt = [torch.zeros((W, 2), **i32) for _ in range(2)]
        self.rcnt = [torch.zeros((W, 2), **i32) for _ in range(2)]
        self.pos = [[torch.empty(max(n_set, 1), **i32), torch.empty(max(n_get, 1), **i32)] for _ in range(2)]
        self.lidx = [[torch.empty(max(self.cap_s, 1), **i32), torch.empty(max(self.cap_g, 1), **i32)]
                     for _ in range(2)]
        self._token = torch.zeros(W, **i32)
        self._token_r = torch.zeros(W, **i32)
        # SPLINTER_XR_PHASES=1 (attribution runs, device path): timing events around every phase of
        # every step on the stream it runs on, and the host time spent inside the collectives
        self._ph = [] if (self.cuda and os.environ.get("SPLINTER_XR_PHASES") == "1") else None
        self._ph_host = {"counts": 0.0, "respond": 0.0}
        if W > 1:
            if transport == "peer":
                if not self._setup_peer():
                    transport = self.transport = "rccl"
                    self.direct = False
                    self.g = XGeom(W, self.cap_s, self.cap_g, ks, vw)
                else:
                    # measured on the one-GPU rehearsal: flags 0.62-0.63 of the 1-rank step vs 0.68 with the
                    # (gloo-staged) collectives (profiles/r5/exchange_sync.md), so collectives by default
                    self.sync = "flags" if os.environ.get("SPLINTER_XR_SYNC", "") == "flags" else "coll"
            if transport in ("rccl", "host"):
                self._win = torch.zeros(self.g.window_b, dtype=torch.uint8, device=dev)
                self._send = torch.zeros(self.g.window_b, dtype=torch.uint8, device=dev)
                self._win_base = self._win.data_ptr()
                self._send_base = self._send.data_ptr()
        self._tables()

    # ------------------------------------------------------------------ set-up --
    def _setup_peer(self) -> bool:
        """Create this rank's window, attach every peer's, validate with a marker round trip.
        False (on every rank alike) if any rank could not: the caller falls back to rccl."""
        from .. import _native as N
        L = N.hip_lib()
        W, r = self.world, self.rank
        dev = torch.cuda.current_device()
        tok = [secrets.token_hex(6) if r == 0 else None]
        dist.broadcast_object_list(tok, src=0, group=self.group)
        names = [f"splxw-{tok[0]}-{q}" for q in range(W)]
        devs = [None] * W
        dist.all_gather_object(devs, dev, group=self.group)
        ok = True
        assert L.spl_xr_flag_bytes() == FLAG_BYTES
        own = L.spl_xw_create(dev, self.g.window_b, names[r].encode())
        why = None
        if not own:
            ok = False
            why = f"rank {r}: spl_xw_create of a {self.g.window_b}-B window failed"
        else:
            self._xw.append(own)
            from ..ops.arena import _device_view
            _device_view(L.spl_xw_base(own) + self.g.off_flag, self.g.flag_b).zero_()  # no step posted yet
            torch.cuda.synchronize()
        dist.barrier(group=self.group)  # every window is being served
        self._peer_base = [0] * W
        if ok:
            self._peer_base[r] = L.spl_xw_base(own)
            for q in range(W):
                if q == r:
                    continue
                if L.spl_xw_peer(dev, int(devs[q])) != 0:
                    ok = False
                    why = f"rank {r}: peer access device {dev} -> {devs[q]} refused"
                    break
                h = L.spl_xw_attach(names[q].encode(), dev)
                if not h:
                    ok = False
                    why = f"rank {r}: attaching rank {q}'s window failed"
                    break
                self._xw.append(h)
                self._peer_base[q] = L.spl_xw_base(h)
        mapped = self._agree(ok)
        ok = mapped
        if ok:
            ok = self._agree(self._validate())
            if not ok:
                why = "marker round trip through the peer windows did not validate"
        if not mapped and why is None:
            why = "another rank could not map the windows"
        if not ok:
            self.fallback_reason = why
        dist.barrier(group=self.group)  # every peer is done with the windows before any is torn down
        if not ok:
            for h in reversed(self._xw):
                L.spl_xw_destroy(h)
            self._xw = []
            return False
        self._win_base = self._peer_base[r]
        return True

    def _agree(self, ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device="cuda")
        self._c.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def _validate(self) -> bool:
        """Each rank stores a marker into its block of every peer's window (a device kernel over
        the mapped peer memory, as the pack kernel will), then checks the markers it received."""
        from ..ops.arena import _device_view
        W, r, g = self.world, self.rank, self.g
        for q in range(W):
            if q != r:
                m = torch.tensor([0x5850524F, r, q, W] * 4, dtype=torch.int32, device="cuda").view(torch.uint8)
                _device_view(self._peer_base[q] + g.req(0, r), 64).copy_(m)
        torch.cuda.synchronize()
        dist.barrier(group=self.group)
        ok = True
        for s in range(W):
            if s != r:
                got = _device_view(self._peer_base[r] + g.req(0, s), 64).view(torch.int32).cpu().tolist()
                ok = ok and got == [0x5850524F, s, r, W] * 4
        for s in range(W):
            _device_view(self._peer_base[r] + g.req(0, s), 64).zero_()
        torch.cuda.synchronize()
        return ok

    def _tables(self):
        """Block pointer tables: pack destinations and gather sources (device), and the exec
        request / response blocks (host, in the spl_xr_step_t struct)."""
        W, r, g = self.world, self.rank, self.g
        self._pack_blk = [None, None]
        self._gath_blk = [None, None]
        self._exec_req = [[0] * W, [0] * W]
        self._exec_resp = [[0] * W, [0] * W]
        if W == 1:
            return
        for p in range(2):
            if self.transport == "peer":
                pk = [self._peer_base[d] + g.req(p, r) for d in range(W)]
                resp = [self._peer_base[s] + g.resp(p, r) for s in range(W)]
            else:
                pk = [self._send_base + g.req(p, d) for d in range(W)]
                resp = [self._send_base + g.resp(p, s) for s in range(W)]
            self._exec_req[p] = [self._win_base + g.req(p, s) for s in range(W)]
            self._exec_resp[p] = resp
            gt = [self._win_base + g.resp(p, o) for o in range(W)]
            if self.cuda:
                self._pack_blk[p] = torch.tensor(pk, dtype=torch.int64, device="cuda")
                self._gath_blk[p] = torch.tensor(gt, dtype=torch.int64, device="cuda")
        if self.transport == "peer":
            self._flag_blk = torch.tensor([self._peer_base[d] + g.off_flag for d in range(W)], dtype=torch.int64,
                                          device="cuda")
            self._own_flag = self._win_base + g.off_flag
            self._xerr = torch.zeros(1, dtype=torch.int32, device="cuda")

    def _post(self, i: int, direction: int, counts=None) -> None:
        from .. import _native as N
        from ..ops.arena import _check, _stream
        _check(N.hip_lib().spl_xr_post(self._flag_blk.data_ptr(), self.world, self.rank, i & 1, direction, i + 1,
                                       counts.data_ptr() if counts is not None else None, _stream()), "xr_post")

    def _wait(self, i: int, direction: int) -> None:
        from .. import _native as N
        from ..ops.arena import _check, _stream
        _check(N.hip_lib().spl_xr_wait(self._own_flag, self.world, self.rank, i & 1, direction, i + 1, self.wait_ms,
                                       self._xerr.data_ptr(), _stream()), "xr_wait")

    def sync_error(self) -> bool:
        """True if a device-side wait (sync "flags") gave up on a peer's post (waits for the device)."""
        return self.sync == "flags" and bool(self._xerr.item())

    def close(self):
        if self._xw:
            from .. import _native as N
            torch.cuda.synchronize()
            if self.world > 1:
                dist.barrier(group=self.group)  # nobody stores into a window that is going away
            for h in reversed(self._xw):
                N.hip_lib().spl_xw_destroy(h)
            self._xw = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ----------------------------------------------------------------- phases --
    def outputs(self, p: int):
        """Direct responses: this rank's client output arrays of parity p -- (set status [n_set] int32,
        get values [n_get, vw] uint8, get lens [n_get] int32, get status [n_get] int32) -- in its own
        window, where the owners write the results.  Pass them to execute / finish for every step of
        that parity (i & 1 == p), and read a step's results before the next request of its parity."""
        assert self.direct, "outputs(): direct responses only (peer transport)"
        from ..ops.arena import _device_view
        g, base = self.g, self._win_base + self.g.resp(p, self.rank)
        u8 = lambda off, nb: _device_view(base + off, nb)  # noqa: E731
        ss = u8(g.off_ss, self.n_set * 4).view(torch.int32)
        gs = u8(g.off_gs, self.n_get * 4).view(torch.int32)
        gl = u8(g.off_gl, self.n_get * 4).view(torch.int32)
        gv = u8(g.off_gv, self.n_get * self.vw).view(self.n_get, self.vw)
        return ss, gv, gl, gs

    # ------------------------------------------------------- phase attribution --
    def _mark(self, i: int, name: str) -> None:
        if self._ph is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.current_stream())
            self._ph.append((i, name, ev))

    def phase_reset(self) -> None:
        if self._ph is not None:
            self._ph.clear()
            self._ph_host = {k: 0.0 for k in self._ph_host}

    def phase_summary(self) -> Optional[dict]:
        """Per step, ms between the phase marks on the device (each phase on its own stream; a phase's
        span includes its waits on the others), and host ms inside the collectives -- averaged over the
        steps marked since phase_reset()."""
        if not self._ph:
            return None
        torch.cuda.synchronize()
        by = {}
        for i, name, ev in self._ph:
            by.setdefault(i, {})[name] = ev
        spans = {"pack": ("pack0", "pack1"), "count_exchange": ("pack1", "req1"), "wait_for_request": ("req1", "exec0"),
                 "owner_grid": ("exec0", "exec1"), "respond": ("resp0", "resp1"), "gather": ("resp1", "gath1"),
                 "step": ("pack0", "gath1")}
        acc = {k: [] for k in spans}
        for m in by.values():
            for k, (a, b) in spans.items():
                if a in m and b in m:
                    acc[k].append(m[a].elapsed_time(m[b]))
        n = max(len(by), 1)
        out = {k: (sum(v) / len(v) if v else None) for k, v in acc.items()}
        out.update({f"host_{k}_ms": v * 1e3 / n for k, v in self._ph_host.items()})
        out["steps"] = len(by)
        return out

    def request(self, i: int, skeys=None, svals=None, slens=None, gkeys=None) -> None:
        """Pack step i's batch into the owners' request blocks and exchange the counts."""
        p = i & 1
        if self._ev_done[p] is not None:
            torch.cuda.current_stream().wait_event(self._ev_done[p])
        self._batch[p] = (skeys, svals, slens, gkeys)
        if self.world == 1:
            return
        self._mark(i, "pack0")
        if self.cuda:
            self._pack_dev(p, skeys, svals, slens, gkeys)
        else:
            self._pack_host(p, skeys, svals, slens, gkeys)
        self._mark(i, "pack1")
        self.scnt[p].copy_(self.cnt[p].t())
        t0 = time.perf_counter()
        if self.sync == "flags":
            self._post(i, 0, self.cnt[p])
        else:
            self._c.all_to_all(self.rcnt[p], self.scnt[p])
        self._ph_host["counts"] += time.perf_counter() - t0
        if self.transport != "peer":
            n = self.world * self.g.req_b
            o = self.g.req(p, 0)
            self._c.all_to_all(self._win[o: o + n].view(self.world, -1), self._send[o: o + n].view(self.world, -1))
        self._mark(i, "req1")

    def execute(self, i: int, kvs=None, sstatus=None, gout=None, glens=None, gstatus=None, retries: int = 64) -> None:
        """Owner kernels of step i: own ops in place into the given client arrays, every peer's
        request block into that peer's response block.  The current stream is the fan-out's origin."""
        p = i & 1
        skeys, svals, slens, gkeys = self._batch[p]
        self._out = (sstatus, gout, glens, gstatus)
        if self.world > 1 and self.sync == "flags":
            self._wait(i, 0)  # every peer's request block and counts of step i are in this window
        self._mark(i, "exec0")
        if self.cuda:
            self._exec_dev(p, kvs, skeys, svals, slens, gkeys, sstatus, gout, glens, gstatus, retries)
        else:
            self._exec_host(p, skeys, svals, slens, gkeys, sstatus, gout, glens, gstatus)
        self._mark(i, "exec1")

    def respond(self, i: int) -> None:
        """Mark step i's responses complete on every rank (rccl / host: move them)."""
        if self.world == 1:
            return
        p = i & 1
        self._mark(i, "resp0")
        t0 = time.perf_counter()
        if self.sync == "flags":
            self._post(i, 1)
        elif self.transport == "peer":
            self._cr.all_to_all(self._token_r, self._token)
        else:
            n = self.world * self.g.resp_b
            o = self.g.resp(p, 0)
            self._cr.all_to_all(self._win[o: o + n].view(self.world, -1), self._send[o: o + n].view(self.world, -1))
        self._ph_host["respond"] += time.perf_counter() - t0
        self._mark(i, "resp1")

    def finish(self, i: int, sstatus=None, gout=None, glens=None, gstatus=None) -> None:
        """Remote ops' results into client order (the own ops' are already there)."""
        p = i & 1
        skeys, svals, slens, gkeys = self._batch[p]
        if self.world > 1:
            if self.sync == "flags":
                self._wait(i, 1)  # every owner's response rows of step i are in this window
            if self.direct:
                pass  # the owners wrote every result in place; block-full ops were marked by the pack
            elif self.cuda:
                self._gather_dev(p, skeys, gkeys, sstatus, gout, glens, gstatus)
            else:
                self._gather_host(p, skeys, gkeys, sstatus, gout, glens, gstatus)
            self._mark(i, "gath1")
        if self.cuda:
            self._ev_done[p] = torch.cuda.current_stream().record_event()
        self._batch[p] = None

    # ------------------------------------------------------------ device path --
    def _pack_dev(self, p, skeys, svals, slens, gkeys):
        from .. import _native as N
        from ..ops.arena import _check, _stream
        L, W, r, g = N.hip_lib(), self.world, self.rank, self.g
        s = _stream()
        ns = skeys.shape[0] if skeys is not None else 0
        ng = gkeys.shape[0] if gkeys is not None else 0
        assert ns <= self.n_set and ng <= self.n_get
        tab = self._pack_blk[p].data_ptr()
        cnt = self.cnt[p]
        # direct responses: the client-index columns, and block-full ops marked EAGAIN in this rank's
        # output arrays right here (no gather follows)
        out = self.outputs(p) if self.direct else None
        if ns:
            assert skeys.shape[1] == self.ks and svals.shape[1] >= self.vw and svals.is_contiguous()
            _check(L.spl_xr_pack(skeys.data_ptr(), self.ks, svals.data_ptr(), svals.shape[1], slens.data_ptr(), ns, W, r,
                                 self.cap_s, tab, g.off_sk, g.off_sl, g.off_sv, self.vw, cnt[0].data_ptr(),
                                 self.lidx[p][0].data_ptr(), self.pos[p][0].data_ptr(), g.off_sp,
                                 out[0].data_ptr() if out else None, None, s), "xr_pack set")
        else:
            cnt[0].zero_()
        if ng:
            assert gkeys.shape[1] == self.ks
            _check(L.spl_xr_pack(gkeys.data_ptr(), self.ks, None, 0, None, ng, W, r, self.cap_g, tab, g.off_gk, 0, 0, 0,
                                 cnt[1].data_ptr(), self.lidx[p][1].data_ptr(), self.pos[p][1].data_ptr(), g.off_gp,
                                 out[3].data_ptr() if out else None, out[2].data_ptr() if out else None, s),
                   "xr_pack get")
        else:
            cnt[1].zero_()

    def _exec_dev(self, p, kvs, skeys, svals, slens, gkeys, sstatus, gout, glens, gstatus, retries):
        from .. import _native as N
        from ..ops.arena import _check, _stream
        W, g = self.world, self.g
        x = N.XrStep()
        x.world, x.rank, x.cap_s, x.cap_g, x.ks, x.vw = W, self.rank, self.cap_s, self.cap_g, self.ks, self.vw
        ns = skeys.shape[0] if skeys is not None else 0
        ng = gkeys.shape[0] if gkeys is not None else 0
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        x.skeys, x.svals, x.slens, x.sstatus, x.n_set = ptr(skeys), ptr(svals), ptr(slens), ptr(sstatus), ns
        x.svstride = svals.shape[1] if svals is not None else 16
        x.gkeys, x.gout, x.glens, x.gstatus, x.n_get = ptr(gkeys), ptr(gout), ptr(glens), ptr(gstatus), ng
        x.gostride = gout.shape[1] if gout is not None else 16
        if W > 1:
            x.lidx_set, x.lidx_get = self.lidx[p][0].data_ptr(), self.lidx[p][1].data_ptr()
            x.own_counts = self.scnt[p].data_ptr()
            # received counts: the all-to-all's output, or (sync "flags") the posts in this window
            x.rcounts = (self._own_flag + (self.g.off_fcnt - self.g.off_flag) + p * 64 * 2 * 4
                         if self.sync == "flags" else self.rcnt[p].data_ptr())
            for s_ in range(W):
                x.req[s_], x.resp[s_] = self._exec_req[p][s_], self._exec_resp[p][s_]
        x.off_sk, x.off_sl, x.off_sv, x.off_gk = g.off_sk, g.off_sl, g.off_sv, g.off_gk
        x.off_ss, x.off_gs, x.off_gl, x.off_gv = g.off_ss, g.off_gs, g.off_gl, g.off_gv
        x.off_sp, x.off_gp = g.off_sp, g.off_gp  # -1 unless direct
        if self.direct and W > 1:  # the owners write into these: they must be this rank's outputs(p)
            o = self.outputs(p)
            assert ((sstatus is None or sstatus.data_ptr() == o[0].data_ptr())
                    and (gout is None or (gout.data_ptr() == o[1].data_ptr() and gout.shape[1] == self.vw))
                    and (glens is None or glens.data_ptr() == o[2].data_ptr())
                    and (gstatus is None or gstatus.data_ptr() == o[3].data_ptr())), \
                "direct responses: pass the arrays of outputs(i & 1) to execute()"
        _check(N.hip_lib().spl_kvs_step_xr(kvs.h, self.local.arena.desc, _stream(), ctypes.byref(x), retries,
                                           self.local.arena.stats.data_ptr()), "kvs_step_xr")

    def _gather_dev(self, p, skeys, gkeys, sstatus, gout, glens, gstatus):
        from .. import _native as N
        from ..ops.arena import _check, _stream
        L, g, s = N.hip_lib(), self.g, _stream()
        tab = self._gath_blk[p].data_ptr()
        if skeys is not None and skeys.shape[0] and sstatus is not None:
            _check(L.spl_xr_gather(self.pos[p][0].data_ptr(), skeys.shape[0], self.cap_s, tab, g.off_ss, 0, 0, 0,
                                   sstatus.data_ptr(), None, None, 0, s), "xr_gather set")
        if gkeys is not None and gkeys.shape[0] and gstatus is not None:
            _check(L.spl_xr_gather(self.pos[p][1].data_ptr(), gkeys.shape[0], self.cap_g, tab, g.off_gs, g.off_gl,
                                   g.off_gv, self.vw, gstatus.data_ptr(), glens.data_ptr(), gout.data_ptr(),
                                   gout.shape[1], s), "xr_gather get")

    # -------------------------------------------------------------- host path --
    # torch reference of the same protocol (CPU tensors, HostShard): the kernels' semantics over
    # the same byte layout, so the exchange logic is tested without a GPU.
    def _pack_host(self, p, skeys, svals, slens, gkeys):
        W, r, g = self.world, self.rank, self.g
        for kind, keys in ((0, skeys), (1, gkeys)):
            cap = self.cap_s if kind == 0 else self.cap_g
            n = keys.shape[0] if keys is not None else 0
            cnt = torch.zeros(W, dtype=torch.int32)
            if n == 0:
                self.cnt[p][kind].copy_(cnt)
                continue
            dest = shard_of(self.local.hash_keys(keys), W)
            pos = self.pos[p][kind]
            for i in range(n):  # client order within a destination (the kernel's order is any)
                d = int(dest[i])
                j = int(cnt[d])
                cnt[d] += 1
                if j >= cap:
                    pos[i] = FULL
                elif d == r:
                    self.lidx[p][kind][j] = i
                    pos[i] = OWN
                else:
                    pos[i] = d * cap + j
                    blk = g.req(p, d)  # send staging block for destination d
                    if kind == 0:
                        _view(self._send, blk + g.off_sk, cap, self.ks)[j] = keys[i]
                        _view(self._send, blk + g.off_sl, cap, 0, torch.int32)[j] = slens[i]
                        _view(self._send, blk + g.off_sv, cap, self.vw)[j] = svals[i, : self.vw]
                    else:
                        _view(self._send, blk + g.off_gk, cap, self.ks)[j] = keys[i]
            self.cnt[p][kind].copy_(cnt)

    def _exec_host(self, p, skeys, svals, slens, gkeys, sstatus, gout, glens, gstatus):
        W, r, g, vw = self.world, self.rank, self.g, self.vw
        for s_ in range(W):
            own = s_ == r
            # sets
            if self.cap_s or (own and W == 1):
                if own:
                    if W == 1:
                        idx = torch.arange(skeys.shape[0] if skeys is not None else 0)
                    else:
                        idx = self.lidx[p][0][: min(int(self.scnt[p][r, 0]), self.cap_s)].long()
                    if idx.numel():
                        sstatus[idx] = self._set_rows(skeys[idx], svals[idx], slens[idx], svals.shape[1])
                else:
                    live = min(int(self.rcnt[p][s_, 0]), self.cap_s)
                    q, o = g.req(p, s_), g.resp(p, s_)
                    if live:
                        st = self._set_rows(_view(self._win, q + g.off_sk, self.cap_s, self.ks)[:live],
                                            _view(self._win, q + g.off_sv, self.cap_s, vw)[:live],
                                            _view(self._win, q + g.off_sl, self.cap_s, 0, torch.int32)[:live], vw)
                        _view(self._send, o + g.off_ss, self.cap_s, 0, torch.int32)[:live] = st
            # gets
            if own:
                if W == 1:
                    idx = torch.arange(gkeys.shape[0] if gkeys is not None else 0)
                else:
                    idx = self.lidx[p][1][: min(int(self.scnt[p][r, 1]), self.cap_g)].long()
                if idx.numel():
                    st, v, ln = self._get_rows(gkeys[idx], gout.shape[1])
                    gstatus[idx], glens[idx] = st, ln
                    gout[idx] = v
            else:
                live = min(int(self.rcnt[p][s_, 1]), self.cap_g)
                q, o = g.req(p, s_), g.resp(p, s_)
                if live:
                    st, v, ln = self._get_rows(_view(self._win, q + g.off_gk, self.cap_g, self.ks)[:live], vw)
                    _view(self._send, o + g.off_gs, self.cap_g, 0, torch.int32)[:live] = st
                    _view(self._send, o + g.off_gl, self.cap_g, 0, torch.int32)[:live] = ln
                    _view(self._send, o + g.off_gv, self.cap_g, vw)[:live] = v

    def _set_rows(self, keys, vals, lens, vstride):
        st = self.local.set(keys.contiguous(), vals.contiguous(), lens.contiguous())
        too_long = lens.to(torch.int64) > vstride  # the kernel's bound on the source row
        return torch.where(too_long, torch.full_like(st, EMSGSIZE), st)

    def _get_rows(self, keys, width):
        st, v, ln = self.local.get(keys.contiguous())
        big = (ln > width) & (st == 0)
        st = torch.where(big, torch.full_like(st, EMSGSIZE), st)
        ln = torch.where(st == 0, ln, torch.zeros_like(ln))
        out = torch.zeros((keys.shape[0], width), dtype=torch.uint8)
        w = min(width, v.shape[1])
        out[:, :w] = v[:, :w] * (st == 0).unsqueeze(1).to(torch.uint8)
        return st, out, ln

    def _gather_host(self, p, skeys, gkeys, sstatus, gout, glens, gstatus):
        g = self.g
        for kind, keys in ((0, skeys), (1, gkeys)):
            if keys is None or keys.shape[0] == 0:
                continue
            cap = self.cap_s if kind == 0 else self.cap_g
            pos = self.pos[p][kind][: keys.shape[0]]
            for i in range(keys.shape[0]):
                q = int(pos[i])
                if q == OWN:
                    continue
                if q == FULL:
                    if kind == 0:
                        sstatus[i] = EAGAIN
                    else:
                        gstatus[i], glens[i] = EAGAIN, 0
                    continue
                d, j = divmod(q, cap)
                o = g.resp(p, d)
                if kind == 0:
                    sstatus[i] = _view(self._win, o + g.off_ss, cap, 0, torch.int32)[j]
                else:
                    st = int(_view(self._win, o + g.off_gs, cap, 0, torch.int32)[j])
                    gstatus[i] = st
                    glens[i] = int(_view(self._win, o + g.off_gl, cap, 0, torch.int32)[j]) if st == 0 else 0
                    if st == 0:
                        w = min(self.vw, gout.shape[1])
                        gout[i, :w] = _view(self._win, o + g.off_gv, cap, self.vw)[j, :w]

    # ----------------------------------------------------------- one-shot API --
    def step(self, i: int, kvs=None, skeys=None, svals=None, slens=None, gkeys=None, gout=None):
        """All four phases on the current stream: -> (set status, get status, get values, get lens)."""
        dev = self.dev
        ns = skeys.shape[0] if skeys is not None else 0
        ng = gkeys.shape[0] if gkeys is not None else 0
        if self.direct:  # the results land in this rank's output arrays: copied out for the caller
            ss, gv, gl, gs = self.outputs(i & 1)
            self.request(i, skeys, svals, slens, gkeys)
            self.execute(i, kvs, ss, gv, gl, gs)
            self.respond(i)
            self.finish(i, ss, gv, gl, gs)
            if gout is None:
                gout = gv[:ng].clone()
            else:
                w = min(self.vw, gout.shape[1])
                gout[:ng, :w] = gv[:ng, :w]
            return ss[:ns].clone(), gs[:ng].clone(), gout, gl[:ng].clone()
        sstatus = torch.empty(ns, dtype=torch.int32, device=dev)
        gstatus = torch.empty(ng, dtype=torch.int32, device=dev)
        glens = torch.empty(ng, dtype=torch.int32, device=dev)
        if gout is None:
            gout = torch.zeros((ng, self.vw), dtype=torch.uint8, device=dev)
        self.request(i, skeys, svals, slens, gkeys)
        self.execute(i, kvs, sstatus, gout, glens, gstatus)
        self.respond(i)
        self.finish(i, sstatus, gout, glens, gstatus)
        return sstatus, gstatus, gout, glens

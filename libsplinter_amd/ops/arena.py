"""Batched GPU arena operations (torch tensors in, torch tensors out).

Thin, checked wrappers over the gfx950 launchers in
``csrc/hip/arena_kernels.hip`` (C API: ``csrc/include/arena_api.h``).  Kernels
run on torch's current HIP stream, so they compose with torch ops, CUDA
graphs and ``torch.distributed`` collectives.

Key batches are uint8 tensors ``[n, kstride]`` (NUL padded, kstride in
{16,32,48,64}); value batches are uint8 ``[n, vstride]`` plus int32 lengths.
Per-op status codes: 0 ok, -11 EAGAIN, -2 ENOENT, -28 ENOSPC, -90 EMSGSIZE,
-91 EPROTOTYPE, -22 EINVAL.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np
import torch

from ..utils.tracing import trace_range
from .. import _native as N
from ..store import Store

OK, EAGAIN, ENOENT, ENOSPC, EMSGSIZE, EPROTOTYPE, EINVAL = 0, -11, -2, -28, -90, -91, -22
META = {"set_label": 0, "unset_label": 1, "bump": 2, "epoch": 3, "watch": 4, "unwatch": 5, "pulse": 6,
        "system": 7, "retrain": 8, "type": 9, "ctime": 10, "atime": 11, "find": 12}
SCAN_LIST, SCAN_LABELS, SCAN_EMBEDDED, SCAN_OCCUPIED, SCAN_ODD = 0, 1, 2, 3, 4


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what}: HIP launch failed (hipError {rc})")


def _keys(keys: torch.Tensor) -> torch.Tensor:
    """Validate a key batch; strided views (e.g. K[::2]) are compacted first."""
    if keys.dtype != torch.uint8 or keys.dim() != 2 or not keys.is_cuda:
        raise TypeError("keys must be a CUDA uint8 tensor [n, kstride]")
    if keys.shape[1] not in (16, 32, 48, 64):
        raise ValueError("kstride must be 16, 32, 48 or 64")
    return keys.contiguous()


def pack_keys(keys: Sequence, kstride: int = 0, device="cuda") -> torch.Tensor:
    """Strings/bytes -> NUL-padded uint8 key records on `device`."""
    bs = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
    longest = max((len(b) for b in bs), default=1)
    if kstride == 0:
        kstride = min(64, (min(longest, 63) + 1 + 15) // 16 * 16)
    arr = np.zeros((len(bs), kstride), dtype=np.uint8)
    for i, b in enumerate(bs):
        b = b[: min(63, kstride - 1)]
        arr[i, : len(b)] = np.frombuffer(b, dtype=np.uint8)
    return torch.from_numpy(arr).to(device)


def pack_values(values: Sequence, vstride: int = 0, device="cuda") -> Tuple[torch.Tensor, torch.Tensor]:
    bs = [v.encode() if isinstance(v, str) else bytes(v) for v in values]
    longest = max((len(b) for b in bs), default=1)
    if vstride == 0:
        vstride = max(16, (longest + 15) // 16 * 16)
    arr = np.zeros((len(bs), vstride), dtype=np.uint8)
    lens = np.zeros(len(bs), dtype=np.int32)
    for i, b in enumerate(bs):
        arr[i, : len(b)] = np.frombuffer(b, dtype=np.uint8)
        lens[i] = len(b)
    return torch.from_numpy(arr).to(device), torch.from_numpy(lens).to(device)


def unpack(vals: torch.Tensor, lens: torch.Tensor) -> list:
    v = vals.cpu().numpy()
    ln = lens.cpu().numpy()
    return [bytes(v[i, : ln[i]]) for i in range(len(ln))]


class KvStreams:
    """A group of concurrent client streams issuing one KV step natively (spl_kvs_*, hip/arena_kernels.hip):
    ``writers`` streams share the set batch, ``readers`` the get batch; the current torch stream
    continues after all of them.  Submission modes (``set_fused``; SPL_KVS_FUSED sets the default):
    0 each slice its own launch on its own stream, 2 every slice in one fused grid on the
    current stream, 3 each client stream posts its slice with a stream-ordered doorbell write and one
    resident server grid consumes the slices as they are posted (16-B keys, <= 64 streams)."""

    def __init__(self, writers: int, readers: int):
        self._H = N.hip_lib()
        self.h = self._H.spl_kvs_create(writers, readers)
        if not self.h:
            raise RuntimeError("spl_kvs_create failed")
        self.writers, self.readers = writers, readers

    def set_fused(self, mode: int):
        """0: one launch per stream slice; 2 (default; 1 is taken as 2): every slice in one fused grid; 3:
        stream-posted slices consumed by a resident server grid."""
        _check(self._H.spl_kvs_set_fused(self.h, int(mode)), "kvs_set_fused")

    def set_sched(self, sched: int):
        """Fused-grid scheduling (mode 2): 0 fixed lane streams with a workgroup barrier per round, 1
        workgroups claim row chunks from a launch-wide counter, 2 fixed lane streams with a wave-vote
        exit (default, SPL_KVS_SCHED); -1 returns to the environment's choice."""
        _check(self._H.spl_kvs_set_sched(self.h, int(sched)), "kvs_set_sched")

    def async_error(self) -> int:
        """Mode 3: 1 if a server grid gave up waiting for a slice's post (those rows did not run; the
        flag is cleared), 0 if not, -1 before the first server step.  Waits for the last server grid."""
        return int(self._H.spl_kvs_async_error(self.h))

    def step(self, arena: "HbmArena", skeys, svals, slens, sstatus, gkeys, gout, glens, gstatus, retries: int = 64):
        n_set = skeys.shape[0] if skeys is not None else 0
        n_get = gkeys.shape[0] if gkeys is not None else 0
        kstride = (skeys if n_set else gkeys).shape[1]
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        _check(self._H.spl_kvs_step(self.h, arena.desc, _stream(), ptr(skeys), kstride, ptr(svals),
                                    svals.shape[1] if svals is not None else 16, ptr(slens), n_set, ptr(sstatus),
                                    ptr(gkeys), ptr(gout), gout.shape[1] if gout is not None else 16, ptr(glens),
                                    n_get, ptr(gstatus), retries, arena.stats.data_ptr()), "kvs_step")

    def close(self):
        if self.h:
            self._H.spl_kvs_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HbmArena:
    """A format-v4 arena resident in HBM, driven by batched kernels.

    Wraps an ``hbm:`` :class:`Store` (which also offers the full single-op
    reference API); ``arena`` is the device descriptor the kernels take.
    """

    def __init__(self, store: Store):
        if store.backend != "hbm":
            raise ValueError("HbmArena needs an hbm: store")
        self.store = store
        self._H = N.hip_lib()
        self.desc = N.Arena()
        if self._H.spl_hbm_arena(store.handle, ctypes.byref(self.desc)) != 0:
            raise RuntimeError("spl_hbm_arena failed")
        self.slots, self.max_val, self.stride = self.desc.slots, self.desc.max_val, self.desc.stride
        self.stats = torch.zeros(4, dtype=torch.int64, device="cuda")  # attempts, ok, eagain, miss

    @classmethod
    def create(cls, name: str, slots: int, max_val: int, embeddings: bool = True) -> "HbmArena":
        n = name if name.startswith("hbm:") else "hbm:" + name
        return cls(Store.create(n, slots, max_val, embeddings=embeddings))

    @classmethod
    def join_node(cls, node: str, rank: int, world: int, slots: int, max_val: int,
                  embeddings: bool = True) -> "HbmArena":
        """This rank's shard of node store ``node:<node>`` (node_store.hpp): the shard arena
        ``hbm:<node>.s<rank>`` on this process's GPU, registered with the node descriptor, so once
        every rank has joined any process -- the CLI, a C / Rust / TS client -- opens
        ``node:<node>`` and reaches every rank's keys through the C ABI.  ``close`` leaves the node."""
        from ..store import NODE_HBM, node_join, node_shard_name
        a = cls(Store.create(node_shard_name(node, rank, NODE_HBM), slots, max_val, embeddings=embeddings))
        try:
            node_join(node, rank, world, NODE_HBM, a.slots, max_val, embeddings)
        except Exception:
            a.store.close()
            raise
        a.node = (node, rank)
        return a

    node = None

    def close(self):
        if self.node is not None:
            from ..store import node_leave
            node_leave(*self.node)
            self.node = None
        self.store.close()

    @property
    def embeddings(self) -> bool:
        return self.stride == 3200

    def refresh(self):
        """Re-read the descriptor (event-bus armed flag)."""
        self._H.spl_hbm_arena(self.store.handle, ctypes.byref(self.desc))

    # ------------------------------------------------------------ batches --
    def set(self, keys: torch.Tensor, vals: torch.Tensor, lens: torch.Tensor, retries: int = 64,
            status: Optional[torch.Tensor] = None) -> torch.Tensor:
        keys = _keys(keys)
        n = keys.shape[0]
        vals, lens = vals.contiguous(), lens.contiguous()
        assert vals.dtype == torch.uint8 and vals.is_cuda
        assert vals.shape[0] == n and lens.shape[0] == n and lens.dtype in (torch.int32, torch.uint32)
        if status is None:
            status = torch.empty(n, dtype=torch.int32, device=keys.device)
        with trace_range("arena.set"):
            _check(self._H.spl_arena_set(self.desc, keys.data_ptr(), keys.shape[1], vals.data_ptr(), vals.shape[1],
                                         lens.data_ptr(), n, status.data_ptr(), retries, self.stats.data_ptr(),
                                         _stream()), "arena_set")
        return status

    def get(self, keys: torch.Tensor, out: Optional[torch.Tensor] = None, retries: int = 64,
            status: Optional[torch.Tensor] = None, out_lens: Optional[torch.Tensor] = None):
        keys = _keys(keys)
        n = keys.shape[0]
        if out is None:
            out = torch.empty((n, (self.max_val + 15) // 16 * 16), dtype=torch.uint8, device=keys.device)
        assert out.shape[0] == n and out.is_contiguous() and out.shape[1] % 16 == 0
        if status is None:
            status = torch.empty(n, dtype=torch.int32, device=keys.device)
        if out_lens is None:
            out_lens = torch.empty(n, dtype=torch.int32, device=keys.device)
        with trace_range("arena.get"):
            _check(self._H.spl_arena_get(self.desc, keys.data_ptr(), keys.shape[1], out.data_ptr(), out.shape[1],
                                         out_lens.data_ptr(), n, status.data_ptr(), retries, self.stats.data_ptr(),
                                         _stream()), "arena_get")
        return status, out, out_lens

    # --------------------------------------------- segmented (routed C1) --
    def set_seg(self, keys: torch.Tensor, vals: torch.Tensor, lens: torch.Tensor, counts: torch.Tensor, cap: int,
                retries: int = 64, status: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Set over a routed buffer of ``n/cap`` segments of which only the first
        ``counts[s]`` rows are live (parallel/sharded.py RoutedKV); dead rows get
        EINVAL and are not counted in the stats."""
        keys = _keys(keys)
        n = keys.shape[0]
        assert vals.is_contiguous() and lens.is_contiguous() and counts.dtype == torch.int32
        assert n % cap == 0 and counts.numel() == n // cap
        if status is None:
            status = torch.empty(n, dtype=torch.int32, device=keys.device)
        with trace_range("arena.set_seg"):
            _check(self._H.spl_arena_set_seg(self.desc, keys.data_ptr(), keys.shape[1], vals.data_ptr(),
                                             vals.shape[1], lens.data_ptr(), n, status.data_ptr(), retries,
                                             self.stats.data_ptr(), counts.data_ptr(), cap, _stream()),
                   "arena_set_seg")
        return status

    def get_seg(self, keys: torch.Tensor, counts: torch.Tensor, cap: int, width: int, retries: int = 64):
        """Get over a routed buffer (see :meth:`set_seg`); values land in ``width``-byte
        rows and a longer value returns EMSGSIZE (-90).  -> (status, vals, lens)."""
        keys = _keys(keys)
        n = keys.shape[0]
        assert n % cap == 0 and counts.numel() == n // cap and counts.dtype == torch.int32 and width % 16 == 0
        out = torch.empty((n, width), dtype=torch.uint8, device=keys.device)
        status = torch.empty(n, dtype=torch.int32, device=keys.device)
        lens = torch.empty(n, dtype=torch.int32, device=keys.device)
        with trace_range("arena.get_seg"):
            _check(self._H.spl_arena_get_seg(self.desc, keys.data_ptr(), keys.shape[1], out.data_ptr(), width,
                                             lens.data_ptr(), n, status.data_ptr(), retries, self.stats.data_ptr(),
                                             counts.data_ptr(), cap, _stream()), "arena_get_seg")
        return status, out, lens

    def unset(self, keys: torch.Tensor, retries: int = 64) -> torch.Tensor:
        keys = _keys(keys)
        n = keys.shape[0]
        status = torch.empty(n, dtype=torch.int32, device=keys.device)
        _check(self._H.spl_arena_unset(self.desc, keys.data_ptr(), keys.shape[1], n, status.data_ptr(), retries,
                                       _stream()), "arena_unset")
        return status

    def integer_op(self, keys: torch.Tensor, ops: torch.Tensor, masks: Optional[torch.Tensor] = None,
                   retries: int = 64) -> Tuple[torch.Tensor, torch.Tensor]:
        keys = _keys(keys)
        n = keys.shape[0]
        ops = ops.to(torch.int32).contiguous()
        masks = None if masks is None else masks.contiguous()
        status = torch.empty(n, dtype=torch.int32, device=keys.device)
        results = torch.empty(n, dtype=torch.int64, device=keys.device)
        _check(self._H.spl_arena_intop(self.desc, keys.data_ptr(), keys.shape[1], ops.data_ptr(), _ptr(masks), n,
                                       status.data_ptr(), results.data_ptr(), retries, _stream()), "arena_intop")
        return status, results

    def meta(self, op: str, keys: torch.Tensor, args: Optional[torch.Tensor] = None):
        keys = _keys(keys)
        args = None if args is None else args.to(torch.int64).contiguous()
        n = keys.shape[0]
        status = torch.empty(n, dtype=torch.int32, device=keys.device)
        out = torch.empty(n, dtype=torch.int64, device=keys.device)
        _check(self._H.spl_arena_meta(self.desc, keys.data_ptr(), keys.shape[1], META[op], _ptr(args), n,
                                      status.data_ptr(), out.data_ptr(), _stream()), "arena_meta")
        return status, out

    def set_embeddings(self, keys: torch.Tensor, vecs: torch.Tensor) -> torch.Tensor:
        keys = _keys(keys)
        n = keys.shape[0]
        assert vecs.dtype == torch.float32 and vecs.shape == (n, 768) and vecs.is_contiguous()
        status = torch.empty(n, dtype=torch.int32, device=keys.device)
        _check(self._H.spl_arena_embed_set(self.desc, keys.data_ptr(), keys.shape[1], vecs.data_ptr(), n,
                                           status.data_ptr(), _stream()), "arena_embed_set")
        return status

    def get_embeddings(self, keys: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        keys = _keys(keys)
        n = keys.shape[0]
        vecs = torch.empty((n, 768), dtype=torch.float32, device=keys.device)
        status = torch.empty(n, dtype=torch.int32, device=keys.device)
        _check(self._H.spl_arena_embed_get(self.desc, keys.data_ptr(), keys.shape[1], vecs.data_ptr(), n,
                                           status.data_ptr(), _stream()), "arena_embed_get")
        return status, vecs

    def scan(self, mode: int = SCAN_LIST, mask: int = 0, cap: Optional[int] = None):
        """Compacted slot indices (uint32 as int32) + epochs of matching slots."""
        cap = self.slots if cap is None else cap
        idx = torch.empty(cap, dtype=torch.int32, device="cuda")
        ep = torch.empty(cap, dtype=torch.int64, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        _check(self._H.spl_arena_scan(self.desc, mode, mask, idx.data_ptr(), ep.data_ptr(), cap, cnt.data_ptr(),
                                      _stream()), "arena_scan")
        n = min(int(cnt.item()), cap)
        return idx[:n], ep[:n]

    def stuck_slots(self, hold_ms: float = 50.0) -> Tuple[torch.Tensor, torch.Tensor]:
        """Watchdog (SURVEY §5 failure detection): slots whose epoch is odd in two
        scans ``hold_ms`` apart with the SAME epoch, i.e. a writer that started and
        never finished (crashed process, killed kernel).  The reference's only
        recovery is retrain (splinter.c:799-833); callers decide whether to
        ``meta("retrain", ...)`` the returned keys.  Returns (slot idx, epoch)."""
        import time
        i1, e1 = self.scan(SCAN_ODD)
        torch.cuda.synchronize()
        time.sleep(hold_ms / 1e3)
        i2, e2 = self.scan(SCAN_ODD)
        if i1.numel() == 0 or i2.numel() == 0:
            return i2[:0], e2[:0]
        first = dict(zip(i1.tolist(), e1.tolist()))
        keep = [k for k, (i, e) in enumerate(zip(i2.tolist(), e2.tolist())) if first.get(i) == e]
        sel = torch.tensor(keep, dtype=torch.long, device=i2.device)
        return i2[sel], e2[sel]

    def purge(self):
        _check(self._H.spl_arena_purge(self.desc, _stream()), "arena_purge")

    # ------------------------------------------------------- raw views ----
    def _tensor_view(self, offset: int, nbytes: int) -> torch.Tensor:
        """uint8 torch view of device bytes [offset, offset+nbytes) of the arena."""
        return _device_view(self.desc.base + offset, nbytes)

    def embedding_matrix(self) -> torch.Tensor:
        """[slots, 768] fp32 strided view of every slot's vector (zero copy).  Writes through this view
        bypass the embedding writers: call :meth:`rebuild_vec16` afterwards so the side region's bf16
        copy (what the batched search streams) matches."""
        assert self.embeddings
        base = self.desc.base + 5440 + 128
        flat = _device_view(base, self.slots * 3200 - 128, dtype=torch.float32)
        return flat.as_strided((self.slots, 768), (800, 1))

    def slot_view(self) -> torch.Tensor:
        """[slots, stride] uint8 view of the slot array."""
        return _device_view(self.desc.base + 5440, self.slots * self.stride).view(self.slots, self.stride)

    def header_view(self) -> torch.Tensor:
        return _device_view(self.desc.base, 5440)

    # side region (csrc/include/splinter_layout.hpp): present on arenas created by this build
    SIDE_ALIGN, SIDE_HDR = 4096, 4096

    def _side_base(self) -> int:
        al = lambda v: (v + self.SIDE_ALIGN - 1) // self.SIDE_ALIGN * self.SIDE_ALIGN  # noqa: E731
        return self.desc.base + al(5440 + self.slots * self.stride + self.slots * self.max_val)

    @property
    def has_vec16(self) -> bool:
        return bool(self.desc.flags & 4)

    def rebuild_vec16(self) -> None:
        """Recompute the bf16 vector copy and squared norms from the fp32 vectors (spl_arena_vec16_rebuild)."""
        if self.has_vec16:
            _check(self._H.spl_arena_vec16_rebuild(self.desc, _stream()), "arena_vec16_rebuild")

    def vec16_view(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """(nrm2 [slots] fp32, vec16 [slots, 768] bf16): the side region's squared norms and bf16
        vector copy that the batched search streams (zero copy)."""
        if not self.has_vec16:
            raise ValueError("arena has no bf16 vector copy")
        al = lambda v: (v + self.SIDE_ALIGN - 1) // self.SIDE_ALIGN * self.SIDE_ALIGN  # noqa: E731
        sb = self._side_base()
        nrm2 = _device_view(sb + self.SIDE_HDR, self.slots * 4, dtype=torch.float32)
        v16 = _device_view(sb + self.SIDE_HDR + al(self.slots * 4), self.slots * 768 * 2).view(torch.bfloat16)
        return nrm2, v16.view(self.slots, 768)

    def checkpoint(self, path: str) -> None:
        torch.cuda.synchronize()
        if self._H.spl_hbm_checkpoint(self.store.handle, path.encode()) != 0:
            raise OSError(ctypes.get_errno(), f"checkpoint to {path} failed")

    def restore(self, path: str) -> None:
        torch.cuda.synchronize()
        if self._H.spl_hbm_restore(self.store.handle, path.encode()) != 0:
            raise OSError(ctypes.get_errno(), f"restore from {path} failed")

    def reset_stats(self):
        self.stats.zero_()


def _device_view(ptr: int, nbytes: int, dtype=torch.uint8) -> torch.Tensor:
    """Wrap raw device memory owned elsewhere as a torch tensor (no copy)."""
    itemsize = torch.tensor([], dtype=dtype).element_size()

    class _Holder:
        pass

    h = _Holder()
    h.__cuda_array_interface__ = {
        "shape": (nbytes // itemsize,),
        "typestr": {torch.uint8: "|u1", torch.float32: "<f4", torch.int64: "<i8"}[dtype],
        "data": (ptr, False),
        "version": 3,
        "strides": None,
    }
    return torch.as_tensor(h, device="cuda")


def format_keys(n: int, prefix: str = "k", width: int = 9, kstride: int = 16, first: int = 0,
                ids: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Device-side key generator (prefix + zero-padded decimal id), for tools and benches."""
    H = N.hip_lib()
    out = torch.empty((n, kstride), dtype=torch.uint8, device="cuda")
    pre = torch.tensor(list(prefix.encode()) + [0], dtype=torch.uint8, device="cuda")
    _check(H.spl_format_keys(out.data_ptr(), kstride, _ptr(ids), first, n, pre.data_ptr(), len(prefix), width,
                             _stream()), "format_keys")
    return out


def format_values(n: int, ver: int, length: int, vstride: int, first: int = 0,
                  ids: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Device-side payload generator: "ver:<v>|id:<id>|data:AAAA..." of `length` bytes."""
    H = N.hip_lib()
    out = torch.empty((n, vstride), dtype=torch.uint8, device="cuda")
    lens = torch.empty(n, dtype=torch.int32, device="cuda")
    _check(H.spl_format_values(out.data_ptr(), vstride, lens.data_ptr(), _ptr(ids), first, n, ver, length,
                               _stream()), "format_values")
    return out, lens

"""Pythonic handle over libsplinter.so (host shm/file stores and HBM stores).

Mirrors the reference's TypeScript ``SplinterStore`` surface
(/root/reference/bindings/ts/splinter.ts:50-68) and the ctypes pattern in
/root/reference/docs/bindings/python.md, but on the handle API so one process
can hold many stores.  Errors follow the C convention: methods that the C API
reports with -1 raise :class:`SplinterError` carrying errno (EAGAIN is
:class:`SplinterBusy`, meaning "retry"), except lookups, which return None.
"""
from __future__ import annotations

import ctypes
import errno as _errno
import os
from typing import Callable, Iterable, List, Optional, Tuple

import numpy as np

from . import _native as N

EMBED_DIM = 768
MAX_GROUPS = 64
MAX_SHARDS = 32

# named types / flags (splinter.h)
SLOT_VOID, SLOT_BIGINT, SLOT_BIGUINT, SLOT_JSON = 1 << 0, 1 << 1, 1 << 2, 1 << 3
SLOT_BINARY, SLOT_IMGDATA, SLOT_AUDIO, SLOT_VARTEXT = 1 << 4, 1 << 5, 1 << 6, 1 << 7
TYPE_NAMES = {SLOT_VOID: "VOID", SLOT_BIGINT: "BIGINT", SLOT_BIGUINT: "BIGUINT", SLOT_JSON: "JSON",
              SLOT_BINARY: "BINARY", SLOT_IMGDATA: "IMGDATA", SLOT_AUDIO: "AUDIO", SLOT_VARTEXT: "VARTEXT"}
SYS_AUTO_SCRUB, SYS_HYBRID_SCRUB = 1, 2
OP_AND, OP_OR, OP_XOR, OP_NOT, OP_INC, OP_DEC = range(6)
INTENT_NONE, INTENT_WILLNEED, INTENT_SEQUENTIAL, INTENT_RANDOM, INTENT_DONTNEED = range(5)
TIME_CTIME, TIME_ATIME = 0, 1
CREATE_EMBEDDINGS, CREATE_PERSISTENT, CREATE_NO_EMBEDDINGS = 1, 2, 4


class SplinterError(OSError):
    pass


class SplinterBusy(SplinterError):
    """EAGAIN: a writer held the slot; the same call succeeds on retry."""


def _raise(what: str, err: Optional[int] = None):
    e = ctypes.get_errno() if err is None else err
    if e == 0:
        e = _errno.EIO
    cls = SplinterBusy if e == _errno.EAGAIN else SplinterError
    raise cls(e, f"{what}: {os.strerror(e)}")


def _k(key) -> bytes:
    return key.encode() if isinstance(key, str) else bytes(key)


def now() -> int:
    """splinter_now(): the tick source used by shard windows."""
    return N.core_lib().splinter_now()


def unlink(name: str) -> int:
    return N.core_lib().spl_unlink(name.encode())


def _load_hip_if_present(required: bool = True) -> None:
    """HBM (and node-of-HBM) stores need libsplinter_hip.so loaded after torch (_native.hip_lib)."""
    try:
        N.hip_lib()
    except (ImportError, N.NativeMissing):
        if required:
            raise


# ------------------------------------------------------------- node stores --
NODE_SHM, NODE_HBM = 0, 1


def node_shard_name(node: str, shard: int, backend: int) -> str:
    """Store name (with its backend prefix) of shard `shard` of node store `node`."""
    buf = ctypes.create_string_buffer(256)
    if N.core_lib().spl_node_shard_name(node.encode(), shard, backend, buf, 256) < 0:
        raise ValueError(node)
    return buf.value.decode()


def node_shard_of(key, nshards: int) -> int:
    """Owning shard of `key` in an n-way node store (== parallel/sharded.py shard_of)."""
    return N.core_lib().spl_node_shard_of(_k(key), nshards)


def node_join(node: str, shard: int, nshards: int, backend: int, slots_per_shard: int, max_val: int,
              embeddings: bool, owned: Optional[bool] = None) -> None:
    """Register this rank's shard store (created first, as node_shard_name(...)) with node `node`;
    once every shard has joined, any process can open "node:<node>".  ``owned``: the shard is served
    only while this process lives (default: HBM shards yes, host shards no) -- see
    spl_node_join_ex and parallel/elastic.py."""
    stride = 3200 if embeddings else 128
    flags = (1 if (owned if owned is not None else backend == NODE_HBM) else 0)
    L = N.core_lib()
    L.spl_node_join_ex.restype = ctypes.c_int
    L.spl_node_join_ex.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_size_t,
                                   ctypes.c_size_t, ctypes.c_uint, ctypes.c_uint]
    if L.spl_node_join_ex(node.encode(), shard, nshards, backend, slots_per_shard, max_val, stride, flags) != 0:
        _raise(f"node_join {node}")


def node_leave(node: str, shard: int) -> None:
    N.core_lib().spl_node_leave(node.encode(), shard)


class ring_hold:
    """Context manager: no per-call ring worker is resident inside the block; per-call ops wait and
    are served afterwards.  For a process about to run a heavy GPU job beside per-call clients: a
    resident worker costs that job queue time-slices (profiles/r4y, r4z).

    ``ring_hold()``: every ring worker THIS process runs (``spl_ring_hold``) -- the rings of the
    stores it owns.  ``ring_hold(store)``: that hbm: store's ring, wherever its worker runs (e.g. a
    daemon whose store's ring server lives in the owner's process; ``spl_hbm_ring_hold``)."""

    def __init__(self, store: "Optional[Store]" = None):
        self.store = store

    def __enter__(self):
        from . import _native as N
        self._L = N.hip_lib()
        if self.store is None:
            self._L.spl_ring_hold(1)
        elif self._L.spl_hbm_ring_hold(self.store.handle, 1) != 0:
            _raise("ring hold")
        return self

    def __exit__(self, *exc):
        if self.store is None:
            self._L.spl_ring_hold(0)
        else:
            self._L.spl_hbm_ring_hold(self.store.handle, 0)
        return False


class Store:
    """One open store.  Use :meth:`create`, :meth:`open` or :meth:`open_or_create`."""

    def __init__(self, handle: int, name: str, owned: bool = True):
        self._h = handle
        self._owned = owned
        self.name = name
        self._L = N.core_lib()
        slots, mv, stride = N.c_u32(), N.c_u32(), N.c_u32()
        self._L.spl_store_geometry(handle, ctypes.byref(slots), ctypes.byref(mv), ctypes.byref(stride))
        self.slots, self.max_val, self.stride = slots.value, mv.value, stride.value

    # ----------------------------------------------------------- lifecycle --
    @classmethod
    def create(cls, name: str, slots: int = 1024, max_val: int = 4096, embeddings: Optional[bool] = None,
               persistent: bool = False) -> "Store":
        if name.startswith("hbm:") or (name.startswith("node:") and os.environ.get("SPLINTER_NODE_BACKEND") != "shm"):
            _load_hip_if_present()
        flags = 0
        if embeddings is True:
            flags |= CREATE_EMBEDDINGS
        elif embeddings is False:
            flags |= CREATE_NO_EMBEDDINGS
        if persistent:
            flags |= CREATE_PERSISTENT
        err = ctypes.c_int(0)
        h = N.core_lib().spl_store_create(name.encode(), slots, max_val, flags, ctypes.byref(err))
        if not h:
            _raise(f"create {name}", err.value)
        return cls(h, name)

    @classmethod
    def open(cls, name: str) -> "Store":
        if name.startswith("hbm:") or name.startswith("node:"):
            _load_hip_if_present(required=name.startswith("hbm:"))
        err = ctypes.c_int(0)
        h = N.core_lib().spl_store_open(name.encode(), ctypes.byref(err))
        if not h:
            _raise(f"open {name}", err.value)
        return cls(h, name)

    @classmethod
    def open_or_create(cls, name: str, slots: int = 1024, max_val: int = 4096, **kw) -> "Store":
        try:
            return cls.open(name)
        except SplinterError:
            return cls.create(name, slots, max_val, **kw)

    def close(self) -> None:
        if self._h:
            if self._owned:
                self._L.spl_store_close(self._h)
            self._h = None

    def shard(self, i: int) -> "Store":
        """Shard i of a node store as a Store of its own (borrowed: the node keeps it open)."""
        h = self._L.spl_node_shard(self._h, i)
        if not h:
            raise IndexError(f"{self.name}: no shard {i}")
        return Store(h, f"{self.name}#s{i}", owned=False)

    def unlink(self) -> None:
        unlink(self.name)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def use(self) -> None:
        """Make this store the current one for the splinter_* C API."""
        self._L.spl_store_use(self._h)

    @property
    def handle(self) -> int:
        return self._h

    @property
    def nshards(self) -> int:
        """Shards of a node store (1 for any other store)."""
        n = self._L.spl_node_nshards(self._h)
        return n if n > 0 else 1

    @property
    def backend(self) -> str:
        return self._L.spl_store_backend(self._h).decode()

    @property
    def embeddings(self) -> bool:
        return self.stride == 3200

    def region(self) -> Optional[memoryview]:
        """Zero-copy view of the whole mapped region (host backends)."""
        base = self._L.spl_store_base(self._h)
        if not base:
            return None
        n = self._L.spl_store_bytes(self._h)
        return memoryview((ctypes.c_uint8 * n).from_address(base)).cast("B")

    # ------------------------------------------------------------- values --
    def set(self, key, value) -> None:
        v = value.encode() if isinstance(value, str) else bytes(value)
        rc = self._L.spl_set(self._h, _k(key), v, len(v))
        if rc != 0:
            _raise(f"set {key!r}")

    def get(self, key) -> Optional[bytes]:
        buf = ctypes.create_string_buffer(self.max_val)
        n = N.c_size_t(0)
        ctypes.set_errno(0)
        rc = self._L.spl_get(self._h, _k(key), buf, self.max_val, ctypes.byref(n))
        if rc != 0:
            e = ctypes.get_errno()
            if e in (0, _errno.ENOENT):
                return None
            _raise(f"get {key!r}", e)
        return buf.raw[: n.value]

    def get_str(self, key) -> Optional[str]:
        v = self.get(key)
        return None if v is None else v.decode("utf-8", "replace")

    def unset(self, key) -> int:
        return self._L.spl_unset(self._h, _k(key))

    def append(self, key, data) -> int:
        d = data.encode() if isinstance(data, str) else bytes(data)
        n = N.c_size_t(0)
        if self._L.spl_append(self._h, _k(key), d, len(d), ctypes.byref(n)) != 0:
            _raise(f"append {key!r}")
        return n.value

    def list(self) -> List[str]:
        cap = max(self.slots, 1)
        arr = (ctypes.c_char_p * cap)()
        n = N.c_size_t(0)
        self._L.spl_list(self._h, arr, cap, ctypes.byref(n))
        return [arr[i].decode("utf-8", "replace") for i in range(n.value)]

    def keys(self) -> List[str]:
        return self.list()

    def poll(self, key, timeout_ms: int) -> bool:
        return self._L.spl_poll(self._h, _k(key), timeout_ms) == 0

    def epoch(self, key) -> int:
        return self._L.spl_get_epoch(self._h, _k(key))

    def raw(self, key) -> Optional[Tuple[memoryview, int]]:
        """Zero-copy (view, epoch) of the value; validate the epoch after use.  On hbm: stores the
        view reads HBM through the CPU mapping of the arena's dmabuf chunks (PCIe BAR)."""
        sz, ep = N.c_size_t(0), N.c_u64(0)
        p = self._L.spl_get_raw_ptr(self._h, _k(key), ctypes.byref(sz), ctypes.byref(ep))
        if not p:
            return None
        return memoryview((ctypes.c_uint8 * sz.value).from_address(p)).cast("B"), ep.value

    def set_as_system(self, key) -> None:
        if self._L.spl_set_as_system(self._h, _k(key)) != 0:
            _raise(f"set_as_system {key!r}", _errno.ENOENT)

    def snapshot(self, key) -> Optional[dict]:
        s = N.SlotSnapshot()
        if self._L.spl_get_slot_snapshot(self._h, _k(key), ctypes.byref(s)) != 0:
            return None
        return {"hash": s.hash, "epoch": s.epoch, "val_off": s.val_off, "val_len": s.val_len,
                "type_flag": s.type_flag, "user_flag": s.user_flag, "ctime": s.ctime, "atime": s.atime,
                "bloom": s.bloom, "key": s.key.decode("utf-8", "replace"),
                "embedding": np.ctypeslib.as_array(s.embedding).copy() if self.embeddings else None}

    def header(self) -> dict:
        h = N.HeaderSnapshot()
        self._L.spl_get_header_snapshot(self._h, ctypes.byref(h))
        return {k: getattr(h, k) for k, _ in N.HeaderSnapshot._fields_}

    # -------------------------------------------------------------- config --
    def set_mop(self, mode: int) -> None:
        if self._L.spl_set_mop(self._h, mode) != 0:
            _raise("set_mop")

    def get_mop(self) -> int:
        return self._L.spl_get_mop(self._h)

    def purge(self) -> None:
        self._L.spl_purge(self._h)

    # ---------------------------------------------------------- embeddings --
    def set_embedding(self, key, vec) -> None:
        v = np.ascontiguousarray(vec, dtype=np.float32).reshape(EMBED_DIM)
        if self._L.spl_set_embedding(self._h, _k(key), v.ctypes.data) != 0:
            _raise(f"set_embedding {key!r}")

    def get_embedding(self, key) -> Optional[np.ndarray]:
        out = np.zeros(EMBED_DIM, dtype=np.float32)
        ctypes.set_errno(0)
        if self._L.spl_get_embedding(self._h, _k(key), out.ctypes.data) != 0:
            e = ctypes.get_errno()
            if e in (0, _errno.ENOENT):
                return None
            _raise(f"get_embedding {key!r}", e)
        return out

    # ------------------------------------------------- typing/time/integer --
    def set_type(self, key, mask: int) -> None:
        if self._L.spl_set_named_type(self._h, _k(key), mask) != 0:
            _raise(f"set_named_type {key!r}")

    def set_time(self, key, mode: int, epoch: int, offset: int = 0) -> None:
        if self._L.spl_set_slot_time(self._h, _k(key), mode, epoch, offset) != 0:
            _raise(f"set_slot_time {key!r}")

    def integer_op(self, key, op: int, mask: int = 0) -> int:
        m = ctypes.c_uint64(mask & 0xFFFFFFFFFFFFFFFF)
        if self._L.spl_integer_op(self._h, _k(key), op, ctypes.byref(m)) != 0:
            _raise(f"integer_op {key!r}")
        v = self.get(key)
        return int.from_bytes(v[:8], "little") if v else 0

    def get_u64(self, key) -> Optional[int]:
        v = self.get(key)
        return None if v is None else int.from_bytes(v[:8].ljust(8, b"\0"), "little")

    # ------------------------------------------------------ epochs / labels --
    def bump(self, key) -> bool:
        return self._L.spl_bump_slot(self._h, _k(key)) == 0

    def retrain(self, key) -> bool:
        return self._L.spl_retrain_slot(self._h, _k(key)) == 0

    def set_label(self, key, mask: int) -> bool:
        return self._L.spl_set_label(self._h, _k(key), mask) == 0

    def unset_label(self, key, mask: int) -> bool:
        return self._L.spl_unset_label(self._h, _k(key), mask) == 0

    def set_tandem(self, base, values: Iterable) -> None:
        for i, v in enumerate(values):
            self.set(base if i == 0 else f"{base}.{i}", v)

    def unset_tandem(self, base, orders: int) -> None:
        for i in range(orders):
            self.unset(base if i == 0 else f"{base}.{i}")

    # ------------------------------------------------------------- signals --
    def watch(self, key, group: int) -> bool:
        return self._L.spl_watch_register(self._h, _k(key), group) == 0

    def unwatch(self, key, group: int) -> bool:
        return self._L.spl_watch_unregister(self._h, _k(key), group) == 0

    def watch_label(self, mask: int, group: int) -> bool:
        return self._L.spl_watch_label_register(self._h, mask, group) == 0

    def pulse(self, key) -> bool:
        return self._L.spl_pulse_keygroup(self._h, _k(key)) == 0

    def signal_count(self, group: int) -> int:
        return self._L.spl_get_signal_count(self._h, group)

    def signal_add(self, group: int, delta: int) -> None:
        """counter[group] += delta, atomically (node-wide signal propagation, parallel/signals.py)."""
        if self._L.spl_signal_add(self._h, group, delta & 0xFFFFFFFFFFFFFFFF) != 0:
            _raise("signal_add")

    def enumerate(self, mask: int) -> List[Tuple[str, int]]:
        out: List[Tuple[str, int]] = []

        @N.ENUM_CB
        def cb(key, epoch, _ud):
            out.append((key.decode("utf-8", "replace"), epoch))

        self._L.spl_enumerate_matches(self._h, mask, cb, None)
        return out

    # ----------------------------------------------------------- event bus --
    def event_bus_init(self) -> None:
        if self._L.spl_event_bus_init(self._h) != 0:
            _raise("event_bus_init")

    def event_bus_open(self) -> int:
        fd = self._L.spl_event_bus_open(self._h)
        if fd < 0:
            _raise("event_bus_open")
        return fd

    @staticmethod
    def event_bus_wait(fd: int, timeout_ms: int) -> bool:
        return N.core_lib().splinter_event_bus_wait(fd, timeout_ms) == 0

    def dirty_mask(self) -> List[int]:
        arr = (N.c_u64 * 16)()
        self._L.spl_event_bus_get_dirty(self._h, arr, 16)
        return list(arr)

    # -------------------------------------------------------------- shards --
    def shard_claim(self, shard_id: int, intent: int, priority: int, duration: int,
                    pid: Optional[int] = None, claimed_at: Optional[int] = None) -> None:
        if pid is None and claimed_at is None:
            rc = self._L.spl_shard_claim(self._h, shard_id, intent, priority, duration)
        else:
            rc = self._L.spl_shard_claim_ex(self._h, shard_id, os.getpid() if pid is None else pid, intent,
                                            priority, duration, now() if claimed_at is None else claimed_at)
        if rc != 0:
            _raise("shard_claim")

    def shard_rebid(self, shard_id: int, intent: int, priority: int, duration: int) -> bool:
        return self._L.spl_shard_rebid(self._h, shard_id, intent, priority, duration) == 0

    def shard_release(self, shard_id: int) -> bool:
        return self._L.spl_shard_release(self._h, shard_id) == 0

    def shard_election(self) -> Tuple[int, int]:
        it = N.c_u8(0)
        sid = self._L.spl_shard_election(self._h, ctypes.byref(it))
        return sid, it.value

    def shard_table(self) -> List[dict]:
        arr = (N.ShardBidSnapshot * MAX_SHARDS)()
        n = self._L.spl_shard_table_snapshot(self._h, arr, MAX_SHARDS)
        return [{k: getattr(arr[i], k) for k, _ in N.ShardBidSnapshot._fields_} for i in range(max(n, 0))]

    def madvise(self, shard_id: int, advice: int, timeout: int = 0) -> None:
        if self._L.spl_madvise(self._h, shard_id, None, 0, advice, timeout) != 0:
            _raise("madvise")

    # ------------------------------------------------------------- batches --
    # The host-array batch ABI (splinter_ext.h spl_*_batch): numpy arrays of fixed-stride NUL-padded
    # key records in, per-op status (0 / -errno) out.  hbm: stores run them through the device
    # kernels, node: stores over every shard concurrently, host stores on `threads` threads.
    @staticmethod
    def _keyrows(keys, kstride: int = 0) -> np.ndarray:
        if isinstance(keys, np.ndarray) and keys.dtype == np.uint8 and keys.ndim == 2:
            return np.ascontiguousarray(keys)
        bs = [_k(k) for k in keys]
        w = kstride or min(64, (max((len(b) for b in bs), default=1) + 1 + 15) // 16 * 16)
        out = np.zeros((len(bs), w), dtype=np.uint8)
        for i, b in enumerate(bs):
            b = b[: min(63, w - 1)]
            out[i, : len(b)] = np.frombuffer(b, dtype=np.uint8)
        return out

    def set_batch(self, keys, values, lens=None, retries: int = 64, threads: int = 8) -> np.ndarray:
        """keys: [n, kstride] uint8 records or a list of str/bytes; values: [n, vstride] uint8 rows
        (with lens) or a list of bytes.  -> int32 status [n]."""
        K = self._keyrows(keys)
        if isinstance(values, np.ndarray) and values.dtype == np.uint8 and values.ndim == 2:
            V = np.ascontiguousarray(values)
            L = np.ascontiguousarray(lens, dtype=np.uint32)
        else:
            vs = [v.encode() if isinstance(v, str) else bytes(v) for v in values]
            w = max(16, (max((len(v) for v in vs), default=1) + 15) // 16 * 16)
            V = np.zeros((len(vs), w), dtype=np.uint8)
            L = np.zeros(len(vs), dtype=np.uint32)
            for i, v in enumerate(vs):
                V[i, : len(v)] = np.frombuffer(v, dtype=np.uint8)
                L[i] = len(v)
        n = K.shape[0]
        assert V.shape[0] == n and L.shape[0] == n
        st = np.zeros(n, dtype=np.int32)
        r = self._L.spl_set_batch(self._h, K.ctypes.data, K.shape[1], V.ctypes.data, V.shape[1], L.ctypes.data, n,
                                  st.ctypes.data, retries, threads)
        if r < 0:
            _raise("set_batch")
        return st

    def get_batch(self, keys, width: int = 0, retries: int = 64, threads: int = 8):
        """-> (status int32 [n], values uint8 [n, width], lens uint32 [n]); width defaults to the
        store's max value size (a longer value: status -EMSGSIZE)."""
        K = self._keyrows(keys)
        n = K.shape[0]
        w = width or self.max_val
        out = np.zeros((n, w), dtype=np.uint8)
        ln = np.zeros(n, dtype=np.uint32)
        st = np.zeros(n, dtype=np.int32)
        r = self._L.spl_get_batch(self._h, K.ctypes.data, K.shape[1], out.ctypes.data, w, ln.ctypes.data, n,
                                  st.ctypes.data, retries, threads)
        if r < 0:
            _raise("get_batch")
        return st, out, ln

    def integer_op_batch(self, keys, ops, masks=None, threads: int = 8):
        """-> (status int32 [n], resulting u64 values [n])."""
        K = self._keyrows(keys)
        n = K.shape[0]
        O = np.ascontiguousarray(ops, dtype=np.int32)
        M = np.ascontiguousarray(masks if masks is not None else np.zeros(n), dtype=np.uint64)
        st = np.zeros(n, dtype=np.int32)
        res = np.zeros(n, dtype=np.uint64)
        r = self._L.spl_intop_batch_ex(self._h, K.ctypes.data, K.shape[1], O.ctypes.data, M.ctypes.data, n,
                                       st.ctypes.data, res.ctypes.data, threads)
        if r < 0:
            _raise("integer_op_batch")
        return st, res

    def set_embedding_batch(self, keys, vecs, threads: int = 8) -> np.ndarray:
        K = self._keyrows(keys)
        V = np.ascontiguousarray(vecs, dtype=np.float32)
        n = K.shape[0]
        assert V.shape == (n, 768)
        st = np.zeros(n, dtype=np.int32)
        r = self._L.spl_set_embedding_batch(self._h, K.ctypes.data, K.shape[1], V.ctypes.data, n, None,
                                            st.ctypes.data, threads)
        if r < 0:
            _raise("set_embedding_batch")
        return st

    # ---------------------------------------------------------------- misc --
    def find_slot(self, key) -> int:
        return self._L.spl_find_slot(self._h, _k(key))

    def sync(self, async_: bool = False) -> None:
        """msync a file-backed (persistent) store to its file."""
        if self._L.spl_store_sync(self._h, int(async_)) != 0:
            _raise(f"sync {self.name}")

    def epochs(self) -> np.ndarray:
        """Zero-copy uint64 view of every slot's seqlock epoch (host backends)."""
        reg = self.region()
        if reg is None:
            raise NotImplementedError("epochs(): host backends only (use HbmArena.stuck_slots on hbm:)")
        raw = np.frombuffer(reg, dtype=np.uint8, count=5440 + self.slots * self.stride)
        return np.lib.stride_tricks.as_strided(raw[5440 + 8:].view(np.uint64), shape=(self.slots,),
                                               strides=(self.stride,), writeable=False)

    def stuck_slots(self, hold_ms: float = 50.0) -> List[int]:
        """Watchdog: slots odd (writer active) with an unchanged epoch across
        ``hold_ms`` -- a writer that died mid-write.  Recovery is the
        caller's call: :meth:`retrain` forces epoch 4 (splinter.c:799-833)."""
        import time
        e1 = self.epochs().copy()
        time.sleep(hold_ms / 1e3)
        e2 = self.epochs()
        return [int(i) for i in np.nonzero((e1 & 1) & (e1 == e2))[0]]

    # ------------------------------------------------- probe-chain health (hbm: / node: of HBM) --
    _PROBE_FIELDS = ("live", "tombstones", "virgin", "busy", "disp_sum", "disp_max", "miss_sum", "miss_max")

    def probe_stats(self) -> dict:
        """One device pass over the slots (spl_hbm_probe_stats): live / tombstone / never-used counts,
        the probe length of a hit per live key (mean, max, histogram over 1, 2, 3-4, ..., >1024) and of
        a miss averaged over every home position, plus the rehash history."""
        L = N.hip_lib()
        buf = (ctypes.c_uint64 * 24)()
        L.spl_hbm_probe_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.spl_hbm_probe_stats.restype = ctypes.c_int
        if L.spl_hbm_probe_stats(self._h, buf) != 0:
            _raise(f"probe_stats {self.name}")
        v = list(buf)
        d = dict(zip(self._PROBE_FIELDS, v[:8]))
        d["hist"] = v[8:20]
        d["rebuilds"], d["reclaimed"], d["moved"] = v[20:23]
        d["hit_mean"] = d["disp_sum"] / d["live"] if d["live"] else 0.0
        d["miss_mean"] = d["miss_sum"] / self.slots if d["virgin"] else float(self.slots)
        return d

    def rehash(self, full: bool = False) -> dict:
        """Tombstone maintenance (spl_hbm_rehash_ex): keys move into tombstones on their own probe path
        and the tombstones left at the end of each cluster become never-used slots.  Online by
        default -- safe beside live batch / per-call ops of any process (moves hold both slots'
        seqlocks; misses and new inserts report EAGAIN while the pass runs).  ``full``: the exclusive
        rebuild (no other op of any process may run meanwhile)."""
        L = N.hip_lib()
        out = (ctypes.c_uint64 * 4)()
        L.spl_hbm_rehash_ex.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
        L.spl_hbm_rehash_ex.restype = ctypes.c_int
        if L.spl_hbm_rehash_ex(self._h, 1 if full else 0, out) != 0:
            _raise(f"rehash {self.name}")
        return dict(zip(("moved", "reclaimed", "clusters", "skipped"), list(out)))

    # ------------------------------------------------ checkpoint / degraded node --
    def checkpoint(self, path: str) -> None:
        """Write the store's v4 image to `path` (spl_store_checkpoint: host stores tmp + rename, hbm:
        stores their device image, a node store every serving shard to PATH.s<i>)."""
        L = N.core_lib()
        L.spl_store_checkpoint.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.spl_store_checkpoint.restype = ctypes.c_int
        if L.spl_store_checkpoint(self._h, path.encode()) != 0:
            _raise(f"checkpoint {self.name} -> {path}")

    def restore(self, path: str) -> None:
        """Load a checkpoint image of the same geometry into this store (exclusive: a restarting rank
        restores its shard before it joins its node)."""
        L = N.core_lib()
        L.spl_store_restore.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.spl_store_restore.restype = ctypes.c_int
        if L.spl_store_restore(self._h, path.encode()) != 0:
            _raise(f"restore {self.name} <- {path}")

    def shard_state(self, shard: int) -> int:
        """Node stores: 0 shard serves, 1 down (its rank's process is gone: ops on its keys raise
        SplinterBusy / batch rows -EAGAIN until the rank re-joins), -1 no such shard."""
        L = N.core_lib()
        L.spl_node_shard_state.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.spl_node_shard_state.restype = ctypes.c_int
        return int(L.spl_node_shard_state(self._h, shard))

    # numpy view of spl_search_hit (splinter_ext.h): key[64], sim, dist, epoch, bloom, len, type, emb, pad[2]
    _HIT_DTYPE = np.dtype([("key", "S64"), ("sim", "<f4"), ("dist", "<f4"), ("epoch", "<u8"), ("bloom", "<u8"),
                           ("len", "<u4"), ("type", "u1"), ("emb", "u1"), ("pad", "u1", (2,))])

    def search_batch(self, queries, k: int = 10, min_sim: float = -2.0, max_dist: float = 3.4e38,
                     mask: int = 0) -> np.ndarray:
        """Batched top-k (spl_search_batch, the C ABI product path): queries [nq, 768] fp32 (host)
        -> structured hits [nq, k] (fields of spl_search_hit; ``emb`` 0 marks an unused entry).  An
        hbm: store, or a node: store of HBM shards (all shards concurrently, merged per query)."""
        q = np.ascontiguousarray(np.asarray(queries, dtype=np.float32).reshape(-1, 768))
        out = np.zeros((q.shape[0], k), dtype=self._HIT_DTYPE)
        L = N.hip_lib()
        rc = L.spl_search_batch(self._h, q.ctypes.data, q.shape[0], k, float(min_sim), float(max_dist), mask,
                                out.ctypes.data)
        if rc != q.shape[0]:
            _raise(f"search_batch {self.name}")
        return out

    def maint_seq(self) -> int:
        """The arena's maintenance seq (odd while a rehash pass runs; spl_hbm_maint_seq)."""
        L = N.hip_lib()
        v = ctypes.c_uint64(0)
        L.spl_hbm_maint_seq.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.spl_hbm_maint_seq.restype = ctypes.c_int
        if L.spl_hbm_maint_seq(self._h, ctypes.byref(v)) != 0:
            _raise(f"maint_seq {self.name}")
        return int(v.value)

    def __repr__(self):
        return (f"Store({self.name!r}, backend={self.backend}, slots={self.slots}, max_val={self.max_val}, "
                f"embeddings={self.embeddings})")


def hash_key(key) -> int:
    return N.core_lib().spl_hash_key(_k(key))

"""Loader for the in-tree native libraries.

* ``libsplinter.so``      — host store + reference-compatible C ABI (g++).
* ``libsplinter_hip.so``  — gfx950 kernels + HBM backend (hipcc).

The HIP library links ``libamdhip64.so.7``.  PyTorch ships its own HIP
runtime under the same SONAME, so ``torch`` must be imported *before* the HIP
library is loaded: the dynamic linker then reuses torch's runtime and the
process holds exactly one HIP runtime.  :func:`hip_lib` enforces that order.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
BIN_DIR = os.path.join(PKG_DIR, "bin")
REPO_DIR = os.path.dirname(PKG_DIR)

_lock = threading.Lock()
_core = None
_hip = None


class NativeMissing(RuntimeError):
    """Raised when a native library is missing (run `make` / build())."""


def build(targets: str = "all", jobs: int = 8) -> None:
    """Build the native libraries in-tree with the repo Makefile."""
    subprocess.run(["make", "-C", REPO_DIR, f"-j{jobs}", targets], check=True)


def lib_path(name: str) -> str:
    return os.path.join(LIB_DIR, name)


def core_lib() -> ctypes.CDLL:
    global _core
    with _lock:
        if _core is None:
            path = lib_path("libsplinter.so")
            if not os.path.exists(path):
                raise NativeMissing(f"{path} not built; run `make host`")
            _core = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL, use_errno=True)
            _declare_core(_core)
        return _core


def hip_lib() -> ctypes.CDLL:
    """Load libsplinter_hip.so (after torch, see module docstring)."""
    global _hip
    import torch  # noqa: F401  (must precede the HIP library: one HIP runtime)

    core_lib()
    with _lock:
        if _hip is None:
            variant = os.environ.get("SPLINTER_HIP_VARIANT")  # A/B builds: lib/libsplinter_hip_<v>.so
            path = lib_path(f"libsplinter_hip_{variant}.so" if variant else "libsplinter_hip.so")
            if not os.path.exists(path):
                raise NativeMissing(f"{path} not built; run `make hip`")
            os.environ.setdefault("SPLINTER_HIP_LIB", path)
            _hip = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL, use_errno=True)
            _declare_hip(_hip)
        return _hip


# ----------------------------------------------------------------- ctypes --
c_void_p, c_char_p, c_size_t, c_int, c_uint = (ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t,
                                               ctypes.c_int, ctypes.c_uint)
c_u8, c_u16, c_u32, c_u64, c_i32, c_long = (ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32,
                                            ctypes.c_uint64, ctypes.c_int32, ctypes.c_long)


class HeaderSnapshot(ctypes.Structure):
    _fields_ = [("magic", c_u32), ("version", c_u32), ("slots", c_u32), ("max_val_sz", c_u32),
                ("epoch", c_u64), ("core_flags", c_u8), ("user_flags", c_u8),
                ("parse_failures", c_u64), ("last_failure_epoch", c_u64)]


class SlotSnapshot(ctypes.Structure):
    _fields_ = [("hash", c_u64), ("epoch", c_u64), ("val_off", c_u32), ("val_len", c_u32),
                ("type_flag", c_u8), ("user_flag", c_u8), ("ctime", c_u64), ("atime", c_u64),
                ("bloom", c_u64), ("key", ctypes.c_char * 64), ("embedding", ctypes.c_float * 768)]


class ShardBidSnapshot(ctypes.Structure):
    _fields_ = [("shard_id", c_u32), ("pid", c_u32), ("intent", c_u8), ("priority", c_u8),
                ("duration_tsc", c_u64), ("claimed_at", c_u64), ("expired", c_int), ("sovereign", c_int)]


class Arena(ctypes.Structure):
    """spl_arena_t (arena_api.h)."""
    _fields_ = [("base", c_void_p), ("slots", c_u32), ("max_val", c_u32), ("stride", c_u32), ("flags", c_u32),
                ("notify", c_u64)]


XR_MAX_WORLD = 64


class XrStep(ctypes.Structure):
    """spl_xr_step_t (csrc/include/arena_api.h): one routed step's owner side."""
    _fields_ = [("world", ctypes.c_int), ("rank", ctypes.c_int), ("cap_s", ctypes.c_long), ("cap_g", ctypes.c_long),
                ("ks", ctypes.c_int), ("vw", ctypes.c_int),
                ("skeys", ctypes.c_void_p), ("svals", ctypes.c_void_p), ("svstride", ctypes.c_int),
                ("slens", ctypes.c_void_p), ("sstatus", ctypes.c_void_p), ("n_set", ctypes.c_long),
                ("gkeys", ctypes.c_void_p), ("gout", ctypes.c_void_p), ("gostride", ctypes.c_int),
                ("glens", ctypes.c_void_p), ("gstatus", ctypes.c_void_p), ("n_get", ctypes.c_long),
                ("lidx_set", ctypes.c_void_p), ("lidx_get", ctypes.c_void_p), ("own_counts", ctypes.c_void_p),
                ("rcounts", ctypes.c_void_p),
                ("req", ctypes.c_uint64 * XR_MAX_WORLD), ("resp", ctypes.c_uint64 * XR_MAX_WORLD),
                ("off_sk", ctypes.c_long), ("off_sl", ctypes.c_long), ("off_sv", ctypes.c_long),
                ("off_gk", ctypes.c_long), ("off_ss", ctypes.c_long), ("off_gs", ctypes.c_long),
                ("off_gl", ctypes.c_long), ("off_gv", ctypes.c_long),
                ("off_sp", ctypes.c_long), ("off_gp", ctypes.c_long)]


ENUM_CB = ctypes.CFUNCTYPE(None, c_char_p, c_u64, c_void_p)
assert ctypes.sizeof(HeaderSnapshot) == 48
assert ctypes.sizeof(SlotSnapshot) == 3192
assert ctypes.sizeof(ShardBidSnapshot) == 40


def _sig(lib, name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)


def _declare_core(L):
    S = c_void_p  # spl_store*
    _sig(L, "spl_store_create", S, c_char_p, c_size_t, c_size_t, c_uint, ctypes.POINTER(c_int))
    _sig(L, "spl_store_open", S, c_char_p, ctypes.POINTER(c_int))
    _sig(L, "spl_store_close", None, S)
    _sig(L, "spl_store_use", c_int, S)
    _sig(L, "spl_store_backend", c_char_p, S)
    _sig(L, "spl_store_geometry", c_int, S, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32), ctypes.POINTER(c_u32))
    _sig(L, "spl_store_base", c_void_p, S)
    _sig(L, "spl_store_bytes", c_size_t, S)
    _sig(L, "spl_store_sync", c_int, S, c_int)
    _sig(L, "spl_unlink", c_int, c_char_p)
    _sig(L, "spl_version", c_char_p)
    _sig(L, "spl_build", c_char_p)
    _sig(L, "spl_set_mop", c_int, S, c_uint)
    _sig(L, "spl_get_mop", c_int, S)
    _sig(L, "spl_purge", None, S)
    _sig(L, "spl_get_header_snapshot", c_int, S, ctypes.POINTER(HeaderSnapshot))
    _sig(L, "spl_set", c_int, S, c_char_p, c_void_p, c_size_t)
    _sig(L, "spl_unset", c_int, S, c_char_p)
    _sig(L, "spl_get", c_int, S, c_char_p, c_void_p, c_size_t, ctypes.POINTER(c_size_t))
    _sig(L, "spl_list", c_int, S, ctypes.POINTER(c_char_p), c_size_t, ctypes.POINTER(c_size_t))
    _sig(L, "spl_poll", c_int, S, c_char_p, c_u64)
    _sig(L, "spl_get_slot_snapshot", c_int, S, c_char_p, ctypes.POINTER(SlotSnapshot))
    _sig(L, "spl_append", c_int, S, c_char_p, c_void_p, c_size_t, ctypes.POINTER(c_size_t))
    _sig(L, "spl_get_raw_ptr", c_void_p, S, c_char_p, ctypes.POINTER(c_size_t), ctypes.POINTER(c_u64))
    _sig(L, "spl_get_epoch", c_u64, S, c_char_p)
    _sig(L, "spl_set_as_system", c_int, S, c_char_p)
    _sig(L, "spl_set_embedding", c_int, S, c_char_p, c_void_p)
    _sig(L, "spl_get_embedding", c_int, S, c_char_p, c_void_p)
    _sig(L, "spl_set_named_type", c_int, S, c_char_p, c_u16)
    _sig(L, "spl_set_slot_time", c_int, S, c_char_p, ctypes.c_ushort, c_u64, c_size_t)
    _sig(L, "spl_integer_op", c_int, S, c_char_p, c_int, c_void_p)
    _sig(L, "spl_bump_slot", c_int, S, c_char_p)
    _sig(L, "spl_retrain_slot", c_int, S, c_char_p)
    _sig(L, "spl_set_label", c_int, S, c_char_p, c_u64)
    _sig(L, "spl_unset_label", c_int, S, c_char_p, c_u64)
    _sig(L, "spl_watch_register", c_int, S, c_char_p, c_u8)
    _sig(L, "spl_watch_unregister", c_int, S, c_char_p, c_u8)
    _sig(L, "spl_watch_label_register", c_int, S, c_u64, c_u8)
    _sig(L, "spl_pulse_keygroup", c_int, S, c_char_p)
    _sig(L, "spl_get_signal_count", c_u64, S, c_u8)
    _sig(L, "spl_signal_add", c_int, S, c_u8, c_u64)
    _sig(L, "spl_enumerate_matches", None, S, c_u64, ENUM_CB, c_void_p)
    _sig(L, "spl_event_bus_init", c_int, S)
    _sig(L, "spl_event_bus_open", c_int, S)
    _sig(L, "spl_event_bus_get_dirty", None, S, ctypes.POINTER(c_u64), c_size_t)
    _sig(L, "splinter_event_bus_wait", c_int, c_int, c_u64)
    _sig(L, "splinter_event_bus_close", None, c_int)
    _sig(L, "spl_shard_claim_ex", c_int, S, c_u32, c_u32, c_u8, c_u8, c_u64, c_u64)
    _sig(L, "spl_shard_claim", c_int, S, c_u32, c_u8, c_u8, c_u64)
    _sig(L, "spl_shard_rebid", c_int, S, c_u32, c_u8, c_u8, c_u64)
    _sig(L, "spl_shard_release", c_int, S, c_u32)
    _sig(L, "spl_shard_election", c_u32, S, ctypes.POINTER(c_u8))
    _sig(L, "spl_shard_table_snapshot", c_int, S, ctypes.POINTER(ShardBidSnapshot), c_size_t)
    _sig(L, "spl_madvise", c_int, S, c_u32, c_void_p, c_size_t, c_int, c_u64)
    _sig(L, "spl_find_slot", c_long, S, c_char_p)
    _sig(L, "spl_hash_key", c_u64, c_char_p)
    # host-array batches (csrc/core/batch_host.cpp)
    P = c_void_p
    _sig(L, "spl_set_batch", c_long, S, P, c_int, P, c_int, P, c_long, P, c_int, c_int)
    _sig(L, "spl_get_batch", c_long, S, P, c_int, P, c_int, P, c_long, P, c_int, c_int)
    _sig(L, "spl_intop_batch_ex", c_long, S, P, c_int, P, P, c_long, P, P, c_int)
    _sig(L, "spl_set_embedding_batch", c_long, S, P, c_int, P, c_long, P, P, c_int)
    _sig(L, "spl_batch_alloc", P, c_size_t)
    _sig(L, "spl_batch_free", None, P)
    _sig(L, "splinter_now", c_u64)
    # node stores (csrc/core/node_store.hpp)
    _sig(L, "spl_node_join", c_int, c_char_p, c_int, c_int, c_uint, c_size_t, c_size_t, c_uint)
    _sig(L, "spl_node_leave", c_int, c_char_p, c_int)
    _sig(L, "spl_node_shard_name", c_int, c_char_p, c_int, c_uint, c_char_p, c_size_t)
    _sig(L, "spl_node_nshards", c_int, S)
    _sig(L, "spl_node_shard", c_void_p, S, c_int)
    _sig(L, "spl_node_shard_of", c_int, c_char_p, c_int)


def _declare_hip(L):
    A = Arena
    P = c_void_p
    _sig(L, "spl_hbm_arena", c_int, c_void_p, ctypes.POINTER(Arena))
    _sig(L, "spl_hbm_checkpoint", c_int, c_void_p, c_char_p)
    _sig(L, "spl_hbm_restore", c_int, c_void_p, c_char_p)
    _sig(L, "spl_arena_init_slots", c_int, A, P)
    _sig(L, "spl_arena_set", c_int, A, P, c_int, P, c_int, P, c_long, P, c_int, P, P)
    _sig(L, "spl_arena_get", c_int, A, P, c_int, P, c_int, P, c_long, P, c_int, P, P)
    _sig(L, "spl_arena_set_seg", c_int, A, P, c_int, P, c_int, P, c_long, P, c_int, P, P, c_long, P)
    _sig(L, "spl_arena_get_seg", c_int, A, P, c_int, P, c_int, P, c_long, P, c_int, P, P, c_long, P)
    _sig(L, "spl_arena_set_idx", c_int, A, P, c_int, P, c_int, P, P, P, c_long, P, c_int, P, P)
    _sig(L, "spl_arena_get_idx", c_int, A, P, c_int, P, c_int, P, P, P, c_long, P, c_int, P, P)
    # routed exchange (route_kernels.hip, parallel/xroute.py)
    _sig(L, "spl_xr_pack", c_int, P, c_int, P, c_int, P, c_long, c_int, c_int, c_long, P, c_long, c_long, c_long,
         c_int, P, P, P, c_long, P, P, P)
    _sig(L, "spl_xr_gather", c_int, P, c_long, c_long, P, c_long, c_long, c_long, c_int, P, P, P, c_int, P)
    _sig(L, "spl_xr_post", c_int, P, c_int, c_int, c_int, c_int, ctypes.c_uint64, P, P)
    _sig(L, "spl_xr_wait", c_int, P, c_int, c_int, c_int, c_int, ctypes.c_uint64, ctypes.c_uint64, P, P)
    _sig(L, "spl_xr_flag_bytes", c_long)
    _sig(L, "spl_xw_create", P, c_int, c_size_t, c_char_p)
    _sig(L, "spl_xw_attach", P, c_char_p, c_int)
    _sig(L, "spl_xw_base", P, P)
    _sig(L, "spl_xw_bytes", c_size_t, P)
    _sig(L, "spl_xw_destroy", None, P)
    _sig(L, "spl_xw_peer", c_int, c_int, c_int)
    _sig(L, "spl_arena_unset", c_int, A, P, c_int, c_long, P, c_int, P)
    _sig(L, "spl_arena_intop", c_int, A, P, c_int, P, P, c_long, P, P, c_int, P)
    _sig(L, "spl_arena_meta", c_int, A, P, c_int, c_int, P, c_long, P, P, P)
    _sig(L, "spl_arena_embed_set", c_int, A, P, c_int, P, c_long, P, P)
    _sig(L, "spl_arena_embed_get", c_int, A, P, c_int, P, c_long, P, P)
    _sig(L, "spl_arena_scan", c_int, A, c_int, c_u64, P, P, c_u32, P, P)
    _sig(L, "spl_arena_scan_range", c_int, A, c_int, c_u64, c_u32, c_u32, P, P, c_u32, P, P)
    _sig(L, "spl_kvs_create", P, c_int, c_int)
    _sig(L, "spl_kvs_destroy", None, P)
    _sig(L, "spl_kvs_set_fused", c_int, P, c_int)
    _sig(L, "spl_kvs_set_sched", c_int, P, c_int)
    _sig(L, "spl_kvs_async_error", c_int, P)
    _sig(L, "spl_kvs_step", c_int, P, A, P, P, c_int, P, c_int, P, c_long, P, P, P, c_int, P, c_long, P, c_int, P)
    _sig(L, "spl_kvs_step_xr", c_int, P, A, P, ctypes.POINTER(XrStep), c_int, P)
    if hasattr(L, "spl_hbm_ring_launches"):
        _sig(L, "spl_hbm_ring_launches", c_u32, c_void_p)
    if hasattr(L, "spl_hbm_ring_mode"):
        _sig(L, "spl_hbm_ring_mode", c_int, c_void_p)
    if hasattr(L, "spl_ring_hold"):
        _sig(L, "spl_ring_hold", None, c_int)
    if hasattr(L, "spl_hbm_ring_hold"):
        _sig(L, "spl_hbm_ring_hold", c_int, c_void_p, c_int)
    _sig(L, "spl_arena_purge", c_int, A, P)
    _sig(L, "spl_arena_vec16_rebuild", c_int, A, P)
    _sig(L, "spl_arena_probe_stats", c_int, A, P, P)
    _sig(L, "spl_hbm_probe_stats", c_int, P, P)
    _sig(L, "spl_hbm_rehash", c_int, P, P)
    _sig(L, "spl_search_batch", ctypes.c_long, P, P, c_int, c_int, ctypes.c_float, ctypes.c_float, c_u64, P)
    _sig(L, "spl_arena_gather_slots", c_int, A, P, c_long, P, P)
    _sig(L, "spl_hash_keys", c_int, P, c_int, c_long, P, P)
    _sig(L, "spl_format_keys", c_int, P, c_int, P, c_u64, c_long, P, c_int, c_int, P)
    _sig(L, "spl_format_values", c_int, P, c_int, P, P, c_u64, c_long, c_u32, c_u32, P)

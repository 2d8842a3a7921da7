"""HIP streams on distinct hardware queues.

The HIP runtime maps streams onto at most GPU_MAX_HW_QUEUES (4 on our boxes)
hardware queues PER PRIORITY LEVEL, reusing the least-used queue once the
pool is full, so two busy streams of the same priority can land on one queue
and serialise (measured: the embed stream and the KV set stream shared queue 4
in profiles/r1_bench_mixed_kernel_stats.csv, so the "overlapped" phases ran
back to back).  Streams created at different priorities come from different
queue pools, so giving each concurrent phase its own priority level
guarantees separate hardware queues; the high-priority queue also wins
dispatch arbitration, which is what the latency-bound KV kernels want while
the MFMA-bound encoder fills the remaining CU slots.
"""
from __future__ import annotations

import ctypes
from typing import Dict

import torch

_hip = None
_created: Dict[int, "torch.cuda.ExternalStream"] = {}


def _lib():
    global _hip
    if _hip is None:
        torch.cuda.init()
        _hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)  # torch's copy: same SONAME, same handle
        _hip.hipStreamCreateWithPriority.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint, ctypes.c_int]
        _hip.hipStreamCreateWithPriority.restype = ctypes.c_int
        _hip.hipDeviceGetStreamPriorityRange.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        _hip.hipDeviceGetStreamPriorityRange.restype = ctypes.c_int
        _hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint32)]
        _hip.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
        _hip.hipExtStreamGetCUMask.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        _hip.hipExtStreamGetCUMask.restype = ctypes.c_int
    return _hip


def priority_range():
    """(least, greatest) priority values of the device (HIP: larger = lower priority)."""
    least, greatest = ctypes.c_int(0), ctypes.c_int(0)
    _lib().hipDeviceGetStreamPriorityRange(ctypes.byref(least), ctypes.byref(greatest))
    return least.value, greatest.value


def stream(level: str = "normal") -> torch.cuda.ExternalStream:
    """A non-blocking stream at priority level 'low' | 'normal' | 'high'."""
    least, greatest = priority_range()
    prio = {"low": least, "normal": 0, "high": greatest}[level]
    h = ctypes.c_void_p()
    rc = _lib().hipStreamCreateWithPriority(ctypes.byref(h), 1, prio)  # 1 = hipStreamNonBlocking
    if rc != 0:
        raise RuntimeError(f"hipStreamCreateWithPriority failed ({rc})")
    s = torch.cuda.ExternalStream(h.value)
    _created[h.value] = s  # keep alive for the process lifetime
    return s


def cu_mask_bits(per_xcd: int, first: int = 0, n_cus: int = 256, n_xcd: int = 8) -> list:
    """CU-mask bit indices giving `per_xcd` CUs (CU slots first .. first+per_xcd-1) on EVERY XCD.

    The CU mask of a queue on a multi-XCD part is dealt out to the XCDs bit by bit (KFD
    mqd_symmetrically_map_cu_mask: bit i -> XCD i % n_xcd, CU slot i // n_xcd).  With 8 XCDs the
    selection is made in whole 8-bit groups, bit i taken when (i // 8) % 4 is in the window, so it
    ALSO gives every XCD the same CU count if the bits were dealt in contiguous 32-bit chunks.
    Every XCD must keep at least one CU: a queue whose mask empties an XCD leaves that XCD's share
    of every grid undispatched."""
    per = n_cus // n_xcd
    if n_xcd == 8 and per == 32:
        if per_xcd % 8 or first % 8 or not (0 < per_xcd and first + per_xcd <= 32):
            raise ValueError("per_xcd / first must be multiples of 8 within 32")
        lo, hi = first // 8, (first + per_xcd) // 8
        return [i for i in range(n_cus) if lo <= (i // 8) % 4 < hi]
    if not (0 < per_xcd and first + per_xcd <= per):
        raise ValueError("CU window outside the XCD")
    return [i for i in range(n_cus) if first <= i // n_xcd < first + per_xcd]


def masked_stream(bits) -> torch.cuda.ExternalStream:
    """A stream on its own hardware queue restricted to the CUs in `bits` (hipExtStreamCreateWithCUMask)."""
    bits = list(bits)
    nw = (max(bits) // 32 + 1) if bits else 1
    words = (ctypes.c_uint32 * nw)()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    h = ctypes.c_void_p()
    rc = _lib().hipExtStreamCreateWithCUMask(ctypes.byref(h), nw, words)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    s = torch.cuda.ExternalStream(h.value)
    _created[h.value] = s
    return s


def stream_cu_mask(s) -> list:
    w = (ctypes.c_uint32 * 8)()
    rc = _lib().hipExtStreamGetCUMask(ctypes.c_void_p(s.cuda_stream), 8, w)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamGetCUMask failed ({rc})")
    return [i for i in range(256) if w[i // 32] >> (i % 32) & 1]

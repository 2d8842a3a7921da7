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

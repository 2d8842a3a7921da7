"""roctx ranges + host-side counters (SURVEY §5 tracing / observability).

The reference has no tracer (timing only via splinter_now TSC reads,
splinter.h:872-893).  Here every batched host entry point can be wrapped in a
roctx range, so `rocprofv3 --marker-trace` (or `--kernel-trace` with
`--marker-trace` in a separate run from any --pmc collection) shows which API
batch launched which kernels.  Ranges are enabled with SPLINTER_ROCTX=1 and
cost nothing otherwise; the library is the rocprofiler-sdk roctx shim shipped
in /opt/rocm/lib, loaded lazily.  ``Counters`` accumulates per-process op /
retry / byte counts for the `stats` views without touching the v4 header.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
import time
from collections import defaultdict
from typing import Dict, Optional

_lib: Optional[ctypes.CDLL] = None
_enabled = os.environ.get("SPLINTER_ROCTX", "0") not in ("", "0")


def _roctx() -> Optional[ctypes.CDLL]:
    global _lib, _enabled
    if _lib is None and _enabled:
        for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "libroctx64.so"):
            try:
                _lib = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if _lib is None:
            _enabled = False
        else:
            _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _lib.roctxRangePushA.restype = ctypes.c_int
            _lib.roctxRangePop.restype = ctypes.c_int
            _lib.roctxMarkA.argtypes = [ctypes.c_char_p]
    return _lib


def enable(on: bool = True) -> bool:
    """Turn ranges on/off at runtime; returns whether the roctx library is usable."""
    global _enabled
    _enabled = on
    return _roctx() is not None if on else False


@contextlib.contextmanager
def trace_range(name: str):
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


class Counters:
    """Thread-safe named counters + wall-time accumulators."""

    def __init__(self):
        self._lock = threading.Lock()
        self.counts: Dict[str, int] = defaultdict(int)
        self.seconds: Dict[str, float] = defaultdict(float)

    def add(self, name: str, n: int = 1) -> None:
        with self._lock:
            self.counts[name] += n

    @contextlib.contextmanager
    def timed(self, name: str):
        t0 = time.perf_counter()
        with trace_range(name):
            yield
        with self._lock:
            self.seconds[name] += time.perf_counter() - t0
            self.counts[name + ".calls"] += 1

    def snapshot(self) -> Dict[str, float]:
        with self._lock:
            out: Dict[str, float] = dict(self.counts)
            out.update({k + ".s": v for k, v in self.seconds.items()})
            return out


GLOBAL = Counters()

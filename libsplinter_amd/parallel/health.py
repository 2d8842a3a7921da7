"""Rank liveness and collective failure handling for the one-process-per-GPU node.

SURVEY §5 asks for per-rank liveness and an abort path: the reference is single-host shared
memory and has neither (a crashed writer leaves an odd epoch; /root/reference/splinter.h:398-412).
On a sharded node a dead rank would leave every peer blocked in its next collective.  Three layers:

* ``init_distributed(backend, timeout_s)``: process group with a finite collective timeout, and
  RCCL's asynchronous error handling on (``TORCH_NCCL_ASYNC_ERROR_HANDLING=1``), so a collective
  that cannot complete aborts its communicator and raises instead of hanging forever;
* ``Liveness``: a heartbeat thread per rank on the rendezvous key-value store (rank r writes
  ``hb/r`` every ``period_s``) plus a monitor that, when any peer's heartbeat is older than
  ``timeout_s`` (or the store itself is gone -- rank 0 hosts it), ends this process with
  ``EXIT_PEER_LOST`` via ``os._exit`` (a blocked collective cannot be interrupted from Python; the
  launcher, torchrun or bench.py, then reports the failure).  Never a re-exec;
* ``guarded(fn)``: run a step, turning a collective error into the same non-zero exit.

Degraded serving instead of the exit: ``Liveness(degrade=True)`` with parallel/elastic.py (the node
store answers EAGAIN for a lost rank's shard; a supervisor restarts the rank as a fresh process
that restores its checkpoint and re-joins).
"""
from __future__ import annotations

import os
import sys
import threading
import time
from datetime import timedelta
from typing import Optional

import torch.distributed as dist

EXIT_PEER_LOST = 17


def init_distributed(backend: str = "nccl", timeout_s: float = 120.0, device_id=None) -> None:
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    kw = {"timeout": timedelta(seconds=timeout_s)}
    if device_id is not None and backend == "nccl":
        kw["device_id"] = device_id
    dist.init_process_group(backend, **kw)


def _default_store():
    from torch.distributed import distributed_c10d as c10d
    return c10d._get_default_store()


class Heartbeat:
    """Rank ``rank``'s heartbeat on a key-value store (``splinter/hb/<rank>`` = wall time, every
    ``period_s``).  A rank restarted as a fresh process (parallel/elastic.py) is no member of the old
    process group, but beats on the same store, so its survivors see it back."""

    def __init__(self, store, rank: int, period_s: float = 1.0):
        self.store, self.rank, self.period = store, rank, period_s
        self._stop = threading.Event()
        self.beat()
        self._t = threading.Thread(target=self._run, name="splinter-heartbeat", daemon=True)
        self._t.start()

    def beat(self):
        self.store.set(f"splinter/hb/{self.rank}", repr(time.time()))

    def _run(self):
        while not self._stop.wait(self.period):
            try:
                self.beat()
            except Exception:  # the store is gone: nothing left to tell
                return

    def stop(self):
        self._stop.set()
        self._t.join(self.period * 4)


class Liveness:
    """Heartbeat + peer monitor.  Default: a lost peer ends this process (EXIT_PEER_LOST).
    ``degrade=True``: the loss is reported (``on_lost(rank)``) and this rank keeps running -- its
    node-store shard keeps serving, ops on the lost rank's shard answer EAGAIN (node_store.hpp) --
    and a peer whose heartbeat comes back (its restarted process) is reported by ``on_back(rank)``."""

    def __init__(self, period_s: float = 1.0, timeout_s: float = 10.0, exit_code: int = EXIT_PEER_LOST,
                 on_lost=None, degrade: bool = False, on_back=None, store=None):
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.period, self.timeout, self.exit_code = period_s, timeout_s, exit_code
        self.on_lost = on_lost  # called instead of os._exit
        self.on_back = on_back
        self.degrade = degrade
        # the heartbeat keys' store: the process group's (default) or one the caller shares with
        # processes outside the group (a restarted rank, parallel/elastic.py)
        self.store = store if store is not None else _default_store()
        self._stop = threading.Event()
        self.lost: Optional[int] = None
        self.down = set()
        self._beat()
        self._t = threading.Thread(target=self._run, name="splinter-liveness", daemon=True)
        self._t.start()

    def _beat(self):
        self.store.set(f"splinter/hb/{self.rank}", repr(time.time()))

    def _lost(self, who: int, why: str):
        self.lost = who
        self.down.add(who)
        tail = "serving degraded" if self.degrade else f"exiting with {self.exit_code}"
        print(f"[splinter] rank {self.rank}: peer {who} lost ({why}); {tail}", file=sys.stderr, flush=True)
        if self.on_lost is not None:
            self.on_lost(who)
            return
        os._exit(self.exit_code)

    def _back(self, who: int):
        self.down.discard(who)
        print(f"[splinter] rank {self.rank}: peer {who} back", file=sys.stderr, flush=True)
        if self.on_back is not None:
            self.on_back(who)

    def _run(self):
        start = time.time()
        while not self._stop.wait(self.period):
            try:
                self._beat()
                now = time.time()
                for r in range(self.world):
                    if r == self.rank:
                        continue
                    key = f"splinter/hb/{r}"
                    if not self.store.check([key]):
                        if now - start > self.timeout and r not in self.down:
                            self._lost(r, "no heartbeat")
                            if not self.degrade:
                                return
                        continue
                    age = now - float(self.store.get(key).decode())
                    if age > self.timeout and r not in self.down:
                        self._lost(r, f"heartbeat {age:.1f} s old")
                        if not self.degrade:
                            return
                    elif age <= self.timeout and r in self.down:
                        self._back(r)
            except Exception as e:  # the store (hosted by rank 0) is gone
                if self._stop.is_set():
                    return
                return self._lost(0, f"store unreachable: {e!r}"[:200])

    def stop(self):
        self._stop.set()
        self._t.join(self.period * 4)


def _collective_errors():
    """Exception types that mean a collective (not local code) failed: the backend error, the
    store/rendezvous timeout and a lost connection to a peer."""
    errs = []
    for name in ("DistBackendError", "DistNetworkError", "DistStoreError"):
        if hasattr(dist, name):
            errs.append(getattr(dist, name))
    return tuple(errs)


_COLLECTIVE_MARKERS = ("NCCL", "RCCL", "Gloo", "gloo", "collective", "timed out", "Connection reset",
                       "Connection closed by peer", "ProcessGroup")


def guarded(fn, *a, exit_code: int = EXIT_PEER_LOST, **kw):
    """Run ``fn``; a collective failure (timeout, aborted communicator, lost peer) ends the
    process with ``exit_code`` instead of leaving it half-alive.  Any other exception -- a HIP
    out-of-memory, a kernel launch failure, a shape bug in the step -- propagates with its
    traceback: it is this rank's fault, not a lost peer."""
    try:
        return fn(*a, **kw)
    except _collective_errors() as e:
        _peer_lost(e, exit_code)
    except RuntimeError as e:
        # older torch builds raise plain RuntimeErrors from the process group: classify by message
        if any(m in str(e) for m in _COLLECTIVE_MARKERS):
            _peer_lost(e, exit_code)
        raise


def _peer_lost(e, exit_code):
    print(f"[splinter] rank {dist.get_rank() if dist.is_initialized() else '?'}: collective failed: {e!r}"[:500],
          file=sys.stderr, flush=True)
    os._exit(exit_code)

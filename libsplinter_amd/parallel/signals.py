"""C2 signal-group propagation across the shards of a node.

In the reference every pulse bumps the one shared ``signal_groups`` array of the store
(/root/reference/splinter.c:941-955), so a watcher sees pulses of every key.  In a sharded arena a
key's pulses land in the counters of the shard that owns it; a watcher polling its local store
(``splinter_get_signal_count`` through the C API, the CLI ``watch --group``, a daemon's 50 ms poll)
must still see them.  ``SignalSync`` runs one background thread per rank that, every
``period_ms``, all-reduces the rank's *locally originated* counter values over a dedicated gloo
group (512 B of host tensors: it never queues behind RCCL traffic on the device) and adds the
remote part into the local store's counters, so every shard's counters converge to the node-wide
sums within one period:

    local_origin = counters - injected          (pulses that happened on this shard)
    total        = all_reduce(local_origin)     (node-wide)
    delta        = (total - local_origin) - injected,   counters += delta,   injected += delta

Counters stay monotonic, and a local watcher wakes exactly as for a local pulse.  Stopping is a
vote carried by the same all-reduce, so every rank leaves on the same round; a peer that dies
makes the all-reduce time out (``timeout_s``) and the thread records the error (see health.py
for the node-level reaction).
"""
from __future__ import annotations

import threading
import time
from datetime import timedelta
from typing import Optional

import torch
import torch.distributed as dist


class SignalSync:
    def __init__(self, shard, period_ms: float = 20.0, timeout_s: float = 30.0, group=None):
        """``shard``: the local shard (GpuShard / HostShard) -- needs ``signal_counts()`` and a
        store with ``signal_add``.  Collective constructor: every rank must create it."""
        self.shard = shard
        self.period = period_ms / 1e3
        self.pg = group if group is not None else dist.new_group(backend="gloo",
                                                                  timeout=timedelta(seconds=timeout_s))
        self.injected = torch.zeros(64, dtype=torch.int64)
        self.rounds = 0
        self.error: Optional[BaseException] = None
        self._stop = False
        self._thread = threading.Thread(target=self._loop, name="splinter-signal-sync", daemon=True)
        self._thread.start()

    def _store(self):
        s = getattr(self.shard, "store", None)
        return s if s is not None else self.shard.arena.store

    def _loop(self):
        store = self._store()
        try:
            while True:
                cur = self.shard.signal_counts().to("cpu", torch.int64)
                local = cur - self.injected
                buf = torch.cat([local, torch.tensor([1 if self._stop else 0], dtype=torch.int64)])
                dist.all_reduce(buf, group=self.pg)
                if int(buf[64]) > 0:
                    break
                delta = ((buf[:64] - local) - self.injected).clamp(min=0)
                for g in torch.nonzero(delta).flatten().tolist():
                    store.signal_add(g, int(delta[g]))
                self.injected += delta
                self.rounds += 1
                time.sleep(self.period)
        except BaseException as e:  # a dead peer or a torn-down group
            self.error = e

    def stop(self, timeout: Optional[float] = None) -> None:
        """Vote to stop; returns once this rank's thread has left (all ranks leave together)."""
        self._stop = True
        self._thread.join(timeout)

    @property
    def alive(self) -> bool:
        return self._thread.is_alive()

"""Hash-sharded KV arena across the GPUs of a node (one process per GPU).

The reference is single-host shared memory (no collectives);
its closest scale-out idea is the disjoint key lanes of splinter_chi_sao
(/root/reference/splinter_chi_sao.c:400-418).  Here the key space is sharded:
shard(key) = (fnv1a(key) >> 40) % world, so a shard's in-arena probe (which
uses fnv1a % slots, the low bits) stays well spread.  Each rank owns one HBM
arena; a batch of client ops is routed to owners with RCCL all-to-all over
xGMI (collective C1 of SURVEY §2.10), executed by the owner's kernels, and the
results are routed back.  All 7 xGMI links are driven at once by the
all-to-all (direct peer exchange, not a ring).

The local shard is pluggable (anything with ``hash_keys / set / get``), so the
routing logic is exercised on CPU with gloo + the host backend in tests.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

SHARD_SHIFT = 40


def shard_of(hashes: torch.Tensor, world: int) -> torch.Tensor:
    """Owner rank for each 64-bit FNV-1a hash (int64 bit pattern)."""
    hi = (hashes >> SHARD_SHIFT) & 0xFFFFFF  # arithmetic shift of int64: mask the sign-extended bits
    return torch.remainder(hi, world)


class ShardedKV:
    def __init__(self, local, group: Optional[dist.ProcessGroup] = None):
        self.local = local
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
        else:
            self.world, self.rank = 1, 0

    # ----------------------------------------------------------- routing --
    def _plan(self, keys: torch.Tensor):
        h = self.local.hash_keys(keys)
        dest = shard_of(h, self.world)
        order = torch.argsort(dest, stable=True)
        send = torch.bincount(dest, minlength=self.world)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        s, r = send.tolist(), recv.tolist()
        return order, s, r

    def _route(self, x: torch.Tensor, send_splits, recv_splits) -> torch.Tensor:
        out = torch.empty((sum(recv_splits),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_to_all_single(out, x.contiguous(), recv_splits, send_splits, group=self.group)
        return out

    def owned_mask(self, keys: torch.Tensor) -> torch.Tensor:
        return shard_of(self.local.hash_keys(keys), self.world) == self.rank

    # -------------------------------------------------------------- ops ----
    def set(self, keys: torch.Tensor, vals: torch.Tensor, lens: torch.Tensor, **kw) -> torch.Tensor:
        if self.world == 1:
            return self.local.set(keys, vals, lens, **kw)
        order, s, r = self._plan(keys)
        rk = self._route(keys[order], s, r)
        rv = self._route(vals[order], s, r)
        rl = self._route(lens[order], s, r)
        st = self.local.set(rk, rv, rl, **kw)
        back = self._route(st, r, s)
        out = torch.empty_like(back)
        out[order] = back
        return out

    def get(self, keys: torch.Tensor, **kw) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        if self.world == 1:
            return self.local.get(keys, **kw)
        order, s, r = self._plan(keys)
        rk = self._route(keys[order], s, r)
        st, vals, lens = self.local.get(rk, **kw)
        b_st, b_vals, b_lens = self._route(st, r, s), self._route(vals, r, s), self._route(lens, r, s)
        o_st, o_vals, o_lens = torch.empty_like(b_st), torch.empty_like(b_vals), torch.empty_like(b_lens)
        o_st[order] = b_st
        o_vals[order] = b_vals
        o_lens[order] = b_lens
        return o_st, o_vals, o_lens

    def signal_counts(self, local_counts: torch.Tensor) -> torch.Tensor:
        """Node-wide signal-group counters (C2): sum of per-shard counters."""
        if self.world == 1:
            return local_counts
        t = local_counts.clone()
        dist.all_reduce(t, group=self.group)
        return t


class GpuShard:
    """Local shard = an HBM arena driven by the gfx950 kernels."""

    def __init__(self, arena):
        self.arena = arena

    def hash_keys(self, keys: torch.Tensor) -> torch.Tensor:
        from .. import _native as N
        from ..ops.arena import _check, _stream
        out = torch.empty(keys.shape[0], dtype=torch.int64, device=keys.device)
        _check(N.hip_lib().spl_hash_keys(keys.data_ptr(), keys.shape[1], keys.shape[0], out.data_ptr(), _stream()),
               "hash_keys")
        return out

    def set(self, keys, vals, lens, **kw):
        return self.arena.set(keys, vals, lens, **kw)

    def get(self, keys, **kw):
        return self.arena.get(keys, **kw)


class HostShard:
    """Local shard = a host (shm) store; CPU tensors; used for gloo tests."""

    def __init__(self, store):
        from .. import _native as N
        self.store = store
        self._L = N.core_lib()

    def hash_keys(self, keys: torch.Tensor) -> torch.Tensor:
        k = keys.cpu().numpy()
        hs = [self._L.spl_hash_key(bytes(row).split(b"\0", 1)[0]) for row in k]
        return torch.tensor([h - (1 << 64) if h >= (1 << 63) else h for h in hs], dtype=torch.int64)

    def set(self, keys, vals, lens, **kw):
        k, v, ln = keys.numpy(), vals.numpy(), lens.numpy()
        st = []
        for i in range(k.shape[0]):
            key = bytes(k[i]).split(b"\0", 1)[0]
            rc = self._L.spl_set(self.store.handle, key, bytes(v[i, : ln[i]]), int(ln[i]))
            st.append(0 if rc == 0 else -11)
        return torch.tensor(st, dtype=torch.int32)

    def get(self, keys, **kw):
        k = keys.numpy()
        width = (self.store.max_val + 15) // 16 * 16
        out = torch.zeros((k.shape[0], width), dtype=torch.uint8)
        lens = torch.zeros(k.shape[0], dtype=torch.int32)
        st = torch.zeros(k.shape[0], dtype=torch.int32)
        for i in range(k.shape[0]):
            v = self.store.get(bytes(k[i]).split(b"\0", 1)[0])
            if v is None:
                st[i] = -2
            else:
                out[i, : len(v)] = torch.frombuffer(bytearray(v), dtype=torch.uint8)
                lens[i] = len(v)
        return st, out, lens

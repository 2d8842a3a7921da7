"""libsplinter_amd — MI355X-native shared-memory KV + vector substrate.

A from-scratch rebuild of splinterhq/libsplinter's capabilities:
  * ``Store``           — reference-compatible store (POSIX shm / file / HBM), format v4
  * ``ops.arena``       — batched gfx950 kernels over HBM arenas (set/get/intop/labels/scan)
  * ``ops.search``      — fused cosine/euclidean top-k vector search
  * ``models.nomic``    — Nomic-BERT embedder on hand-written CDNA4 kernels
  * ``parallel``        — hash-sharded arenas over RCCL/xGMI (one process per GPU)
"""
from .store import Store, SplinterError, SplinterBusy, hash_key, now, unlink  # noqa: F401

__version__ = "0.1.0"

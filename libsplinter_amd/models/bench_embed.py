"""Embed phase of bench.py: random-init Nomic-BERT (full 12-layer nomic-embed-text-v1.5
geometry) over a batch of synthetic documents, vectors written into the slots of an
embedding-enabled HBM arena by the fused pooling kernel (BASELINE config #3)."""
from __future__ import annotations

import os

import numpy as np
import torch

from ..ops.arena import HbmArena, format_keys, format_values
from ..parallel.sharded import GpuShard
from .nomic import Batch, NomicConfig, NomicEncoder, NomicWeights, random_weights


class EmbedPhase:
    def __init__(self, kv_arena=None, batch: int = 512, seq: int = 512, rank: int = 0, layers: int = 12,
                 vary: bool = False):
        self.cfg = NomicConfig(layers=layers)
        w = NomicWeights.from_numpy(self.cfg, random_weights(self.cfg, seed=rank))
        rng = np.random.default_rng(100 + rank)
        lens = rng.integers(seq // 2, seq + 1, size=batch) if vary else np.full(batch, seq)
        seqs = [rng.integers(1000, self.cfg.vocab, size=int(n)).tolist() for n in lens]
        self.batch = Batch(seqs)
        self.enc = NomicEncoder(w, max_tokens=self.batch.T_pad)
        self.docs_per_step = batch
        self.tokens_per_step = int(self.batch.T)
        # documents live in their own embedding-stride arena (128-B KV slots carry no vectors)
        self.arena = HbmArena.create(f"docs{os.getpid()}r{rank}", slots=max(2 * batch, 1024), max_val=256,
                                     embeddings=True)
        K = format_keys(batch, "doc", 9, 16)
        V, L = format_values(batch, 1, 64, 256)
        st = self.arena.set(K, V, L)
        st_f, idx = self.arena.meta("find", K)
        torch.cuda.synchronize()
        assert int((st != 0).sum()) == 0 and int((st_f != 0).sum()) == 0
        self.keys = K
        self.slots = idx
        self.hashes = GpuShard(self.arena).hash_keys(K)
        self.out = torch.empty((batch, 768), dtype=torch.float32, device="cuda")
        self.flops_per_step = self.enc.flops(self.batch)

    def run(self):
        return self.enc.embed(self.batch, arena=self.arena, slots=self.slots, hashes=self.hashes, out=self.out)

    def close(self):
        self.arena.close()

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
                 vary: bool = False, doc_arena=None):
        self.cfg = NomicConfig(layers=layers)
        w = NomicWeights.from_numpy(self.cfg, random_weights(self.cfg, seed=rank))
        rng = np.random.default_rng(100 + rank)
        lens = rng.integers(seq // 2, seq + 1, size=batch) if vary else np.full(batch, seq)
        seqs = [rng.integers(1000, self.cfg.vocab, size=int(n)).tolist() for n in lens]
        self.batch = Batch(seqs)
        self.enc = NomicEncoder(w, max_tokens=self.batch.T_pad)
        self.docs_per_step = batch
        self.tokens_per_step = int(self.batch.T)
        # documents live in an embedding-stride arena (128-B KV slots carry no vectors): the caller's
        # (bench.py: the 25M-key search arena, so the slot lookup and the pooled writes hit a large
        # arena) or a small one of their own
        self.own = doc_arena is None
        self.arena = doc_arena if doc_arena is not None else HbmArena.create(
            f"docs{os.getpid()}r{rank}", slots=max(2 * batch, 1024), max_val=256, embeddings=True)
        K = format_keys(batch, "doc", 9, 16)
        V, L = format_values(batch, 1, 32, min(256, self.arena.max_val))
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
        if self.own:
            self.arena.close()


class EmbedE2E:
    """End-to-end embedding of the splinference path for one batch of pending documents,
    measured separately from the kernel-only EmbedPhase (bench.py reports both):

      fetch     the documents' text from their slots (batched arena get, device -> host)
      tokenize  native WordPiece on the host (csrc/core/wordpiece.cpp, threaded), varlen docs
      pack      the varlen Batch (ids / offsets / q-blocks to the device)
      find      slot lookup and key hashes (batched meta kernel)
      embed     encoder forward + mean pool written into the slots under the seqlock, with the
                reference's "slot still holds this key" check (k_pool status)
      label     the pending label cleared; the simulated producer then re-arms it for the next
                step (one more meta kernel, kept inside the timed step)

    Reference loop: splinference.cpp:236-300 (tokenize, llama_decode, set_embedding, +2 epoch
    check, label updates)."""

    WAITING = 1 << 6

    def __init__(self, enc: NomicEncoder, batch: int = 64, seq: int = 512, rank: int = 0):
        from ..models.tokenizer import WordPieceTokenizer, synthetic_vocab
        from ..ops.arena import pack_values
        self.enc = enc
        cfg = enc.cfg
        vocab = synthetic_vocab(cfg.vocab)
        self.tok = WordPieceTokenizer(vocab)
        words = [t[1:] for t in vocab if t.startswith("▁") and len(t) > 2]
        rng = np.random.default_rng(200 + rank)
        texts = []
        for _ in range(2 * batch):  # varlen documents of about seq/2 .. seq-2 word tokens
            n = int(rng.integers(seq // 2, seq - 2))
            texts.append(" ".join(words[int(i)] for i in rng.integers(0, len(words), size=n)))
        self.max_tokens = seq
        self.arena = HbmArena.create(f"e2e{os.getpid()}r{rank}", slots=max(4 * batch, 1024), max_val=4096,
                                     embeddings=True)
        # two disjoint sets of pending documents, taken in turn: a batch's fetch overlaps the encoder
        # pass of the previous batch, as in the daemon, where consecutive batches hold different keys
        all_keys = format_keys(2 * batch, "txt", 9, 16)
        V, L = pack_values(texts, 4096)
        st = self.arena.set(all_keys, V, L)
        st_l, _ = self.arena.meta("set_label", all_keys, torch.full((2 * batch,), self.WAITING, dtype=torch.int64,
                                                                    device="cuda"))
        self.key_sets = [all_keys[:batch], all_keys[batch:]]
        self.turn = 0
        torch.cuda.synchronize()
        assert int((st != 0).sum()) == 0 and int((st_l != 0).sum()) == 0
        self.mask = torch.full((batch,), self.WAITING, dtype=torch.int64, device="cuda")
        self.shard = GpuShard(self.arena)
        self.docs = batch
        self.host_rows = torch.empty((batch, 4096), dtype=torch.uint8, pin_memory=True)
        self.host_lens = torch.empty(batch, dtype=torch.int32, pin_memory=True)
        self.out = torch.empty((batch, 768), dtype=torch.float32, device="cuda")
        self.tokens = 0
        self.failures = 0
        self.pending = None  # (keys, Batch) of the next batch, prepared while the previous one ran
        # where the host's time per batch goes (bench JSON): waiting for the GPU (the previous
        # batch's encoder, ahead of the next fetch on the stream) vs tokenizing + packing.  Wait ~ 0
        # means the pipeline is bound by the host's tokenizer, not by the encoder
        self.t_wait = self.t_tok = 0.0
        self.calls = 0

    def _fetch(self):
        """Enqueue the next key set's text fetch (batched get + copy to pinned host memory) on the
        current stream; returns the keys and an event marking the copy."""
        keys = self.key_sets[self.turn]
        self.turn ^= 1
        st, rows, lens = self.arena.get(keys)
        self.host_rows.copy_(rows, non_blocking=True)
        self.host_lens.copy_(lens, non_blocking=True)
        return keys, torch.cuda.current_stream().record_event()

    def _prepare(self, fetched):
        """Host side of a batch: wait for its fetch only, tokenize, pack (one async upload)."""
        import time
        keys, ev = fetched
        t0 = time.perf_counter()
        ev.synchronize()
        t1 = time.perf_counter()
        hr, hl = self.host_rows.numpy(), self.host_lens.numpy()
        texts = [hr[i, : hl[i]].tobytes() for i in range(self.docs)]
        ids, offs, _ = self.tok.encode_batch(texts, self.max_tokens)
        b = Batch([ids[offs[i]: offs[i + 1]] for i in range(self.docs)])
        self.t_wait += t1 - t0
        self.t_tok += time.perf_counter() - t1
        self.calls += 1
        return keys, b

    def run(self):
        # Software pipeline with one batch of lookahead, on ONE stream (a second stream claims
        # another hardware queue, and the queue scheduler then time-slices the encoder's queue:
        # profiles/r2_hw_queues.md): the next batch's fetch is enqueued AHEAD of this batch's
        # encoder, so the host waits only for that fetch and tokenizes / packs the next batch
        # while this one's encoder runs.  The daemon does the same (daemons/splinference.py).
        if self.pending is None:  # pipeline prologue (the warm-up call)
            self.pending = self._prepare(self._fetch())
        self.keys, b = self.pending
        nxt = self._fetch()
        self.tokens = int(b.T)
        st_f, slots = self.arena.meta("find", self.keys)
        hashes = self.shard.hash_keys(self.keys)
        _, status = self.enc.embed(b, arena=self.arena, slots=slots, hashes=hashes, out=self.out)
        self.arena.meta("unset_label", self.keys, self.mask)
        self.arena.meta("set_label", self.keys, self.mask)  # the producer re-arms the documents
        self.pending = self._prepare(nxt)
        return status

    def close(self):
        self.arena.close()

#!/usr/bin/env python3
"""splinference — the embedding sidecar, rebuilt on the gfx950 Nomic encoder.

Contract kept from the reference daemon (/root/reference/splinference.cpp,
SURVEY §2.7):
  argv   [--backfill-text-keys] [--oneshot] [--vector-training] <store> <gguf> <group>
  labels 0x1 "embed me" -> bound to <group> (:404); WAITING 0x40 cleared after
         the vector lands (:545); CONTEXT_EXCEEDED 0x80 on oversize input
         (:142-194: zero vector + diagnostic value + label + bump)
  ceiling 0.9 * n_ctx tokens (:228-233)
  write-once --vector-training: never overwrite a non-zero vector (:263-269)
  stale race: the post-write epoch must be pre + 2 (:282-286)
  after a batch: ctime backfill (:530-537), pulse "__lane_dw_2" (:547)
  Logic-shard bid 0x5F10 (WILLNEED prio 40 live, SEQUENTIAL prio 20 backfill)
Differences (the point of the rebuild): every pending key is tokenised in
one native batch and embedded in length-sorted varlen batches on the GPU
(the reference runs one llama_decode per key); for hbm: stores the pooled
vectors are written straight into the arena slots by the pooling kernel.
Extra flags: --random-init (no GGUF: random weights + synthetic vocab),
--batch-tokens, --poll-ms, --normalize, --layers (random-init only).

Node stores ("node:NAME", one arena per GPU): one daemon per GPU (--rank, default $RANK), each
embedding the pending keys of ITS shard on its own GPU -- data parallel, owner computes: vectors
are pooled into local slots and no vector crosses xGMI.  Every daemon watches the node's summed
signal counter (a pulse on any shard wakes all of them; each finds work only in its own shard).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import sys
import time
from typing import Dict, List, Optional, Tuple

import numpy as np

EMBED_LABEL = 0x1
WAITING_LABEL = 0x40
CONTEXT_EXCEEDED_LABEL = 0x80
SHARD_ID = 0x5F10
SHARD_DUR_LIVE, SHARD_DUR_BACKFILL = 1 << 30, 1 << 36
SHARD_PRIO_LIVE, SHARD_PRIO_BACKFILL = 40, 20
LANE_KEY = "__lane_dw_2"
POSIX_MADV_WILLNEED = 3
POSIX_MADV_SEQUENTIAL = 2


def log(*a):
    print("[splinference]", *a, file=sys.stderr, flush=True)


class Splinference:
    def __init__(self, store, encoder, tokenizer, group: int, vector_training: bool = False,
                 batch_tokens: int = 1 << 16, normalize: bool = False, rank: Optional[int] = None,
                 hold_ring: Optional[bool] = None):
        import torch  # noqa: F401
        from ..store import SLOT_VARTEXT
        # `node`: the store clients use (signals, label map, bids, lane pulses); `store`: the one
        # whose keys this daemon embeds -- the whole store, or this rank's shard of a node store
        self.node = store
        self.rank = 0
        if getattr(store, "backend", None) == "node":
            self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
            if not 0 <= self.rank < store.nshards:
                raise ValueError(f"rank {self.rank} outside the node's {store.nshards} shards")
            store = store.shard(self.rank)
        self.store = store
        # hold_ring (SPLINTER_DAEMON_RING_HOLD=1): the store's per-call ring worker stays off the GPU
        # while a pass embeds on it (store.ring_hold(store)): a resident worker costs the encoder
        # queue time-slices (+29 %, profiles/r4z); clients' per-call ops wait for the pass instead
        self.hold_ring = (os.environ.get("SPLINTER_DAEMON_RING_HOLD", "0") == "1") if hold_ring is None else hold_ring
        self.enc = encoder
        self.tok = tokenizer
        self.group = group
        self.vector_training = vector_training
        self.batch_tokens = batch_tokens
        self.normalize = normalize
        self.ceiling = int(0.9 * encoder.cfg.n_ctx)
        self.processed: Dict[str, int] = {}
        self.vartext = SLOT_VARTEXT
        self.stats = {"embedded": 0, "exceeded": 0, "stale": 0, "skipped_trained": 0, "batches": 0}
        self.node.watch_label(EMBED_LABEL, group)
        try:
            self.node.shard_claim(SHARD_ID, 1, SHARD_PRIO_LIVE, SHARD_DUR_LIVE)
        except Exception:
            pass
        # hbm: stores take the batched device path: one kernel per step for a whole batch of keys
        # (epochs, text reads, slot lookup, vectors pooled into the slots under the seqlock, label
        # updates) instead of several per-call ring round trips per key
        self.arena = None
        if getattr(store, "backend", None) == "hbm":
            from ..ops.arena import HbmArena
            from ..parallel.sharded import GpuShard
            self.arena = HbmArena(store)
            self.shard = GpuShard(self.arena)

    # ---------------------------------------------------------------- util --
    def _zero_vec(self, key: str) -> bool:
        v = self.store.get_embedding(key)
        return v is None or float(np.linalg.norm(v)) < 1e-6

    def cold_start(self):
        """Baseline keys that already hold vectors so they are not re-embedded."""
        for key in self.store.list():
            if not self._zero_vec(key):
                self.processed[key] = self.store.epoch(key)

    def pending(self) -> List[str]:
        if self.arena is not None:
            return self._pending_hbm()
        out = []
        for key in self.store.list():
            e = self.store.epoch(key)
            if e & 1:
                continue
            if e > self.processed.get(key, -1):
                out.append(key)
        return out

    def backfill_keys(self) -> List[str]:
        out = []
        for key in self.store.list():
            snap = self.store.snapshot(key)
            if snap and (snap["type_flag"] & self.vartext) and self._zero_vec(key):
                out.append(key)
        return out

    # ------------------------------------------------------- batched (hbm:) --
    def _keys_u8(self, keys: List[str]):
        from ..ops.arena import pack_keys
        return pack_keys(keys, 64)

    def _pending_hbm(self) -> List[str]:
        names = [k for k in self.store.list()]
        if not names:
            return []
        _, ep = self.arena.meta("epoch", self._keys_u8(names))
        ep = ep.cpu().numpy()
        return [k for k, e in zip(names, ep) if not (e & 1) and int(e) > self.processed.get(k, -1)]

    def _read_hbm(self, keys: List[str]) -> Tuple[List[str], List[bytes], List[int]]:
        """Seqlock-consistent batch read: epochs, values, epochs again (a key whose epoch moved or
        is odd is skipped this round, as the reference's per-key check)."""
        K = self._keys_u8(keys)
        _, e0 = self.arena.meta("epoch", K)
        st, rows, lens = self.arena.get(K)
        _, e1 = self.arena.meta("epoch", K)
        e0, e1, st, lens = e0.cpu().numpy(), e1.cpu().numpy(), st.cpu().numpy(), lens.cpu().numpy()
        rows = rows.cpu().numpy()
        trained = None
        if self.vector_training:
            _, vecs = self.arena.get_embeddings(K)
            trained = (vecs.norm(dim=1) > 1e-6).cpu().numpy()
        ks, texts, eps = [], [], []
        for i, k in enumerate(keys):
            if st[i] != 0 or (e0[i] & 1) or e0[i] != e1[i]:
                continue
            if trained is not None and trained[i]:
                self.stats["skipped_trained"] += 1
                self.processed[k] = int(e0[i])
                continue
            ks.append(k)
            texts.append(rows[i, : lens[i]].tobytes().split(b"\0", 1)[0])
            eps.append(int(e0[i]))
        return ks, texts, eps

    def _launch_hbm(self, idx: List[int], ks, ids, offs):
        """Enqueue one batch: encoder + mean pool written straight into the keys' slots under the
        seqlock (k_pool, which also checks the slot still holds the key) and the post-write epochs
        -- no host sync; _finish_hbm reads the results back."""
        from ..models.nomic import Batch
        b = Batch([ids[offs[i]: offs[i + 1]] for i in idx])
        K = self._keys_u8([ks[i] for i in idx])
        _, slots = self.arena.meta("find", K)
        hashes = self.shard.hash_keys(K)
        _, status = self.enc.embed(b, normalize=self.normalize, arena=self.arena, slots=slots, hashes=hashes)
        _, post = self.arena.meta("epoch", K)
        return idx, K, status, post

    def _finish_hbm(self, rec, ks, eps) -> int:
        """The +2 epoch check and the WAITING label cleared for the keys that passed it (batched)."""
        import torch
        idx, K, status, post = rec
        status, post = status.cpu().numpy(), post.cpu().numpy()
        self.stats["batches"] += 1
        ok_rows = []
        for j, i in enumerate(idx):
            if status[j] != 0 or int(post[j]) != eps[i] + 2:  # stale-race detection (reference :282-286)
                self.stats["stale"] += 1
                continue
            self.processed[ks[i]] = int(post[j])
            ok_rows.append(j)
        if ok_rows:
            sel = torch.tensor(ok_rows, device=K.device)
            self.arena.meta("unset_label", K[sel],
                            torch.full((len(ok_rows),), WAITING_LABEL, dtype=torch.int64, device=K.device))
        return len(ok_rows)

    # ------------------------------------------------------------ embedding --
    def _read(self, keys: List[str]) -> Tuple[List[str], List[bytes], List[int]]:
        if self.arena is not None:
            return self._read_hbm(keys)
        ks, texts, eps = [], [], []
        for k in keys:
            e1 = self.store.epoch(k)
            if e1 & 1:
                continue
            v = self.store.get(k)
            if v is None or self.store.epoch(k) != e1:
                continue
            if self.vector_training and not self._zero_vec(k):
                self.stats["skipped_trained"] += 1
                self.processed[k] = e1
                continue
            ks.append(k)
            texts.append(v.split(b"\0", 1)[0])
            eps.append(e1)
        return ks, texts, eps

    def _exceeded(self, key: str, ntok: int):
        """Reference policy for oversize inputs (splinference.cpp:142-194)."""
        msg = (f"CONTEXT_EXCEEDED: {ntok} tokens > limit {self.ceiling} (n_ctx {self.enc.cfg.n_ctx}); "
               f"host={socket.gethostname()} time={int(time.time())}").encode()[: self.store.max_val]
        try:
            self.store.set_embedding(key, np.zeros(768, np.float32))
            self.store.set(key, msg)
            self.store.set_label(key, CONTEXT_EXCEEDED_LABEL)
            self.store.bump(key)
        except Exception as ex:  # noqa: BLE001
            log("context-exceeded marker failed for", key, ex)
        self.processed[key] = self.store.epoch(key)
        self.stats["exceeded"] += 1

    def process(self, keys: List[str]) -> int:
        import torch
        from ..models.nomic import Batch
        if not keys:
            return 0
        t_start = time.time()
        tick0 = self._ticks()
        ks, texts, eps = self._read(keys)
        if not ks:
            return 0
        ids, offs, full = self.tok.encode_batch(texts, self.ceiling + 1)
        good = []
        for i, k in enumerate(ks):
            if full[i] > self.ceiling:
                self._exceeded(k, int(full[i]))
            else:
                good.append(i)
        order = sorted(good, key=lambda i: offs[i + 1] - offs[i])
        if self.hold_ring and self.arena is not None:  # the HBM batches make no per-call op
            from ..store import ring_hold
            with ring_hold(self.store):
                done = self._process_batches(order, ks, ids, offs, eps)
        else:
            done = self._process_batches(order, ks, ids, offs, eps)
        # ctime backfill: wall time minus processing ticks (reference :530-537)
        now_s, dt = int(time.time()), self._ticks() - tick0
        if self.arena is not None and good:
            K = self._keys_u8([ks[i] for i in good])
            self.arena.meta("ctime", K, torch.full((len(good),), now_s, dtype=torch.int64, device=K.device))
        else:
            for i in good:
                try:
                    self.store.set_time(ks[i], 0, now_s, 0)
                except Exception:  # noqa: BLE001
                    pass
        self.node.pulse(LANE_KEY)
        self.stats["embedded"] += done
        log(f"embedded {done}/{len(ks)} keys in {time.time() - t_start:.3f}s (ticks {dt})")
        return done

    def _process_batches(self, order, ks, ids, offs, eps) -> int:
        done = 0
        batch: List[int] = []
        ntok = 0
        inflight = None  # hbm: one batch of lookahead -- batch j+1 is packed and enqueued before
        for i in order + [None]:  # batch j's results are read back, so the GPU never waits on the host
            n = 0 if i is None else int(offs[i + 1] - offs[i])
            if batch and (i is None or ntok + n > self.batch_tokens):
                if self.arena is not None:
                    rec = self._launch_hbm(batch, ks, ids, offs)
                    if inflight is not None:
                        done += self._finish_hbm(inflight, ks, eps)
                    inflight = rec
                else:
                    done += self._run(batch, ks, eps, ids, offs)
                batch, ntok = [], 0
            if i is not None:
                batch.append(i)
                ntok += n
        if inflight is not None:
            done += self._finish_hbm(inflight, ks, eps)
        return done

    @staticmethod
    def _ticks():
        from ..store import now
        return now()

    def _run(self, idx: List[int], ks, eps, ids, offs) -> int:
        if self.arena is not None:
            return self._finish_hbm(self._launch_hbm(idx, ks, ids, offs), ks, eps)
        import torch
        from ..models.nomic import Batch
        seqs = [ids[offs[i]: offs[i + 1]] for i in idx]
        b = Batch(seqs)
        vec = self.enc.embed(b, normalize=self.normalize)
        host = vec.float().cpu().numpy()
        self.stats["batches"] += 1
        ok = 0
        for j, i in enumerate(idx):
            k = ks[i]
            if self.store.epoch(k) != eps[i]:
                self.stats["stale"] += 1  # text changed while we embedded: retry next round
                continue
            try:
                self.store.set_embedding(k, host[j])
            except Exception:  # noqa: BLE001
                self.stats["stale"] += 1
                continue
            post = self.store.epoch(k)
            if post != eps[i] + 2:  # stale-race detection (reference :282-286)
                self.stats["stale"] += 1
                continue
            self.processed[k] = post
            try:
                self.store.unset_label(k, WAITING_LABEL)
            except Exception:  # noqa: BLE001
                pass
            ok += 1
        return ok

    # ----------------------------------------------------------------- loop --
    def run(self, oneshot: bool = False, backfill: bool = False, poll_ms: int = 10, stop=lambda: False):
        self.cold_start()
        if backfill:
            try:
                self.node.shard_rebid(SHARD_ID, 2, SHARD_PRIO_BACKFILL, SHARD_DUR_BACKFILL)
            except Exception:  # noqa: BLE001
                pass
            self.process(self.backfill_keys())
        last = -1
        while not stop():
            sig = self.node.signal_count(self.group)
            if sig != last or oneshot:
                last = sig
                try:
                    self.node.shard_rebid(SHARD_ID, 1, SHARD_PRIO_LIVE, SHARD_DUR_LIVE)
                    self.node.madvise(SHARD_ID, POSIX_MADV_WILLNEED, 0)
                except Exception:  # noqa: BLE001
                    pass  # not sovereign: defer (non-blocking bid, as the reference)
                self.process(self.pending())
            if oneshot:
                break
            time.sleep(poll_ms / 1000.0)
        try:
            self.node.shard_release(SHARD_ID)
        except Exception:  # noqa: BLE001
            pass


def build_encoder(gguf: Optional[str], random_init: bool, layers: int = 12, max_tokens: int = 1 << 16):
    from ..models.gguf import GGUFFile
    from ..models.nomic import NomicConfig, NomicEncoder, NomicWeights, random_weights
    from ..models.tokenizer import WordPieceTokenizer, synthetic_vocab
    if random_init or not gguf or not os.path.exists(gguf):
        if not random_init:
            raise FileNotFoundError(gguf)
        cfg = NomicConfig(layers=layers)
        w = NomicWeights.from_numpy(cfg, random_weights(cfg, seed=0))
        tok = WordPieceTokenizer(synthetic_vocab(cfg.vocab))
    else:
        g = GGUFFile(gguf)
        if g.arch() not in ("nomic-bert", "bert", "nomic-bert-moe"):
            log(f"warning: GGUF architecture {g.arch()!r} is not nomic-bert")
        cfg = NomicConfig.from_gguf(g)
        w = NomicWeights.from_gguf(g, cfg)
        tok = WordPieceTokenizer.from_gguf(g)
    return NomicEncoder(w, max_tokens=max_tokens), tok


def main(argv=None):
    ap = argparse.ArgumentParser(prog="splinference")
    ap.add_argument("--backfill-text-keys", action="store_true")
    ap.add_argument("--oneshot", action="store_true")
    ap.add_argument("--vector-training", action="store_true")
    ap.add_argument("--random-init", action="store_true")
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--batch-tokens", type=int, default=1 << 16)
    ap.add_argument("--poll-ms", type=int, default=10)
    ap.add_argument("--normalize", action="store_true")
    ap.add_argument("--rank", type=int, default=None,
                    help="node stores: the shard this daemon embeds (default $RANK); runs on GPU rank %% devices")
    ap.add_argument("bus")
    ap.add_argument("gguf")
    ap.add_argument("group", type=int)
    a = ap.parse_args(argv)
    if not 0 <= a.group < 64:
        ap.error("group must be 0..63")
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import torch
    from libsplinter_amd.store import Store
    if a.bus.startswith("node:"):
        rank = int(os.environ.get("RANK", "0")) if a.rank is None else a.rank
        n = torch.cuda.device_count()
        if n:
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % n)
    store = Store.open(a.bus)
    if not store.embeddings:
        log("store has no embedding stride (128-B slots): recreate it with embeddings")
        return 2
    enc, tok = build_encoder(a.gguf, a.random_init, a.layers, a.batch_tokens + 4096)
    d = Splinference(store, enc, tok, a.group, a.vector_training, a.batch_tokens, a.normalize, rank=a.rank)
    stop = {"v": False}
    signal.signal(signal.SIGINT, lambda *_: stop.__setitem__("v", True))
    signal.signal(signal.SIGTERM, lambda *_: stop.__setitem__("v", True))
    log(f"serving {a.bus} group {a.group} (ceiling {d.ceiling} tokens)" +
        (f", shard {d.rank}/{store.nshards}" if store.backend == "node" else ""))
    d.run(oneshot=a.oneshot, backfill=a.backfill_text_keys, poll_ms=a.poll_ms, stop=lambda: stop["v"])
    log("stats", d.stats)
    store.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())

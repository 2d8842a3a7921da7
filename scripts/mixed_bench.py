"""Mixed embed + insert + query workload (BASELINE config #5, one GPU's shard).

python scripts/mixed_bench.py [--slots 8000000] [--docs 64] [--seq 512] [--nq 256] [--steps 5]

Per step: insert `docs` new keys, embed their synthetic documents with the random-init
Nomic-BERT (12 layers, nomic-embed-text-v1.5 geometry) straight into their slots, then answer
`nq` queries (top-10 cosine) over the whole arena with the batched MFMA search.  The arena is
pre-filled with `slots * 0.9` random clustered vectors.  Prints one JSON line (synthetic data).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=8_000_000)
    ap.add_argument("--docs", type=int, default=64)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    import numpy as np
    import torch
    from libsplinter_amd.models.nomic import Batch, NomicConfig, NomicEncoder, NomicWeights, random_weights
    from libsplinter_amd.ops.arena import HbmArena, format_keys, format_values
    from libsplinter_amd.ops.search import VectorSearch
    from libsplinter_amd.parallel.sharded import GpuShard

    ar = HbmArena.create(f"mixed{os.getpid()}", slots=a.slots, max_val=64, embeddings=True)
    try:
        g = torch.Generator(device="cuda").manual_seed(0)
        centers = torch.randn(4096, 768, device="cuda", generator=g)
        n0 = int(a.slots * 0.9)
        em = ar.embedding_matrix()
        step = 1_000_000
        for b in range(0, n0, step):
            m = min(step, n0 - b)
            keys = format_keys(m, "base", 10, 16, first=b)
            vals, lens = format_values(m, 1, 16, 64, first=b)
            ar.set(keys, vals, lens)
        for b in range(0, a.slots, step):
            m = min(step, a.slots - b)
            lab = torch.randint(0, 4096, (m,), device="cuda", generator=g)
            em[b: b + m] = centers[lab] + 0.5 * torch.randn(m, 768, device="cuda", generator=g)
        ar.rebuild_vec16()  # raw writes through the view bypass the vector writers: recompute the bf16 copy
        torch.cuda.synchronize()

        cfg = NomicConfig()
        enc_w = NomicWeights.from_numpy(cfg, random_weights(cfg, seed=0))
        rng = np.random.default_rng(7)
        batch = Batch([rng.integers(1000, cfg.vocab, size=a.seq).tolist() for _ in range(a.docs)])
        enc = NomicEncoder(enc_w, max_tokens=batch.T_pad)
        shard = GpuShard(ar)
        vs = VectorSearch(ar)
        out = torch.empty((a.docs, 768), dtype=torch.float32, device="cuda")
        lab = torch.randint(0, 4096, (a.nq,), device="cuda", generator=g)
        q = centers[lab] + 0.5 * torch.randn(a.nq, 768, device="cuda", generator=g)
        stats = {}
        next_id = [0]

        def one_step():
            ids = next_id[0]
            next_id[0] += a.docs
            keys = format_keys(a.docs, "new", 10, 16, first=ids)
            vals, lens = format_values(a.docs, 1, 16, 64, first=ids)
            st = ar.set(keys, vals, lens)                      # insert
            _, idx = ar.meta("find", keys)
            enc.embed(batch, arena=ar, slots=idx, hashes=shard.hash_keys(keys), out=out)  # embed -> slots
            res = vs.search_batch(q, k=a.k, stats=stats)      # query the updated arena
            return st, res

        for _ in range(a.warmup):
            one_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            st, (idx, sim, _) = one_step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        # the last step's documents are findable: their own vectors are their nearest neighbours
        qd = out[:4]
        di, ds, _ = vs.search(qd, k=1)
        ok_insert = bool((ds[:, 0] > 0.999).all())
        ei, _, _ = vs.search(q[:16], k=a.k)
        print(json.dumps({"bench": "mixed_embed_insert_query", "slots": a.slots, "docs_per_step": a.docs,
                          "seq": a.seq, "queries_per_step": a.nq, "k": a.k, "ms_per_step": dt * 1e3,
                          "inserted_vectors_per_s": a.docs / dt, "qps": a.nq / dt,
                          "insert_status_ok": bool((st == 0).all()), "new_vectors_searchable": ok_insert,
                          "exact_match_16q": bool(torch.equal(idx[:16], ei)),
                          "data": "synthetic: random-init Nomic weights, random token documents, clustered base vectors"}),
              flush=True)
    finally:
        ar.close()


if __name__ == "__main__":
    main()

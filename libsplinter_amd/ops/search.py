"""Fused cosine/euclidean top-k vector search over an HBM arena (gfx950).

Semantics of the reference CLI `search` (/root/reference/splinter_cli_cmd_search.c:
43-72 scoring, :374-416 filter/sort/limit): cosine similarity and euclidean
distance for every embedded slot, optional label (bloom) filter, min-sim /
max-dist filters, ordered by similarity desc then distance asc.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import numpy as np
import torch

from .. import _native as N

MAX_Q, MAX_K = 16, 32
MMA_Q = 256          # queries per MFMA launch
TILE = 256           # slots per MFMA tile
MMA_GRID = 256       # persistent blocks of the MFMA pass (one per CU); candidate segments per query
# |cos_bf16 - cos| <= 2u + u^2 (u = 2^-8: both operands rounded once to bf16,
# Cauchy-Schwarz over the 768 products) plus fp32 accumulation / norm error
DELTA = 2.0 ** -7 + 2.0 ** -16 + 4e-4


def _lib():
    L = N.hip_lib()
    if not getattr(L, "_search_declared", False):
        P = ctypes.c_void_p
        L.spl_search.argtypes = [N.Arena, P, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                 ctypes.c_uint64, ctypes.c_int, P, P, P]
        L.spl_search.restype = ctypes.c_int
        L.spl_search_lists.argtypes = [ctypes.c_int]
        L.spl_search_lists.restype = ctypes.c_int
        L.spl_search_mma_pass.argtypes = [N.Arena, P, ctypes.c_int, ctypes.c_long, ctypes.c_long, ctypes.c_uint64,
                                          ctypes.c_int, P, P, P, P, ctypes.c_int, ctypes.c_int, P]
        L.spl_search_mma_pass.restype = ctypes.c_int
        L.spl_search_rescore.argtypes = [N.Arena, P, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                         ctypes.c_uint64, P, P, ctypes.c_int, ctypes.c_int, P, P]
        L.spl_search_rescore.restype = ctypes.c_int
        L._search_declared = True
    return L


class VectorSearch:
    """Reusable search context bound to one HbmArena."""

    def __init__(self, arena, grid: int = 512):
        if arena.stride != 3200:
            raise ValueError("arena has no embeddings")
        self.arena = arena
        self.grid = grid
        self.L = _lib()
        lists = self.L.spl_search_lists(grid)
        self.scratch = torch.empty(lists * MAX_Q * MAX_K * 4, dtype=torch.int32, device="cuda")
        self.result = torch.empty(MAX_Q * MAX_K * 4, dtype=torch.int32, device="cuda")

    def search(self, queries: torch.Tensor, k: int = 10, min_sim: float = -2.0, max_dist: float = 3.4e38,
               label_mask: int = 0) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """queries [nq, 768] -> (slot idx int64 [nq, k] (-1 = none), sim [nq, k], dist [nq, k])."""
        q = queries.to(device="cuda", dtype=torch.float32).reshape(-1, 768).contiguous()
        if not 1 <= k <= MAX_K:
            raise ValueError(f"k must be 1..{MAX_K}")
        outs_i, outs_s, outs_d = [], [], []
        for b in range(0, q.shape[0], MAX_Q):
            qq = q[b: b + MAX_Q]
            nq = qq.shape[0]
            rc = self.L.spl_search(self.arena.desc, qq.data_ptr(), nq, k, float(min_sim), float(max_dist),
                                   label_mask, self.grid, self.scratch.data_ptr(), self.result.data_ptr(),
                                   torch.cuda.current_stream().cuda_stream)
            if rc != 0:
                raise RuntimeError(f"spl_search failed ({rc})")
            r = self.result[: nq * k * 4].view(nq, k, 4)
            idx = r[..., 2].to(torch.int64) & 0xFFFFFFFF
            idx = torch.where(idx == 0xFFFFFFFF, torch.full_like(idx, -1), idx)
            outs_i.append(idx)
            outs_s.append(r[..., 0].view(torch.float32).clone())
            outs_d.append(r[..., 1].view(torch.float32).clone())
        return torch.cat(outs_i), torch.cat(outs_s), torch.cat(outs_d)

    def search_batch(self, queries: torch.Tensor, k: int = 10, min_sim: float = -2.0, max_dist: float = 3.4e38,
                     label_mask: int = 0, capb: int = 64, sample: Optional[int] = None, stats: Optional[dict] = None
                     ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Many-query search on the matrix cores; same results as `search` (exact fp32 ranking).

        Per launch of up to 512 queries: a bf16 MFMA pass over a slot sample gives a per-query
        threshold (k-th largest per-tile max - 2*DELTA), a bf16 MFMA pass over the arena emits
        candidates above it, and a fp32 re-score with the exact kernel's arithmetic ranks them.
        Each of the MMA_GRID blocks keeps up to `capb` candidates per query; a query whose
        segment overflows anywhere is redone with the exact kernel.
        """
        q = queries.to(device="cuda", dtype=torch.float32).reshape(-1, 768).contiguous()
        slots = self.arena.slots
        if not 1 <= k <= MAX_K:
            raise ValueError(f"k must be 1..{MAX_K}")
        if q.shape[0] < 32 or slots < TILE:
            return self.search(q, k, min_sim, max_dist, label_mask)
        st = torch.cuda.current_stream().cuda_stream
        if sample is None:
            sample = min(slots, max(TILE * 4096, slots // 16))
        sample = max(TILE, sample // TILE * TILE)
        bounded = max_dist < 3.0e38
        outs_i, outs_s, outs_d = [], [], []
        nover = ncand = 0
        for b in range(0, q.shape[0], MMA_Q):
            qq = q[b: b + MMA_Q]
            n = qq.shape[0]
            qpad = MMA_Q
            qb = torch.zeros(qpad, 768, dtype=torch.bfloat16, device="cuda")
            qb[:n] = (qq / qq.norm(dim=1, keepdim=True).clamp_min(1e-30)).to(torch.bfloat16)
            # fragment order [q/16][24 steps][4 kq][16 r][8]: lane 16*kq + r of a wave load
            qf = qb.view(qpad // 16, 16, 24, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
            floor = torch.full((n,), float(min_sim) - DELTA, device="cuda")
            if bounded:
                thr = floor
            else:
                bmax = torch.empty(sample // TILE, n, dtype=torch.float32, device="cuda")
                rc = self.L.spl_search_mma_pass(self.arena.desc, qf.data_ptr(), n, 0, sample, label_mask, 0, None,
                                                bmax.data_ptr(), None, None, 0, MMA_GRID, st)
                if rc != 0:
                    raise RuntimeError(f"spl_search_mma_pass(bmax) failed ({rc})")
                kk = min(k, bmax.shape[0])
                kth = bmax.topk(kk, dim=0).values[-1]
                if kk < k:
                    kth = torch.full_like(kth, -3.0e38)
                thr = torch.maximum(kth - 2 * DELTA, floor)
            cnt = torch.zeros(n, MMA_GRID, dtype=torch.int32, device="cuda")
            cand = torch.empty(n * MMA_GRID * capb, dtype=torch.int32, device="cuda")
            rc = self.L.spl_search_mma_pass(self.arena.desc, qf.data_ptr(), n, 0, slots, label_mask, 1,
                                            thr.data_ptr(), None, cnt.data_ptr(), cand.data_ptr(), capb, MMA_GRID, st)
            if rc != 0:
                raise RuntimeError(f"spl_search_mma_pass(cand) failed ({rc})")
            res = torch.empty(n * k * 4, dtype=torch.int32, device="cuda")
            rc = self.L.spl_search_rescore(self.arena.desc, qq.data_ptr(), n, k, float(min_sim), float(max_dist),
                                           label_mask, cnt.data_ptr(), cand.data_ptr(), MMA_GRID, capb,
                                           res.data_ptr(), st)
            if rc != 0:
                raise RuntimeError(f"spl_search_rescore failed ({rc})")
            r = res.view(n, k, 4)
            idx = r[..., 2].to(torch.int64) & 0xFFFFFFFF
            idx = torch.where(idx == 0xFFFFFFFF, torch.full_like(idx, -1), idx)
            sim = r[..., 0].view(torch.float32).clone()
            dist = r[..., 1].view(torch.float32).clone()
            over = torch.nonzero((cnt > capb).any(dim=1)).flatten()
            if over.numel():
                oi, osim, od = self.search(qq[over], k, min_sim, max_dist, label_mask)
                idx[over], sim[over], dist[over] = oi, osim, od
            if stats is not None:
                nover += int(over.numel())
                ncand += int(cnt.clamp_max(capb).sum())
            outs_i.append(idx)
            outs_s.append(sim)
            outs_d.append(dist)
        if stats is not None:
            stats.update(overflow=nover, candidates=ncand, sample=sample)
        return torch.cat(outs_i), torch.cat(outs_s), torch.cat(outs_d)

    def keys_of(self, idx: torch.Tensor) -> List[List[Optional[str]]]:
        """Map slot indices to key strings (one gather of the slot cores)."""
        flat = idx.reshape(-1)
        valid = flat >= 0
        out = [None] * flat.numel()
        if valid.any():
            sel = flat[valid].to(torch.int32).contiguous()
            core = torch.empty((sel.numel(), 128), dtype=torch.uint8, device="cuda")
            H = N.hip_lib()
            H.spl_arena_gather_slots(self.arena.desc, sel.data_ptr(), sel.numel(), core.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream)
            keys = core[:, 64:].cpu().numpy()
            pos = torch.nonzero(valid).flatten().tolist()
            for p, row in zip(pos, keys):
                out[p] = bytes(row).split(b"\0", 1)[0].decode("utf-8", "replace")
        k = idx.shape[-1]
        return [out[i: i + k] for i in range(0, len(out), k)]


def search_reference(matrix: np.ndarray, occupied: np.ndarray, q: np.ndarray, k: int,
                     min_sim: float = -2.0, max_dist: float = 3.4e38):
    """Scalar reference of the CLI search ranking (for tests)."""
    res = []
    qn = float(np.sqrt((q.astype(np.float64) ** 2).sum()))
    for i in np.nonzero(occupied)[0]:
        v = matrix[i].astype(np.float64)
        vn = float(np.sqrt((v ** 2).sum()))
        if vn < 1e-6:
            continue
        sim = float(v @ q) / (vn * qn)
        dist = float(np.sqrt(((v - q) ** 2).sum()))
        if sim < min_sim or dist > max_dist:
            continue
        res.append((-sim, dist, int(i)))
    res.sort()
    return [(i, -s, d) for s, d, i in res[:k]]

/* search_api.h — fused cosine/euclidean top-k over an HBM arena (gfx950). */
#ifndef SPLINTER_SEARCH_API_H
#define SPLINTER_SEARCH_API_H
#include <stdint.h>
#include "arena_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* number of per-wave candidate lists produced for a given grid */
int spl_search_lists(int grid);
/* queries [nq <= 16, 768] fp32, K <= 32; scratch: spl_search_lists(grid) * nq * K * 16 bytes;
 * result: [nq, K] x {float sim, float dist, uint32 slot, uint32 pad}, slot 0xffffffff = empty.
 * Ranking: similarity desc, then distance asc (reference cmd_search.c:412). */
int spl_search(spl_arena_t a, const float *queries, int nq, int K, float min_sim, float max_dist, uint64_t mask,
               int grid, void *scratch, void *result, hipStream_t stream);

/* Batched MFMA search (many queries).  qfrag: queries L2-normalised, bf16, zero-padded to 256
 * queries and permuted to fragment order [16 tiles][24 steps][64 lanes] x 16 B, where lane =
 * 16*kq + r holds query (16*tile + r), dims [32*step + 8*kq, +8).  Scores slots
 * [slot_begin, slot_end) (slot_begin a multiple of spl_search_mma_tile(), at least one tile).
 * mode 0: bmax[tile - slot_begin/256][nq] = max approximate cosine per 256-slot tile and query
 * (-FLT_MAX if no live slot); mode 1: `grid` blocks, each appends the live slots of its tiles
 * with approximate cosine >= thr[q] to its private segment cand[q][block][0..capb) and stores
 * the segment's count (may exceed capb: overflow) in cnt[q][block].  cnt must be zeroed first. */
int spl_search_mma_queries(void);
int spl_search_mma_tile(void);
int spl_search_mma_pass(spl_arena_t a, const void *qfrag, int nq, long slot_begin, long slot_end, uint64_t mask,
                        int mode, const float *thr, float *bmax, uint32_t *cnt, uint32_t *cand, int capb, int grid,
                        hipStream_t stream);
/* queries [nq <= 256, 768] fp32 (device) -> qfrag as spl_search_mma_pass takes it (normalised,
 * bf16, zero-padded to 256 queries, fragment order) */
int spl_search_qprep(const float *queries, int nq, void *qfrag, hipStream_t stream);
/* slot cores (128 B each) of n result entries (spl_search result layout) -> out_cores[n][128] */
int spl_search_cores(spl_arena_t a, const void *result, int n, void *out_cores, hipStream_t stream);
/* over[q] = 1 when cnt[q][0..nblk) has a segment count > capb (the query must be redone exactly) */
int spl_search_overflow(const uint32_t *cnt, int nq, int nblk, int capb, uint32_t *over, hipStream_t stream);
/* per-query candidate threshold from a bmax pass: max(k-th largest of bmax[tiles][nq] - delta2, floor) */
int spl_search_thr(const float *bmax, int tiles, int nq, int K, float delta2, float floor_v, float *thr,
                   hipStream_t stream);
// the same, and the k largest sampled tile maxima per query into topv [nq][K] (descending,
// -FLT_MAX past the sample): a node search merges them over its shards
int spl_search_thr_topk(const float* bmax, int tiles, int nq, int K, float delta2, float floor_v, float* thr,
                        float* topv, hipStream_t s);
/* Exact fp32 re-score of the candidate segments (queries [nq, 768] fp32, unnormalised) and top-K:
 * result layout and ranking as spl_search. */
int spl_search_rescore(spl_arena_t a, const float *queries, int nq, int K, float min_sim, float max_dist,
                       uint64_t mask, const uint32_t *cnt, const uint32_t *cand, int nblk, int capb, void *result,
                       hipStream_t stream);

/* Score every candidate slot against one query [768] fp32 (device pointers): out[slots] float2
 * {sim, dist}; {0, -1} = candidate without a vector, {NaN, NaN} = not a candidate / filtered out.
 * Candidates and filters as the reference CLI search (see search_kernels.hip). */
int spl_arena_score_all(spl_arena_t a, const float *query, float min_sim, float max_dist, uint64_t mask, void *out,
                        hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif

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

#ifdef __cplusplus
}
#endif
#endif

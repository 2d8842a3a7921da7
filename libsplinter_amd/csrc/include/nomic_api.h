/*
 * nomic_api.h — C launch API of the Nomic-BERT encoder kernels (gfx950).
 * All tensors are device pointers, bf16 stored as uint16.  Row counts that
 * feed nomic_gemm must be padded to a multiple of 128 in the A buffer.
 */
#ifndef SPLINTER_NOMIC_API_H
#define SPLINTER_NOMIC_API_H
#include <stdint.h>
#include "arena_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* GEMM epilogues */
#define NOMIC_EPI_STORE    0   /* out = bf16(acc)                                   */
#define NOMIC_EPI_RESIDUAL 1   /* out = bf16(acc + res)                             */
#define NOMIC_EPI_SWIGLU   2   /* W rows interleaved [up16|gate16] (pack_upgate): out = up*silu(gate) */
#define NOMIC_EPI_ROPE     3   /* qkv projection, W rows per head [d0-15|d32-47|d16-31|d48-63]
                                  (pack_qkv); NEOX RoPE on cols < rope_cols; out in natural order */
#define NOMIC_EPI_F32      4   /* out = acc as fp32                                 */
/* Post-LayerNorm folded into the GEMMs around it (nomic_gemm_ln).  A producer (o-proj / down)
 * writes the raw residual sum h and per-row partial statistics of h; the consumer combines them
 * into (mean, rstd) per row in its prologue, reads raw h against W' = W diag(g) and its
 * epilogue applies  y = rstd (acc - mean c1[n]) + c2[n]  (c1 = W' 1, c2 = W b), which equals
 * LN(h) W^T; a residual GEMM normalises its residual operand on the fly.                    */
#define NOMIC_EPI_ROPE_FOLD    5  /* ROPE with the LN fold applied first                    */
#define NOMIC_EPI_SWIGLU_FOLD  6  /* SWIGLU with the LN fold applied to up and gate         */
#define NOMIC_EPI_RES_STATS    7  /* out = bf16(acc + res); partial row stats of out         */
#define NOMIC_EPI_RES_LN_STATS 8  /* out = bf16(acc + LN(res)); partial row stats of out     */

int nomic_gemm(int mode, const void *A, long lda, const void *W, long ldw, long M, int N, int K,
               void *out, long ldo, const void *res, long ldr, const float *rope, const int32_t *pos,
               int rope_cols, hipStream_t stream);
/* nomic_gemm with the LN-fold operands: part_in [M][nparts] (mean, M2) 128-column partials of
 * A's rows (fold modes) or of res's rows (RES_LN_STATS), as a stats mode wrote them (nparts <= 8;
 * the kernel combines them per row, eps added to the variance); c1, c2 [N] fold vectors; ln_g,
 * ln_b [N] bf16 LayerNorm of res; part [M][N/128] partials written by the stats modes.        */
int nomic_gemm_ln(int mode, const void *A, long lda, const void *W, long ldw, long M, int N, int K, void *out,
                  long ldo, const void *res, long ldr, const float *rope, const int32_t *pos, int rope_cols,
                  const float *part_in, int nparts, float eps, const float *c1, const float *c2,
                  const void *ln_g, const void *ln_b, float *part, hipStream_t stream);
/* combine nparts (mean, M2) partials of 128 columns each into (mean, 1/sqrt(var + eps)) per row */
int nomic_row_stats(const float *part, int nparts, long M, float eps, float *st, hipStream_t stream);
/* GEMM kernel selection: 0 = auto, 512 = persistent 256x256 kernel with register
 * epilogue, 256 = launch-per-tile 256x256 phased kernel, 128 = 128x128 (where the
 * shape allows; otherwise the next one that does).  Returns the previous setting. */
int nomic_gemm_set_variant(int variant);

/* x[t] = LN(tok[ids[t]] + type_row) ; bf16 out [T, 768] */
int nomic_embed_ln(const int32_t *ids, long T, const void *tok_emb, const void *type_row,
                   const void *gamma, const void *beta, float eps, void *out, hipStream_t stream);
/* in-place (or out-of-place) LayerNorm over 768 columns, bf16 */
int nomic_layernorm(const void *x, long T, const void *gamma, const void *beta, float eps, void *out,
                    hipStream_t stream);
/* attention kernel: 2 = swapped-product 128-row kernel (default), 1 = 64-row kernel */
int nomic_attention_set_variant(int variant);
/* varlen non-causal attention; qkv [T, 3*H*64] (q|k|v), out [T, H*64].
 * qblocks: [nqb] int32 pairs (seq index, q start offset in the sequence) of
 * 128-row query blocks (q starts are multiples of 128)                    */
int nomic_attention(const void *qkv, void *out, const int32_t *cu_seqlens, const int32_t *qblocks,
                    int nqb, int heads, float scale, hipStream_t stream);
/* mean over each sequence's tokens -> fp32 [B, 768]; if slots != NULL also
 * write each vector into arena slot slots[b] (>= 0) under the seqlock, after
 * checking the slot still holds hashes[b]; status[b] gets 0 / -11 / -2.     */
int nomic_mean_pool(const void *x, const int32_t *cu_seqlens, int B, float *pooled, int normalize,
                    spl_arena_t arena, const int64_t *slots, const uint64_t *hashes, int32_t *status,
                    hipStream_t stream);
/* GGUF tensor dequantisation to bf16 (ggml type ids) */
int nomic_dequant(int ggml_type, const void *src, long nelems, void *dst_bf16, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif

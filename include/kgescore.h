/*
 * kgescore.h -- C ABI of libkgescore.so, the MI355X (gfx950) scoring engine behind the
 * LibKGE KgeModel / RelationalScorer plugin API.
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer owned by the caller (no allocation inside,
 *     except the entry points that say otherwise); tables are fp32 row-major with an
 *     explicit leading dimension in elements; indexes are int64;
 *   - `stream` is a hipStream_t passed as void* (PyTorch-ROCm's current stream);
 *     launches are asynchronous, no host synchronisation happens inside;
 *   - the return value is 0 on success, otherwise a hipError_t or one of the
 *     KGE_ERR_* codes below; kge_error_string() turns it into text.  The Python layer
 *     raises RuntimeError / ValueError on a non-zero status (reference error
 *     conventions: kge_model.py:155-180 asserts / ValueError).
 *
 * Which reference interface each entry point replaces is cited per function
 * (file:line into the reference checkout, kge/...).
 */
#ifndef KGESCORE_H
#define KGESCORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- enums ------------------------------------------------------------------- */
#define KGE_COMPLEX 0  /* kge/model/complex.py            */
#define KGE_DISTMULT 1 /* kge/model/distmult.py           */
#define KGE_RESCAL 2   /* kge/model/rescal.py             */
#define KGE_TRANSE 3   /* kge/model/transe.py             */
#define KGE_ROTATE 4   /* kge/model/rotate.py             */
#define KGE_CP 5       /* kge/model/cp.py: query width d_e/2; sp_ contracts with the
                          entity rows' second half, _po with their first half       */
#define KGE_SIMPLE 6   /* kge/model/simple.py                                       */

#define KGE_DIR_SP 0 /* (s, p, ?): combine="sp_" */
#define KGE_DIR_PO 1 /* (?, p, o): combine="_po" */

#define KGE_PREC_FP32 0   /* fp32-input MFMA (v_mfma_f32_32x32x2_f32): exact f32 FMA chain */
#define KGE_PREC_BF16X3 1 /* split-bf16 MFMA, hi*hi + hi*lo + lo*hi: ~2^-16 rel. per product */

#define KGE_DIST_L1 0     /* sum_k |q_k - e_k|                                   */
#define KGE_DIST_L2 1     /* sqrt(sum_k (q_k - e_k)^2)                           */
#define KGE_DIST_ROT_L1 2 /* sum_k |q_k - e_k|_C  over complex pairs [re|im]       */
#define KGE_DIST_ROT_L2 3 /* sqrt(sum_k |q_k - e_k|_C^2)                           */

#define KGE_TIE_ROUNDED_MEAN 0 /* entity_ranking.tie_handling (entity_ranking.py:531-551) */
#define KGE_TIE_BEST 1
#define KGE_TIE_WORST 2

#define KGE_ERR_ARG 1001     /* invalid argument (shape, enum, null pointer) */
#define KGE_ERR_ALIGN 1002   /* pointer / leading dimension alignment        */
#define KGE_ERR_NOGPU 1003   /* no gfx950 device visible                      */
#define KGE_ERR_SCRATCH 1004 /* needs more than the library's static scratch  */

int kge_version(void);
const char* kge_error_string(int status);

/* ---- query preparation (fused LookupEmbedder gather) --------------------------
 * Q[i, :] = prep(model, dir, ent[eidx[i]], rel[ridx[i]])      i in [0, n)
 * eidx / ridx may be NULL (row i is then taken as row i: score_emb on embeddings).
 *   dir = SP: complex cmul(s, r)            complex.py:31-38
 *             distmult s*r                  distmult.py:20
 *             rescal   s^T M_r              rescal.py:37-43
 *             transe   s + r                transe.py:19
 *             rotate   s * rot(r)           rotate.py:41-50
 *             cp       s_h * r              cp.py:23  (Q has d_e/2 columns)
 *             simple   [s_t*r_b | s_h*r_f]/2   simple.py:24-26,34
 *   dir = PO: complex conj(r)*o             complex.py:40
 *             distmult o*r                  distmult.py:22
 *             rescal   M_r o                rescal.py:44-49
 *             transe   o - r                transe.py:21
 *             rotate   o * conj(rot(r))     rotate.py:51-60 (|e*rot - o| = |e - o*conj(rot)|)
 *             cp       o_t * r              cp.py:25  (Q has d_e/2 columns)
 *             simple   [o_t*r_f | o_h*r_b]/2   simple.py:28-30,34
 * (x_h / x_t: first / second half of an entity row; r_f / r_b: of a relation row.)
 * Replaces LookupEmbedder.embed (lookup_embedder.py:91-92) + the per-scorer prologue.
 */
int kge_prep_query(int model, int dir, const float* ent, int64_t ld_ent,
                   const int64_t* eidx, const float* rel, int64_t ld_rel,
                   const int64_t* ridx, int64_t n, int d_e, int d_r, float* q,
                   int64_t ldq, void* stream);

/* kge_prep_query that can also (or only) emit the bf16 hi / lo planes of Q consumed by
 * kge_score_dot_split: q may be NULL; planes are [n][ldp], ldp >= d_e and a multiple of 8
 * (use round_up(d_e, 32)); columns d_e .. min(ldp, round_up(d_e, 32)) - 1 -- the K padding the
 * contraction reads -- are zeroed (so hi and lo may share rows of stride ldp = 2 round_up(d_e, 32):
 * [hi | lo], one buffer to exchange between GPUs).  Saves the separate kge_split_rows pass on the
 * score_sp / score_po path. */
int kge_prep_query_split(int model, int dir, const float* ent, int64_t ld_ent,
                         const int64_t* eidx, const float* rel, int64_t ld_rel,
                         const int64_t* ridx, int64_t n, int d_e, int d_r, float* q,
                         int64_t ldq, void* q_hi, void* q_lo, int64_t ldp, void* stream);

/* kge_prep_query_split for TWO stacked query batches in one launch: rows [0, n_a) are prepared
 * in direction dir_a, rows [n_a, n) in direction dir_b (eidx / ridx index all n rows) -- the
 * (s, p, ?) and (?, p, o) halves of a 1vsAll / KvsAll step (train.py:1041-1057, 699-756) or of
 * an evaluation batch (entity_ranking.py:153-168).  n_a_dev != NULL: the split point is read
 * from device memory (a launch recorded in a HIP graph then serves batches whose split differs);
 * n_a is ignored then. */
int kge_prep_query_split2(int model, int dir_a, int dir_b, int64_t n_a, const int64_t* n_a_dev,
                          const float* ent, int64_t ld_ent, const int64_t* eidx, const float* rel,
                          int64_t ld_rel, const int64_t* ridx, int64_t n, int d_e, int d_r, float* q,
                          int64_t ldq, void* q_hi, void* q_lo, int64_t ldp, void* stream);

/* kge_prep_query_split2 for an evaluation batch that will be ranked with near-tie refinement: the
 * same launch also writes band[i] = band_rel * |q_i|_2 * t_norm_max[0] (see kge_rank_band; a hair
 * wider, never narrower) -- q, both planes and band are required.  (entity_ranking.py:153-168: the
 * query side of score_sp_po for one batch.) */
int kge_prep_query_split2_band(int model, int dir_a, int dir_b, int64_t n_a, const float* ent, int64_t ld_ent,
                               const int64_t* eidx, const float* rel, int64_t ld_rel, const int64_t* ridx,
                               int64_t n, int d_e, int d_r, float* q, int64_t ldq, void* q_hi, void* q_lo,
                               int64_t ldp, float band_rel, const float* t_norm_max, float* band, void* stream);

/* backward of kge_prep_query_split2 (see kge_prep_query_bwd) */
int kge_prep_query_bwd2(int model, int dir_a, int dir_b, int64_t n_a, const int64_t* n_a_dev,
                        const float* ent, int64_t ld_ent, const int64_t* eidx, const float* rel,
                        int64_t ld_rel, const int64_t* ridx, int64_t n, int d_e, int d_r,
                        const float* dq, int64_t lddq, float* d_ent, int64_t ld_dent, float* d_rel,
                        int64_t ld_drel, void* stream);

/* backward of kge_prep_query: scatter-adds dL/d(ent row) and dL/d(rel row) into
 * d_ent / d_rel (atomic fp32 adds; either may be NULL to skip). */
int kge_prep_query_bwd(int model, int dir, const float* ent, int64_t ld_ent,
                       const int64_t* eidx, const float* rel, int64_t ld_rel,
                       const int64_t* ridx, int64_t n, int d_e, int d_r,
                       const float* dq, int64_t lddq, float* d_ent, int64_t ld_dent,
                       float* d_rel, int64_t ld_drel, void* stream);

/* ---- all-entities contraction (bilinear models) --------------------------------
 * S[i, j] = sum_k Q[i, k] * T[row(j), k],  row(j) = tidx ? tidx[j] : j
 * i in [0, n), j in [0, m), k in [0, d).  Output leading dim lds.
 * Replaces the mm in complex.py:38,40 / distmult.py:20,22 / rescal.py:42,48.
 */
int kge_score_dot(const float* q, int64_t ldq, const float* t, int64_t ldt,
                  const int64_t* tidx, int64_t n, int64_t m, int d, float* s,
                  int64_t lds, int precision, void* stream);

/* Split n fp32 rows into bf16 hi / lo planes with x ~= hi + lo (|x - hi - lo| <= 2^-16|x|).
 * Planes are row-major [n][ldo], ldo >= round_up(d, 32) and a multiple of 8; columns
 * d .. ldo-1 are written as zero.  Feeds kge_score_dot_split. */
int kge_split_rows(const float* x, int64_t ldx, int64_t n, int d, void* hi, void* lo,
                   int64_t ldo, void* stream);

/* The production bf16x3 contraction: S[i, j] = sum_k (qhi + qlo)[i, k] * T[row(j), k]
 * with the query rows pre-split (kge_split_rows) and the entity rows split on the fly.
 * Persistent, XCD-grouped 256 x 256 (n > 128) or 128 x 256 tiles.  Requires d % 4 == 0,
 * ldt % 4 == 0, 16-B aligned t / q planes. */
int kge_score_dot_split(const void* q_hi, const void* q_lo, int64_t ldq, const float* t,
                        int64_t ldt, const int64_t* tidx, int64_t n, int64_t m, int d,
                        float* s, int64_t lds, void* stream);

/* dQ[i, k] (+)= sum_j G[i, j] * T[row(j), k]   (accumulate != 0: add into dQ) */
int kge_score_dot_bwd_q(const float* g, int64_t ldg, const float* t, int64_t ldt,
                        const int64_t* tidx, int64_t n, int64_t m, int d, float* dq,
                        int64_t lddq, int accumulate, int precision, void* stream);

/* The same with a caller-owned workspace of ws_elems floats (16-B aligned).  When it holds
 * kge_score_dot_bwd_q_ws_size(n, m, d, precision) floats, the bf16x3 path's K chunks write
 * partial slabs that one pass adds in a fixed order (no float atomics: deterministic, and
 * no zero fill of dQ); otherwise it behaves as kge_score_dot_bwd_q.  Replaces the same
 * autograd step as kge_score_dot_bwd_q (mm backward of complex.py:36-44). */
int64_t kge_score_dot_bwd_q_ws_size(int64_t n, int64_t m, int d, int precision);
int kge_score_dot_bwd_q_ws(const float* g, int64_t ldg, const float* t, int64_t ldt,
                           const int64_t* tidx, int64_t n, int64_t m, int d, float* dq,
                           int64_t lddq, int accumulate, int precision, float* ws,
                           int64_t ws_elems, void* stream);

/* kge_score_dot_bwd_q (bf16x3) for callers that cannot allocate device memory -- code under
 * HIP graph capture, tight serving loops, harnesses that forbid hipMalloc.  It has no
 * counterpart in the reference.  The split-K partial slabs go to a 32 MiB static device array
 * inside the library (one copy per GPU, held until the process ends) instead of a caller
 * workspace; no hipMalloc / hipFree / allocating routine is called.  The first call on a
 * device resolves that array's address (do it once outside a graph capture).  Limits:
 * splits * n * d <= 8 Mi floats, else KGE_ERR_SCRATCH (never reached on a device of <= 256
 * CUs); 16-B aligned g / t / dq with ldg, ldt, lddq, d multiples of 4 and ldg >= round_up(m, 4),
 * else KGE_ERR_ALIGN.  Calls on one GPU share the array: calls that overlap there (two
 * streams) race.  Results equal kge_score_dot_bwd_q_ws with a full-size workspace bit for bit. */
int kge_score_dot_bwd_q_noalloc(const float* g, int64_t ldg, const float* t, int64_t ldt,
                                const int64_t* tidx, int64_t n, int64_t m, int d, float* dq,
                                int64_t lddq, int accumulate, void* stream);

/* The backward GEMMs on pre-split operand planes (bf16x3; mm backward of complex.py:36-44 /
 * distmult.py:20-22 / rescal.py:42,48, as kge_score_dot_bwd_q / _t):
 *   dQ[i, k] (+)= gscale * sum_j G[i, j] * T[j, k]          i < n, j < m, k < d
 *   dT[j, k] (+)= gscale * sum_i G[i, j] * Q[i, k]
 * g_hi / g_lo: the G planes left by kge_softmax_*_planes, row stride ldgp bf16 elements (for
 * that layout g_lo = g_hi + lds and ldgp = 2 lds); q_hi / q_lo: the query planes the forward
 * contraction used (kge_prep_query_split), row stride ldqp, with rows [n, n_pad) zero.
 * gscale: NULL or a DEVICE pointer to one float (the upstream gradient of the loss).  The dQ
 * GEMM splits its long reduction into kge_score_dot_bwd_q_planes_ws_size(n, m, d) floats of
 * caller workspace, summed in a fixed order.  All operands staged by LDS-DMA: no split, no
 * masks.  Requires d % 4 == 0 and 16-B aligned rows everywhere (else KGE_ERR_ALIGN). */
int64_t kge_score_dot_bwd_q_planes_ws_size(int64_t n, int64_t m, int d);
int kge_score_dot_bwd_q_planes(const void* g_hi, const void* g_lo, int64_t ldgp, const float* t,
                               int64_t ldt, int64_t n, int64_t m, int d, float* dq, int64_t lddq,
                               int accumulate, const float* gscale, float* ws, int64_t ws_elems,
                               void* stream);
int kge_score_dot_bwd_t_planes(const void* g_hi, const void* g_lo, int64_t ldgp, const void* q_hi,
                               const void* q_lo, int64_t ldqp, int64_t n_pad, int64_t m, int d, float* dt,
                               int64_t lddt, int accumulate, const float* gscale, void* stream);

/* dT[row(j), k] += sum_i G[i, j] * Q[i, k]   (always accumulates; rows scattered
 * atomically when tidx != NULL) */
int kge_score_dot_bwd_t(const float* g, int64_t ldg, const float* q, int64_t ldq,
                        const int64_t* tidx, int64_t n, int64_t m, int d, float* dt,
                        int64_t lddt, int precision, void* stream);

/* kge_score_dot_bwd_t with accumulate = 0: dT[j, k] = sum_i G[i, j] * Q[i, k] overwrites
 * rows 0 .. m-1 (no zero-fill pass, no read of dT; tidx must be NULL).  accumulate = 1 is
 * kge_score_dot_bwd_t. */
int kge_score_dot_bwd_t_ex(const float* g, int64_t ldg, const float* q, int64_t ldq,
                           const int64_t* tidx, int64_t n, int64_t m, int d, float* dt,
                           int64_t lddt, int accumulate, int precision, void* stream);

/* ---- all-entities distance scoring (TransE, RotatE; VALU, no MFMA) -------------
 * S[i, j] = sign * dist_kind(Q[i, :], T[row(j), :])
 * Replaces torch.cdist in transe.py:19,21 and the pairwise tensors of rotate.py:41-60.
 */
int kge_score_dist(int kind, float sign, const float* q, int64_t ldq, const float* t,
                   int64_t ldt, const int64_t* tidx, int64_t n, int64_t m, int d,
                   float* s, int64_t lds, void* stream);

/* dQ[i,:] (+)= sum_j G[i,j] * d dist/dq ;  dT[row(j),:] += sum_i G[i,j] * d dist/de */
int kge_score_dist_bwd(int kind, float sign, const float* g, int64_t ldg,
                       const float* q, int64_t ldq, const float* t, int64_t ldt,
                       const int64_t* tidx, int64_t n, int64_t m, int d, float* dq,
                       int64_t lddq, float* dt, int64_t lddt, void* stream);

/* The same gradients from READY pair weights W [n, m]: dQ[i,:] += sum_j W[i,j] phi(Q[i] - T[j]),
 * dT[row(j),:] += sum_i W[i,j] phi(T[j] - Q[i]); W = sign * G for the L1 kinds (phi = sign(x), or
 * z / |z| per complex component for RotatE), W = sign * G / dist for the L2 kinds (phi = identity)
 * -- the autograd of torch.cdist / of the norm over rotate.py:41-60's pairwise tensor with the
 * per-pair factor left to the caller, who holds the [n, m] block anyway.  Requires
 * (d or d/2 for RotatE) % 4 == 0 and 16-B aligned rows of q and t (else KGE_ERR_ALIGN). */
int kge_score_dist_bwd_weighted(int kind, const float* w, int64_t ldw, const float* q, int64_t ldq,
                                const float* t, int64_t ldt, const int64_t* tidx, int64_t n,
                                int64_t m, int d, float* dq, int64_t lddq, float* dt,
                                int64_t lddt, void* stream);

/* ---- row-wise triple scores ------------------------------------------------------
 * out[i] = score(ent[sidx[i]], rel[pidx[i]], ent[oidx[i]])      (combine="spo")
 * Replaces KgeModel.score_spo (kge_model.py:620-637) for the five scorers.  TransE uses
 * F.pairwise_distance semantics (|s+p-o+1e-6|, transe.py:17).
 */
int kge_score_spo(int model, float l_norm, const float* ent, int64_t ld_ent,
                  const int64_t* sidx, const float* rel, int64_t ld_rel,
                  const int64_t* pidx, const int64_t* oidx, int64_t n, int d_e, int d_r,
                  float* out, void* stream);

/* backward of kge_score_spo: scatter-adds g[i] * d score / d rows into d_ent, d_rel */
int kge_score_spo_bwd(int model, float l_norm, const float* ent, int64_t ld_ent,
                      const int64_t* sidx, const float* rel, int64_t ld_rel,
                      const int64_t* pidx, const int64_t* oidx, int64_t n, int d_e,
                      int d_r, const float* g, float* d_ent, int64_t ld_dent,
                      float* d_rel, int64_t ld_drel, void* stream);

/* ---- 1vsAll loss fused with its gradient ---------------------------------------------
 * loss[i] = logsumexp_j S[i, j] - S[i, labels[i]]                      (NaN if label out of range)
 * g[i, j] = scale * (softmax_j(S[i, :]) - [j == labels[i]])            (g may be NULL, or == s
 *                                                                      with ldg == lds: in place)
 * i in [0, n), j in [0, m).  scale = 1 / batch_size gives the gradient of
 * sum_i loss[i] / batch_size, the reference's 1vsAll objective:
 * KLDivWithSoftmaxKgeLoss with index labels (kge/util/loss.py:192-208) / batch size
 * (kge/job/train.py:1042, 1052).  Replaces log_softmax + nll_loss forward and backward. */
int kge_softmax_xent(const float* s, int64_t lds, int64_t n, int64_t m, const int64_t* labels,
                     float scale, float* loss, float* g, int64_t ldg, void* stream);

/* KvsAll: KL(t_i || softmax(S[i, :])) with the target built from the CSR list of positive
 * columns of row i (l_ptr[n+1], l_col; unique per row) and label smoothing eps in [0, 1):
 * labels = (1 - eps) y + 1/m if eps > 0 (kge/job/train.py:715-721), t = labels / |labels|_1
 * (KLDivWithSoftmaxKgeLoss with a label matrix, kge/util/loss.py:209-213, reduction sum);
 * g = scale * (sum_j t_ij * softmax(S[i, :]) - t_i).  Same aliasing rules as above.
 * Replaces the dense label matrix + log_softmax + kl_div forward and backward. */
int kge_softmax_kl(const float* s, int64_t lds, int64_t n, int64_t m, const int64_t* l_ptr,
                   const int64_t* l_col, float smoothing, float scale, float* loss, float* g,
                   int64_t ldg, void* stream);

/* The two losses above with the gradient left as bf16 hi / lo PLANES in place of the score
 * rows, for kge_score_dot_bwd_q_planes / _t_planes: on return row i of the buffer (lds floats)
 * holds the hi plane of G[i, 0 .. lds) in its first lds bf16 and the lo plane in its second lds
 * bf16 (G = hi + lo to 2^-16 relative; columns [m, lds) zero), and rows [n, n_pad) are zero in
 * both planes (K padding of the dT GEMM).  Requires lds % 32 == 0, a 16-B aligned buffer of
 * n_pad rows and m <= kge_softmax_planes_max_columns() (the row is held in registers); the
 * scores are consumed.  Same objectives and reference lines as kge_softmax_xent / _kl. */
int64_t kge_softmax_planes_max_columns(void);
int kge_softmax_xent_planes(float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m,
                            const int64_t* labels, float scale, float* loss, void* stream);
int kge_softmax_kl_planes(float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m, const int64_t* l_ptr,
                          const int64_t* l_col, float smoothing, float scale, float* loss, void* stream);

/* The "bce" loss (BCEWithLogitsLoss, reduction sum: kge/util/loss.py:137-158) in the same
 * in-place plane form: x = s + offset, label row y_j = (1 - smoothing) [j in P_i] + (smoothing > 0
 * ? 1 / m : 0) (KvsAll's smoothed labels, train.py:715-721; they are not normalised for this
 * loss), loss[i] = sum_j softplus(x_j) - y_j x_j, G = scale (sigmoid(x) - y) as bf16 hi / lo
 * planes.  l_ptr NULL: one positive per row, l_col[i] (1vsAll index labels, loss.py:109-117;
 * smoothing must be 0); else CSR positives.  Buffer requirements as kge_softmax_kl_planes. */
int kge_bce_planes(float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m, const int64_t* l_ptr,
                   const int64_t* l_col, float smoothing, float offset, float scale, float* loss, void* stream);

/* Negative-sampling losses on a [n, k] score block whose column 0 is each row's positive and
 * whose columns 1 .. k-1 are its negatives (the label matrix [1, 0, ..., 0] of train.py:858-871),
 * loss[i] and g = scale * dloss/ds in one launch:
 *   KGE_NS_MARGIN: sum_j max(0, arg - s_i0 + s_ij)  -- MarginRankingLoss(positives, negatives, +1)
 *                  with margin = arg, reduction sum (loss.py:227-250);
 *   KGE_NS_BCE:    BCEWithLogitsLoss(sum) of s + arg against that label row (loss.py:137-158). */
#define KGE_NS_MARGIN 0
#define KGE_NS_BCE 1
int kge_ns_loss(int kind, const float* s, int64_t lds, int64_t n, int64_t k, float arg, float scale, float* loss,
                float* g, int64_t ldg, void* stream);

/* The per-row losses of a fused two-part step reduced in one launch, in a fixed order:
 * parts[0] = scale * sum loss[0 .. n_first), parts[1] = scale * sum loss[n_first .. n),
 * total[0] = parts[0] + parts[1]  (the sp_ and _po losses of train.py:1042-1053 and their sum).
 * n_first_dev != NULL: the split point is read from device memory instead (see
 * kge_prep_query_split2). */
int kge_loss_sums(const float* loss, int64_t n, int64_t n_first, const int64_t* n_first_dev, float scale,
                  float* parts, float* total, void* stream);

/* Vocab-parallel 1vsAll (entity table row-sharded over the GPUs): S holds columns
 * [c0, c0 + m) of the full score rows, labels are global column ids.
 * row_stats: row_max[i], row_sumexp[i] = sum_j exp(S[i, j] - row_max[i]) over the slice, and
 *            target[i] = S[i, labels[i] - c0] when the label is in the slice, else 0
 *            (target may be NULL) -- reduce across shards (MAX; rescaled SUM; SUM) to get
 *            lse_i and the target score.
 * grad     : g[i, j] = scale * (exp(S[i, j] - lse[i]) - [j + c0 == labels[i]])  (labels may
 *            be NULL: no one-hot term; g may alias s with ldg == lds). */
int kge_softmax_row_stats(const float* s, int64_t lds, int64_t n, int64_t m, int64_t c0,
                          const int64_t* labels, float* row_max, float* row_sumexp, float* target,
                          void* stream);
int kge_softmax_grad(const float* s, int64_t lds, int64_t n, int64_t m, int64_t c0,
                     const int64_t* labels, const float* lse, float scale, float* g, int64_t ldg,
                     void* stream);

/* kge_softmax_grad with G left as bf16 hi / lo planes in `planes` (n_pad rows of ld floats: ld bf16
 * of the hi plane, then ld bf16 of the lo plane; columns [m, ld) and rows [n, n_pad) zeroed) -- what
 * kge_score_dot_bwd_q_planes / _t_planes read.  Out of place and elementwise, so a row may be a
 * whole shard of a large entity table.  ld % 32 == 0, 16-B aligned planes (else KGE_ERR_ALIGN). */
int kge_softmax_grad_planes(const float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m,
                            int64_t c0, const int64_t* labels, const float* lse, float scale,
                            float* planes, int64_t ld, void* stream);

/* The same planes for train.loss bce on a row shard (loss.py:137-158 BCEWithLogitsKgeLoss, reduction
 * "sum", on scores + offset against the one-hot rows of 1vsAll, train.py:1041-1057): G = scale *
 * (sigmoid(s + offset) - y), y = 1 in column labels[i] - c0 when that lies in [0, m).  Binary cross
 * entropy couples no columns, so a shard needs nothing from the others.  loss_part [n,
 * kge_grad_planes_chunks(ld)] receives each column chunk's share of row i's loss,
 * sum_j softplus(x_ij) - y_ij x_ij (unscaled; the caller sums it in a fixed order); rows
 * [n, n_pad) of loss_part are not written. */
int64_t kge_grad_planes_chunks(int64_t ld);
int kge_bce_grad_planes(const float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m, int64_t c0,
                        const int64_t* labels, float offset, float scale, float* planes, int64_t ld,
                        float* loss_part, void* stream);

/* ---- per-row candidate lists (negative sampling) -------------------------------------
 * out[i, c] = score(Q[i, :], ent[cand[i, c], :])  i in [0, n), c in [0, k), with the
 * semantics of KgeModel.score_spo on the triple the candidate completes (kge_model.py:620-637):
 *   ComplEx / DistMult / RESCAL / CP / SimplE: <q, e>   (Q from kge_prep_query, either
 *            direction; for CP, ent / d are the entity-row window of width d_e/2)
 *   TransE : -|| sigma (q - e) + 1e-6 ||_p, sigma = +1 (dir SP: s+p-o') / -1 (dir PO: s'+p-o)
 *            (F.pairwise_distance, transe.py:17)
 *   RotatE : sum_k |q_k - e_k|_C (p = 1) or its L2 form; (s o rot(p)) - o' / s' o rot(p) - o
 *            via |s' - o conj(rot(p))| = |s' o rot(p) - o|  (rotate.py:18-50)
 * Replaces the B x (1 + N) triple construction + score_spo of TrainingJobNegativeSampling's
 * "triple" implementation (kge/job/train.py:868-892).  d <= 4096. */
int kge_score_cand(int model, float l_norm, int dir, const float* q, int64_t ldq, const float* ent,
                   int64_t ld_ent, const int64_t* cand, int64_t ldc, int64_t n, int64_t k, int d,
                   float* out, int64_t ldo, void* stream);

/* backward: dq[i, :] = sum_c g[i, c] d out[i, c] / d q (written; dq may be NULL) and
 * d_ent[cand[i, c], :] += g[i, c] d out[i, c] / d e (atomic; may be NULL).  s = the forward
 * scores (needed by TransE / RotatE, whose L2 norms it holds).  d <= 3584. */
int kge_score_cand_bwd(int model, float l_norm, int dir, const float* q, int64_t ldq,
                       const float* ent, int64_t ld_ent, const int64_t* cand, int64_t ldc,
                       int64_t n, int64_t k, int d, const float* s, int64_t lds, const float* g,
                       int64_t ldg, float* dq, int64_t lddq, float* d_ent, int64_t ld_dent,
                       void* stream);

/* The same two passes for candidate lists given in a caller-chosen ORDER: position c of row i
 * holds candidate cand[i, c] whose score belongs to column col[i, c] of out / g / s (col[i, :] a
 * permutation of 0 .. k-1).  With every row in ascending candidate order the workgroups of an XCD
 * sweep the entity table together and find most rows in that XCD's L2 (same result, same
 * reference code: kge/job/train.py:868-892; the order of a row's candidates carries no meaning
 * there).  kge_score_cand_bwd_q_ordered writes dq only and needs the vector layout of
 * kge_score_cand_bwd's fast path ((d or d/2 for RotatE) % 4 == 0, 16-B aligned rows, at most
 * 2048 such elements; else KGE_ERR_ALIGN). */
int kge_score_cand_ordered(int model, float l_norm, int dir, const float* q, int64_t ldq,
                           const float* ent, int64_t ld_ent, const int64_t* cand, int64_t ldc,
                           const int64_t* col, int64_t ldcol, int64_t n, int64_t k, int d,
                           float* out, int64_t ldo, void* stream);
int kge_score_cand_bwd_q_ordered(int model, float l_norm, int dir, const float* q, int64_t ldq,
                                 const float* ent, int64_t ld_ent, const int64_t* cand,
                                 int64_t ldc, const int64_t* col, int64_t ldcol, int64_t n,
                                 int64_t k, int d, const float* s, int64_t lds, const float* g,
                                 int64_t ldg, float* dq, int64_t lddq, void* stream);

/* d_ent part of kge_score_cand_bwd without atomics, for candidate lists with many repeats:
 * the caller groups the n*k pairs by entity -- order[] = the flattened pair indexes
 * (i*k + c; cand contiguous [n][k]) sorted by cand value, seg_ptr[nseg+1] the group
 * boundaries -- and each entity row is accumulated once (d_ent[e] += ..., plain RMW).
 * Requires (d or d/2 for RotatE) % 4 == 0 and 16-B aligned rows (else KGE_ERR_ALIGN). */
int kge_score_cand_bwd_ent(int model, float l_norm, int dir, const float* q, int64_t ldq,
                           const float* ent, int64_t ld_ent, const int64_t* cand, int64_t n,
                           int64_t k, int d, const int64_t* order, const int64_t* seg_ptr,
                           int64_t nseg, const float* s, int64_t lds, const float* g, int64_t ldg,
                           float* d_ent, int64_t ld_dent, void* stream);

/* Counting-sort scatter: order[cursor[idx[t]]++] = t for t in [0, n) (int64 atomics on
 * cursor; order within a bucket unspecified).  With cursor = the exclusive prefix sum of the
 * bucket counts this groups t by idx[t] -- the order / seg_ptr input of
 * kge_score_cand_bwd_ent. */
int kge_bucket_scatter(const int64_t* idx, int64_t n, int64_t* cursor, int64_t* order,
                       void* stream);

/* Every row of x[n, k] (ids in [0, 2^50), k <= 8192) sorted ascending, stably: sorted[i, :] and the
 * positions col[i, :] the ids came from (both contiguous [n, k]) -- torch.sort(x, 1, stable=True)
 * as one launch, the cand / col input of kge_score_cand_ordered.  id_bound: 0, or an exclusive
 * upper bound of the ids (the number of entities); with id_bound <= 2^21 and k <= 2048 the sort
 * runs on 32-bit keys, and ids outside [0, id_bound) -- invalid for every consumer -- come out
 * clamped into that range. */
int kge_sort_rows(const int64_t* x, int64_t ldx, int64_t n, int64_t k, int64_t id_bound, int64_t* sorted,
                  int64_t* col, void* stream);

/* The order / seg_ptr input of kge_score_cand_bwd_ent from candidate lists that kge_sort_rows has
 * sorted (srt, col: contiguous [n, k], n <= 4096): seg_ptr[nbuckets + 1] and order[n * k] with
 * order[slot] = i * k + col[i, position] -- the counting sort of kge_bucket_count +
 * exclusive scan + kge_bucket_scatter in one launch and without global atomics (every workgroup
 * owns a range of ids, which is one contiguous run of each sorted row). */
int kge_group_sorted_rows(const int64_t* srt, const int64_t* col, int64_t n, int64_t k, int64_t nbuckets,
                          int64_t* seg_ptr, int64_t* order, void* stream);

/* The bucket counts that go with it: counts[idx[t]] += 1 for t in [0, n) (int64 atomics; the
 * caller zeroes counts; indexes outside [0, nbuckets) are skipped) -- torch.bincount without its
 * host round trip for the maximum. */
int kge_bucket_count(const int64_t* idx, int64_t n, int64_t nbuckets, int64_t* counts, void* stream);

/* ---- optimizer ------------------------------------------------------------------------
 * One fused Adagrad step over n contiguous fp32 elements (an embedding table, its dense
 * gradient and its state sum), element-wise as torch.optim.Adagrad's multi-tensor path:
 *   g = maximize ? -grad : grad;  g += weight_decay * p;  sum += g * g;
 *   p += (g * minus_clr) / (sqrt(sum) + eps),   minus_clr = -lr / (1 + (step - 1) lr_decay)
 * Replaces the torch.optim.Adagrad step behind train.optimizer "Adagrad"
 * (kge/util/optimizer.py:11-32). */
int kge_adagrad_step(float* param, const float* grad, float* state_sum, int64_t n,
                     float minus_clr, float eps, float weight_decay, int maximize,
                     void* stream);

/* The same step for up to 8 tensors in ONE launch (the entity and the relation table of a
 * training step): host arrays of `count` device pointers / element counts / per-tensor
 * minus_clr; eps, weight_decay and maximize are shared (one torch param group). */
int kge_adagrad_step_multi(int count, float* const* params, const float* const* grads,
                           float* const* state_sums, const int64_t* ns, const float* minus_clrs,
                           float eps, float weight_decay, int maximize, void* stream);

/* ---- frequency-weighted Lp penalty of a lookup embedder ------------------------------------------
 * The weighted branch of LookupEmbedder.penalty (lookup_embedder.py:138-158) summed over the
 * OCCURRENCES of the batch's indexes instead of over unique indexes times their counts (the same
 * number, without torch.unique's data-dependent shape):
 *   row_sums[i] = sum_k |w[idx[i], k]|^p;        the caller sums them and scales by weight / (p n)
 *   dw[idx[i], k] += gscale[0] * coeff * d/dx |x|^p at x = w[idx[i], k]        (gscale may be NULL: 1)
 * p = 1 .. 4. */
int kge_lp_rows(const float* w, int64_t ldw, const int64_t* idx, int64_t n, int d, int p,
                float* row_sums, void* stream);
int kge_lp_rows_bwd(const float* w, int64_t ldw, const int64_t* idx, int64_t n, int d, int p,
                    const float* gscale, float coeff, float* dw, int64_t lddw, void* stream);

/* Copy n int64 from host-pinned, device-visible memory (hipHostMalloc) into device memory
 * with a kernel on `stream`: the per-batch index upload of the replayed 1vsAll training
 * step (engine.graph_step).  Internal plumbing; no reference counterpart (the reference
 * moves each batch with triples.to(device), train.py:1035). */
int kge_stage_i64(const int64_t* src, int64_t* dst, int64_t n, void* stream);

/* ---- entity-ranking counts (eval) --------------------------------------------------
 * For row i of a score chunk S[n, m] covering entities [c0, c0 + m):
 *   v_j = S[i, j], with v_{true_i - c0} := true_score[i] when true_i is in the chunk;
 *   NaN -> -inf, filtered entries -> -inf (entity_ranking.py:172-177, 497-502, 519-523).
 *   greater[r, i] += #{j : v_j > t_i},  ties[r, i] += #{j : v_j == t_i}
 * for ranking r in {0: raw, 1: filtered by F, 2: filtered by F u T}.
 * F and T are CSR lists of GLOBAL entity ids per row (f_ptr[n+1], f_col[...]); each
 * list must hold unique ids; T entries that are also in F are ignored; the true entity
 * itself is never filtered.  t_ptr may be NULL (only rankings 0 and 1 are produced).
 * Counts accumulate (+=) so chunks / shards sum exactly (entity_ranking.py:153-216).
 * Replaces _filter_and_rank / _get_ranks_and_num_ties (entity_ranking.py:469-529).
 */
int kge_rank_counts(const float* s, int64_t lds, int64_t n, int64_t m, int64_t c0,
                    const int64_t* true_idx, const float* true_score,
                    const int64_t* f_ptr, const int64_t* f_col, const int64_t* t_ptr,
                    const int64_t* t_col, int64_t* greater, int64_t* ties,
                    void* stream);

/* ranks[i] = tie rule(greater[i], ties[i]) and hist[ranks[i]] += 1 (float histogram
 * of length hist_len, eval.py:148-171); ranks may be NULL. */
int kge_rank_hist(const int64_t* greater, const int64_t* ties, int64_t n,
                  int tie_handling, int64_t* ranks, float* hist, int64_t hist_len,
                  void* stream);

/* Metrics of K rank histograms in one launch (kge/job/entity_ranking.py:553-577: mean rank,
 * mean reciprocal rank, hits@k from a histogram of ranks).  hists: [k, e] fp32 counts with
 * leading dimension ld, hists[i][j] = how many triples got rank j + 1.  out: [k, 3 + kmax]
 * doubles per histogram: the count n, sum_j h[j] (j + 1), sum_j h[j] * fl32(1 / (j + 1)), then
 * hits@1 .. hits@kmax = fl32(cumulative count / n) (0 when n = 0).  The weighted sums use the
 * reference's fp32 operands and accumulate in fp64 in a fixed order. */
int kge_rank_metrics(const float* hists, int64_t ld, int64_t k, int64_t e, int kmax, double* out, void* stream);

/* The same for several rankings in one launch: row i counts into histogram
 * i / rows_per_hist of hist[(n / rows_per_hist) x hist_len] (the raw / filtered /
 * filtered-with-test histograms of one eval batch direction, eval.py:148-171). */
int kge_rank_hist_multi(const int64_t* greater, const int64_t* ties, int64_t n,
                        int64_t rows_per_hist, int tie_handling, int64_t* ranks,
                        float* hist, int64_t hist_len, void* stream);

/* One launch for a whole evaluation batch: the score block S[n_a + n_b, m] stacks the
 * (s, p, ?) queries (rows [0, n_a), true column o, entity_ranking.py:153-168 "sp" half) on
 * the (?, p, o) queries (rows [n_a, n_a + n_b), true column s, the "po" half); each batch
 * brings its own true_idx / true_score / CSR pointers, the CSR columns (f_col, t_col) are
 * shared.  Counting follows kge_rank_counts; greater / ties are [1 + #filters][n_a + n_b]
 * (ranking-major), added to when accumulate != 0 and overwritten otherwise.
 * tie_handling >= 0 (needs accumulate == 0: one chunk covers every entity) also finishes
 * the batch: ranks[r, i] by the tie rule and hist[(r * n + i) / rows_per_hist][rank] += 1
 * (entity_ranking.py:531-551, eval.py:148-171).
 * q != NULL refines scores produced by a reduced-precision contraction: with
 *   band_i = band_rel * |q_i|_2 * t_norm_max[0]      (t_norm_max: kge_row_norm_max)
 * an entry with |S[i, j] - true_score_i| <= band_i is replaced, before it is compared, by
 * the correctly rounded fp32 value of the exact dot product q_i . t_j (fp64 accumulation,
 * fixed order; q: fp32 query rows [n, d], t: the chunk's fp32 candidate rows [m, d]).
 * When the contraction's error stays below the band, the counts equal those of exactly
 * computed scores.  The reference ranks fp32 scores (entity_ranking.py:469-529). */
int kge_rank_rows(const float* s, int64_t lds, int64_t n_a, int64_t n_b, int64_t m, int64_t c0,
                  const int64_t* true_idx_a, const float* true_score_a, const int64_t* f_ptr_a,
                  const int64_t* t_ptr_a, const int64_t* true_idx_b, const float* true_score_b,
                  const int64_t* f_ptr_b, const int64_t* t_ptr_b, const int64_t* f_col,
                  const int64_t* t_col, int64_t* greater, int64_t* ties, int accumulate,
                  int tie_handling, int64_t* ranks, float* hist, int64_t hist_len,
                  int64_t rows_per_hist, const float* q, int64_t ldq, const float* t, int64_t ldt,
                  int d, float band_rel, const float* t_norm_max, void* stream);

/* The evaluation contraction with the ranking fused into its epilogue: S = Q . T^T as in
 * kge_score_dot_split (bf16 hi / lo query planes, fp32 table rows t [m, d] = columns
 * c0 .. c0 + m of the entity axis), but the scores never reach memory.  Each score is compared
 * with its row's true score in registers and leaves as a 2-bit code -- 0: below (also the true
 * column itself and columns past m), 1: above, 2: equal, 3: |score - true_score_i| <= band[i],
 * to be rescored exactly by kge_rank_rows_codes -- 16 codes per 32-bit word, ldc words per row
 * (ldc >= kge_rank_codes_ld(m)).  Rows [0, n_a) are query batch A, rows [n_a, n_a + n_b) batch B
 * (the (s, p, ?) and the (?, p, o) queries of an evaluation batch): each brings its true scores
 * and true columns (global ids); band: one per row, band < 0 switches code 3 off.  Replaces scores -> "scores > true" / "scores == true"
 * sums of entity_ranking.py:164-216, 469-529 without the [n, m] score block in memory. */
int kge_score_dot_split_rank(const void* q_hi, const void* q_lo, int64_t ldq, const float* t, int64_t ldt,
                             int64_t n_a, int64_t n_b, int64_t m, int d, const float* true_score_a,
                             const int64_t* true_idx_a, const float* true_score_b, const int64_t* true_idx_b,
                             const float* band, int64_t c0, void* codes, int64_t ldc, void* stream);

/* Words per row of the code block of kge_score_dot_split_rank for m columns. */
int64_t kge_rank_codes_ld(int64_t m);

/* band[i] = band_rel * |q_i|_2 * t_norm_max[0] for the n fp32 query rows q [n, d]: the per-row
 * refinement band kge_score_dot_split_rank takes (the band kge_rank_rows derives for itself).
 * No counterpart in the reference, which ranks exact fp32 scores (entity_ranking.py:469-529). */
int kge_rank_band(const float* q, int64_t ldq, int64_t n, int d, float band_rel, const float* t_norm_max,
                  float* band, void* stream);

/* kge_rank_rows on the code block of kge_score_dot_split_rank instead of a score block: counts
 * codes 1 / 2, rescores every code-3 entry exactly (q, t, d as in kge_rank_rows; q may be null
 * only when no code 3 can occur, i.e. band < 0), adds the true entry's own tie, applies the
 * filter lists (a listed column's code is looked up; code 3 is rescored), tie policy, ranks and
 * histograms exactly as kge_rank_rows does (entity_ranking.py:172-216, 469-551). */
int kge_rank_rows_codes(const void* codes, int64_t ldc, int64_t n_a, int64_t n_b, int64_t m, int64_t c0,
                        const int64_t* true_idx_a, const float* true_score_a, const int64_t* f_ptr_a,
                        const int64_t* t_ptr_a, const int64_t* true_idx_b, const float* true_score_b,
                        const int64_t* f_ptr_b, const int64_t* t_ptr_b, const int64_t* f_col,
                        const int64_t* t_col, int64_t* greater, int64_t* ties, int accumulate,
                        int tie_handling, int64_t* ranks, float* hist, int64_t hist_len,
                        int64_t rows_per_hist, const float* q, int64_t ldq, const float* t, int64_t ldt,
                        int d, float band_rel, const float* t_norm_max, void* stream);

/* out[0] = max_j |t_j|_2 over the m rows of t (device scalar; the refinement band of
 * kge_rank_rows).  No counterpart in the reference, which ranks exact fp32 scores
 * (entity_ranking.py:469-529). */
int kge_row_norm_max(const float* t, int64_t ldt, int64_t m, int d, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KGESCORE_H */

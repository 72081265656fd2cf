// Scores of each query against its OWN candidate list -- the negative-sampling hot path
// (TrainingJobNegativeSampling "triple" implementation, train.py:868-892: score_spo over the
// B x (1 + N) triples that share (s, p) or (p, o) with a positive), with score_spo's
// per-model semantics (kge_model.py:620-637):
//   out[i, c] = score(q_i, ent[cand[i, c]])
//     dot models : <q_i, e>                                   (q = prep(s, r) / prep(r, o))
//     TransE     : -|| sigma (q_i - e) + 1e-6 ||_p            (F.pairwise_distance,
//                  sigma = +1 for sp_ queries (s+p-o'), -1 for _po (s'+p-o), transe.py:17)
//     RotatE     : + sum_k |q_ik - e_k|_C  (p=1) / sqrt(sum |.|^2) (p=2)   (rotate.py:18-50)
// Nothing is shared between rows, so the kernel is a gather: one workgroup per query row,
// the query staged in LDS, each wave streams whole candidate rows (float4 per lane, two
// rows in flight) and reduces across the wave.  4*d bytes per scored triple; the FB15K-237
// table (14,541 x 1024 x 4 = 59.6 MB) stays resident in the 256 MB MALL across rows.
//
// Backward (same gather shape, no atomics on the fast path):
//   dq_i  = sum_c g_ic d score / d q   -- one workgroup per query row, each lane keeping
//           its slice of the row in registers (all of a candidate row's loads in flight),
//           waves reduced through LDS;
//   d_ent = per entity e: sum over the (i, c) with cand[i, c] = e -- the caller groups the
//           pairs by entity (kge_bucket_scatter), one wave per entity accumulates its row
//           in registers and writes it once.
// A scalar fallback (any d / alignment) scatters d_ent with fp32 atomics.
#include <type_traits>

#include "common.h"

namespace {

constexpr int NT = 512, NW = NT / 64;
enum { K_DOT = 0, K_TRANSE = 1, K_ROTATE = 2 };

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 f4(float v) { return make_float4(v, v, v, v); }

// Per-element contribution to the reduction for (q, e) components.  For RotatE (re, im)
// pairs are handled by the caller.
template <int KIND>
__device__ __forceinline__ float elem(float q, float e, float sigma, bool l1) {
  if (KIND == K_DOT) return q * e;
  const float df = sigma * (q - e) + 1e-6f;
  return l1 ? fabsf(df) : df * df;
}

// |dr + i di| (p = 1) or its square: the hardware square root (1 ulp), as the all-entities
// distance kernels take it -- sqrtf's correctly rounded expansion is ten instructions per element
__device__ __forceinline__ float cabs_term(float dr, float di, bool l1) {
  const float sq = fmaf(di, di, dr * dr);
  return l1 ? __builtin_amdgcn_sqrtf(sq) : sq;
}

template <int KIND>
__device__ __forceinline__ float finish(float acc, bool l1) {
  if (KIND == K_DOT) return acc;
  if (KIND == K_TRANSE) return -(l1 ? acc : sqrtf(acc));
  return l1 ? acc : sqrtf(acc);
}

// sum over the row of the candidate at `e`; lane-strided, q from LDS
template <int KIND, bool VEC>
__device__ __forceinline__ float row_reduce(const float* qs, const float* e, int d, int lane, float sigma, bool l1) {
  float acc = 0.f;
  if (KIND == K_ROTATE) {
    const int h = d / 2;
    if (VEC) {
      for (int k = lane * 4; k < h; k += 256) {
        const float4 er = ld4(e + k), ei = ld4(e + k + h);
        const float4 qr = *reinterpret_cast<const float4*>(qs + k), qi = *reinterpret_cast<const float4*>(qs + k + h);
        acc += cabs_term(qr.x - er.x, qi.x - ei.x, l1) + cabs_term(qr.y - er.y, qi.y - ei.y, l1) +
               cabs_term(qr.z - er.z, qi.z - ei.z, l1) + cabs_term(qr.w - er.w, qi.w - ei.w, l1);
      }
    } else {
      for (int k = lane; k < h; k += 64) acc += cabs_term(qs[k] - e[k], qs[k + h] - e[k + h], l1);
    }
  } else {
    if (VEC) {
      for (int k = lane * 4; k < d; k += 256) {
        const float4 ev = ld4(e + k);
        const float4 qv = *reinterpret_cast<const float4*>(qs + k);
        acc += elem<KIND>(qv.x, ev.x, sigma, l1) + elem<KIND>(qv.y, ev.y, sigma, l1) +
               elem<KIND>(qv.z, ev.z, sigma, l1) + elem<KIND>(qv.w, ev.w, sigma, l1);
      }
    } else {
      for (int k = lane; k < d; k += 64) acc += elem<KIND>(qs[k], e[k], sigma, l1);
    }
  }
  return acc;
}

template <int KIND, bool VEC>
__global__ void __launch_bounds__(NT) cand_kernel(bool l1, float sigma, const float* __restrict__ q, int64_t ldq,
                                                  const float* __restrict__ ent, int64_t ld_ent,
                                                  const int64_t* __restrict__ cand, int64_t ldc,
                                                  const int64_t* __restrict__ col, int64_t ldcol, int k, int d,
                                                  float* __restrict__ out, int64_t ldo) {
  extern __shared__ __attribute__((aligned(16))) float qs[];
  const int64_t i = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int t = threadIdx.x; t < d; t += NT) qs[t] = q[i * ldq + t];
  __syncthreads();
  const int64_t* ci = cand + i * ldc;
  // two candidate rows per wave per iteration: their loads are independent
  for (int c = w; c < k; c += 2 * NW) {
    const int c2 = c + NW;
    const float* e1 = ent + ci[c] * ld_ent;
    const float* e2 = ent + ci[c2 < k ? c2 : c] * ld_ent;
    float a1 = row_reduce<KIND, VEC>(qs, e1, d, lane, sigma, l1);
    float a2 = row_reduce<KIND, VEC>(qs, e2, d, lane, sigma, l1);
    a1 = wave_sum(a1);
    a2 = wave_sum(a2);
    if (lane == 0) {  // col: the output column of the candidate at position c (ordered lists)
      out[i * ldo + (col ? col[i * ldcol + c] : c)] = finish<KIND>(a1, l1);
      if (c2 < k) out[i * ldo + (col ? col[i * ldcol + c2] : c2)] = finish<KIND>(a2, l1);
    }
  }
}

// Sum over the wave without LDS traffic: four DPP steps leave every lane with the sum of its row of
// 16 lanes, the four row sums are read by v_readlane.  (wave_sum's ds_bpermute butterfly is a
// chain of six LDS round trips per candidate row, which the one-row-in-flight loop cannot hide.)
__device__ __forceinline__ float dpp_add(float v, const int ctrl_tag) {
  const int x = __builtin_bit_cast(int, v);
  int y;
  switch (ctrl_tag) {  // the control word must be an immediate
    case 0: y = __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false); break;   // quad_perm [1,0,3,2]
    case 1: y = __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false); break;   // quad_perm [2,3,0,1]
    case 2: y = __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false); break;  // row_half_mirror
    default: y = __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false); break; // row_mirror
  }
  return v + __builtin_bit_cast(float, y);
}

__device__ __forceinline__ float wave_sum_rows(float v) {
  v = dpp_add(v, 0);
  v = dpp_add(v, 1);
  v = dpp_add(v, 2);
  v = dpp_add(v, 3);
  const int x = __builtin_bit_cast(int, v);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 48));
  return (r0 + r1) + (r2 + r3);
}

// The same scores with the query's slice in registers (lane owns elements ch*256 + lane*4 .. +3,
// as the backward kernels) and a whole candidate row requested at once.
template <int KIND, int NCH>
__global__ void __launch_bounds__(NT) cand_fwd_kernel(bool l1, float sigma, const float* __restrict__ q, int64_t ldq,
                                                      const float* __restrict__ ent, int64_t ld_ent,
                                                      const int64_t* __restrict__ cand, int64_t ldc,
                                                      const int64_t* __restrict__ col, int64_t ldcol, int k, int d,
                                                      float* __restrict__ out, int64_t ldo) {
  constexpr int P = KIND == K_ROTATE ? 2 : 1;
  const int64_t i = blockIdx.x;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int unit = KIND == K_ROTATE ? d / 2 : d;
  const float* qi = q + i * ldq;
  float4 qv[NCH][P];
  int off[NCH];
  bool own[NCH];  // lanes past the row's end re-read its last elements and count nothing
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    own[ch] = ch * 256 + lane * 4 < unit;
    off[ch] = min(ch * 256 + lane * 4, unit - 4);
#pragma unroll
    for (int pl = 0; pl < P; ++pl) qv[ch][pl] = ld4(qi + off[ch] + pl * unit);
  }
  const int64_t* ci = cand + i * ldc;
  const int64_t* coli = col ? col + i * ldcol : nullptr;
  auto rows = [&](float4 (&ev)[NCH][P], int64_t id) {
    const float* e = ent + id * ld_ent;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
      for (int pl = 0; pl < P; ++pl) ev[ch][pl] = ld4(e + off[ch] + pl * unit);
  };
  auto reduce = [&](const float4 (&ev)[NCH][P]) {
    float acc = 0.f;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const float4 a = qv[ch][0], b = ev[ch][0];
      float t;
      if (KIND == K_ROTATE) {
        const float4 ai = qv[ch][P - 1], bi = ev[ch][P - 1];
        t = cabs_term(a.x - b.x, ai.x - bi.x, l1) + cabs_term(a.y - b.y, ai.y - bi.y, l1) +
            cabs_term(a.z - b.z, ai.z - bi.z, l1) + cabs_term(a.w - b.w, ai.w - bi.w, l1);
      } else {
        t = elem<KIND>(a.x, b.x, sigma, l1) + elem<KIND>(a.y, b.y, sigma, l1) + elem<KIND>(a.z, b.z, sigma, l1) +
            elem<KIND>(a.w, b.w, sigma, l1);
      }
      if (own[ch]) acc += t;
    }
    return wave_sum_rows(acc);
  };
  auto put = [&](int c, float a) {
    if (lane == 0 && c < k) out[i * ldo + (coli ? coli[c] : c)] = finish<KIND>(a, l1);
  };
  // ONE row per wave on its way at a time: the candidate lists of the queries resident on an XCD
  // are swept together (ascending lists), and the rows they share are found in that XCD's L2 only
  // while everything in flight plus the spread between the workgroups fits into it -- at 4-KB rows
  // two rows per wave in flight cost 15 % and four 50 % (measured at 512 x 1,025 x 1,024 floats).
  int64_t id = ci[w < k ? w : 0];
  for (int c = w; c < k; c += NW) {
    float4 a[NCH][P];
    rows(a, id);
    id = ci[min(c + NW, k - 1)];
    put(c, reduce(a));
  }
}

// ---------------------------------------------------------------------------- backward
// g * d score / d q for one element (re part / both parts for RotatE); d score / d e is
// its negative for the distance models and g * q for the dot models.
template <int KIND>
__device__ __forceinline__ void grad_q(bool l1, float sigma, float inv, float gc, float qr, float qi, float er,
                                       float ei, float& gr, float& gi) {
  if (KIND == K_DOT) {
    gr = gc * er;
  } else if (KIND == K_TRANSE) {  // score = -||diff||, diff = sigma (q - e) + eps
    const float df = sigma * (qr - er) + 1e-6f;
    // p = 1: sign(df) as the median of (df * 2^126, -1, 1) -- every normal df saturates, 0 stays 0
    const float dn = l1 ? __builtin_amdgcn_fmed3f(df * 0x1p126f, -1.f, 1.f) : df * inv;
    gr = -gc * sigma * dn;
  } else {  // score = sum |q - e|_C or its L2 form
    const float dr = qr - er, di = qi - ei;
    float f = inv;
    if (l1) {  // 1 / |dr + i di| by the hardware reciprocal square root (1 ulp); 0 at 0
      const float sq = fmaf(di, di, dr * dr);
      f = sq > 0.f ? __builtin_amdgcn_rsqf(sq) : 0.f;
    }
    f *= gc;
    gr = dr * f;
    gi = di * f;
  }
}

// 1 / (L2 norm) of pair (i, c) from its forward score (TransE: -||.||, RotatE: +||.||)
template <int KIND>
__device__ __forceinline__ float inv_norm(bool l1, const float* s, int64_t idx) {
  if (KIND == K_DOT || l1) return 0.f;
  const float nrm = KIND == K_TRANSE ? -s[idx] : s[idx];
  return nrm > 0.f ? 1.f / nrm : 0.f;
}

// dq, vectorised: lane owns elements ch*256 + lane*4 .. +3 (and the RotatE im parts)
template <int KIND, int NCH>
__global__ void __launch_bounds__(NT) cand_bwd_q_kernel(bool l1, float sigma, const float* __restrict__ q,
                                                        int64_t ldq, const float* __restrict__ ent, int64_t ld_ent,
                                                        const int64_t* __restrict__ cand, int64_t ldc,
                                                        const int64_t* __restrict__ col, int64_t ldcol, int k, int d,
                                                        const float* __restrict__ s, int64_t lds,
                                                        const float* __restrict__ g, int64_t ldg, float* __restrict__ dq,
                                                        int64_t lddq) {
  constexpr int P = KIND == K_ROTATE ? 2 : 1;  // float4 planes per chunk
  extern __shared__ __attribute__((aligned(16))) float red[];  // NW x d
  const int64_t i = blockIdx.x;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int unit = KIND == K_ROTATE ? d / 2 : d;
  const float* qi = q + i * ldq;
  float4 qv[NCH][P], acc[NCH][P];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int kk = min(ch * 256 + lane * 4, unit - 4);
#pragma unroll
    for (int pl = 0; pl < P; ++pl) {
      qv[ch][pl] = ld4(qi + kk + pl * unit);
      acc[ch][pl] = f4(0.f);
    }
  }
  const int64_t* ci = cand + i * ldc;
  const int64_t* coli = col ? col + i * ldcol : nullptr;
  // gradient and inverse norm of the candidate at position c (its column in g and s: col)
  auto meta = [&](int c, float& gc, float& inv) {
    const int64_t cc = coli ? coli[c] : c;
    gc = g[i * ldg + cc];
    inv = inv_norm<KIND>(l1, s, i * lds + cc);
  };
  auto rows = [&](float4 (&ev)[NCH][P], int64_t id) {
    const float* e = ent + id * ld_ent;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
      for (int pl = 0; pl < P; ++pl) ev[ch][pl] = ld4(e + min(ch * 256 + lane * 4, unit - 4) + pl * unit);
  };
  auto accumulate = [&](const float4 (&ev)[NCH][P], float gc, float inv) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const float4 a = qv[ch][0], b = ev[ch][0];
      const float4 ai = P > 1 ? qv[ch][P - 1] : a, bi = P > 1 ? ev[ch][P - 1] : b;
      float gr[4], gi[4];
      grad_q<KIND>(l1, sigma, inv, gc, a.x, ai.x, b.x, bi.x, gr[0], gi[0]);
      grad_q<KIND>(l1, sigma, inv, gc, a.y, ai.y, b.y, bi.y, gr[1], gi[1]);
      grad_q<KIND>(l1, sigma, inv, gc, a.z, ai.z, b.z, bi.z, gr[2], gi[2]);
      grad_q<KIND>(l1, sigma, inv, gc, a.w, ai.w, b.w, bi.w, gr[3], gi[3]);
      acc[ch][0].x += gr[0]; acc[ch][0].y += gr[1]; acc[ch][0].z += gr[2]; acc[ch][0].w += gr[3];
      if (P > 1) {
        acc[ch][P - 1].x += gi[0]; acc[ch][P - 1].y += gi[1]; acc[ch][P - 1].z += gi[2]; acc[ch][P - 1].w += gi[3];
      }
    }
  };
  // A candidate is a chain of dependent loads (column -> gradient / norm, id -> row): the next
  // candidate's gradient, norm and id are fetched while this one's row is on its way.  One row
  // per wave in flight, no more (see cand_fwd_kernel).
  // The distance kinds spend enough arithmetic per row for the waves of a workgroup to drift apart
  // along the candidate list, and with them the table rows they share with the XCD's other
  // workgroups: a barrier every 16 candidates keeps them together (RotatE-L1 160 -> 128 us at
  // 512 x 1,025 x 1,024; dot scores, 96 us without, lose 10 us to it).  Uniform trip count.
  constexpr int SYNC_EVERY = KIND == K_DOT ? 0 : 16;
  {
    const int iters = (k + NW - 1) / NW;
    float gc_n = 0.f, inv_n = 0.f;
    int64_t id_n = 0;
    if (w < k) {
      meta(w, gc_n, inv_n);
      id_n = ci[w];
    }
    for (int it = 0; it < iters; ++it) {
      const int c = w + it * NW;
      if (c < k) {
        const float gc = gc_n, inv = inv_n;
        float4 ev[NCH][P];
        rows(ev, id_n);
        if (c + NW < k) {
          meta(c + NW, gc_n, inv_n);
          id_n = ci[c + NW];
        }
        if (gc != 0.f) accumulate(ev, gc, inv);
      }
      if (SYNC_EVERY > 0 && (it & (SYNC_EVERY - 1)) == SYNC_EVERY - 1) __syncthreads();
    }
  }
  // cross-wave reduction through LDS (each wave's partial row), then one store of dq_i
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int kk = ch * 256 + lane * 4;
    if (kk < unit)
#pragma unroll
      for (int pl = 0; pl < P; ++pl) *reinterpret_cast<float4*>(red + w * d + kk + pl * unit) = acc[ch][pl];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < d; t += NT) {
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < NW; ++u) v += red[u * d + t];
    dq[i * lddq + t] = v;
  }
}

// d_ent, vectorised, one wave per entity group (pairs of order[seg_ptr[u] .. seg_ptr[u+1])).
// A pair is a chain of dependent loads (pair index -> gradient / norm -> query row): the loop takes
// several pairs per round trip.
template <int KIND, int NCH>
__global__ void __launch_bounds__(256) cand_bwd_ent_kernel(bool l1, float sigma, const float* __restrict__ q,
                                                           int64_t ldq, const float* __restrict__ ent,
                                                           int64_t ld_ent, const int64_t* __restrict__ cand, int k,
                                                           const int64_t* __restrict__ order,
                                                           const int64_t* __restrict__ seg_ptr, int64_t nseg, int d,
                                                           const float* __restrict__ s, int64_t lds,
                                                           const float* __restrict__ g, int64_t ldg, float* d_ent,
                                                           int64_t ld_dent) {
  constexpr int P = KIND == K_ROTATE ? 2 : 1;
  const int lane = threadIdx.x & 63;
  // the wave's group, known to be the same in every lane: its bookkeeping goes to the scalar unit
  const int64_t u = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (u >= nseg) return;
  const int64_t p0 = seg_ptr[u], p1 = seg_ptr[u + 1];
  if (p0 >= p1) return;  // entity without pairs (seg_ptr may have one slot per entity)
  const int64_t row = cand[order[p0]];  // order indexes the flattened [n, k] candidate matrix
  const int unit = KIND == K_ROTATE ? d / 2 : d;
  const float* e = ent + row * ld_ent;
  float4 ev[NCH][P], acc[NCH][P];
  int off[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    off[ch] = min(ch * 256 + lane * 4, unit - 4);
#pragma unroll
    for (int pl = 0; pl < P; ++pl) {
      ev[ch][pl] = ld4(e + off[ch] + pl * unit);
      acc[ch][pl] = f4(0.f);
    }
  }
  // D pairs at a time: their indexes were fetched during the previous batch, their gradients /
  // norms and query rows (the 2-MB query block is L2 resident, so several rows in flight cost
  // nothing here) are requested together, then accumulated in the order of `order`.
  constexpr int D = NCH * P <= 4 ? 4 : (NCH * P <= 8 ? 2 : 1);
  auto accumulate = [&](const float4 (&qv)[NCH][P], float gc, float inv) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const float4 a = qv[ch][0], b = ev[ch][0];
      const float4 ai = P > 1 ? qv[ch][P - 1] : a, bi = P > 1 ? ev[ch][P - 1] : b;
      if (KIND == K_DOT) {  // d score / d e = q
        acc[ch][0].x += gc * a.x; acc[ch][0].y += gc * a.y; acc[ch][0].z += gc * a.z; acc[ch][0].w += gc * a.w;
      } else {  // d score / d e = -(d score / d q)
        float gr[4], gi[4];
        grad_q<KIND>(l1, sigma, inv, gc, a.x, ai.x, b.x, bi.x, gr[0], gi[0]);
        grad_q<KIND>(l1, sigma, inv, gc, a.y, ai.y, b.y, bi.y, gr[1], gi[1]);
        grad_q<KIND>(l1, sigma, inv, gc, a.z, ai.z, b.z, bi.z, gr[2], gi[2]);
        grad_q<KIND>(l1, sigma, inv, gc, a.w, ai.w, b.w, bi.w, gr[3], gi[3]);
        acc[ch][0].x -= gr[0]; acc[ch][0].y -= gr[1]; acc[ch][0].z -= gr[2]; acc[ch][0].w -= gr[3];
        if (P > 1) {
          acc[ch][P - 1].x -= gi[0]; acc[ch][P - 1].y -= gi[1]; acc[ch][P - 1].z -= gi[2]; acc[ch][P - 1].w -= gi[3];
        }
      }
    }
  };
  int64_t pr[D];
#pragma unroll
  for (int u = 0; u < D; ++u) pr[u] = order[p0 + u < p1 ? p0 + u : p1 - 1];
  for (int64_t t = p0; t < p1; t += D) {
    float gc[D], inv[D];
    float4 qv[D][NCH][P];
#pragma unroll
    for (int u = 0; u < D; ++u) {  // (a slot past the group's end repeats its last pair with gradient 0)
      const int64_t pair = pr[u], i = pair / k, c = pair - i * k;
      gc[u] = t + u < p1 ? g[i * ldg + c] : 0.f;
      inv[u] = inv_norm<KIND>(l1, s, i * lds + c);
      const float* qi = q + i * ldq;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
        for (int pl = 0; pl < P; ++pl) qv[u][ch][pl] = ld4(qi + off[ch] + pl * unit);
    }
#pragma unroll
    for (int u = 0; u < D; ++u) pr[u] = order[t + D + u < p1 ? t + D + u : p1 - 1];
#pragma unroll
    for (int u = 0; u < D; ++u)
      if (gc[u] != 0.f) accumulate(qv[u], gc[u], inv[u]);
  }
  float* de = d_ent + row * ld_dent;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int kk = ch * 256 + lane * 4;
    if (kk >= unit) continue;
#pragma unroll
    for (int pl = 0; pl < P; ++pl) {
      float4* p = reinterpret_cast<float4*>(de + kk + pl * unit);
      float4 v = *p;
      v.x += acc[ch][pl].x; v.y += acc[ch][pl].y; v.z += acc[ch][pl].z; v.w += acc[ch][pl].w;
      *p = v;
    }
  }
}

// scalar fallback (any d, any alignment): dq through per-wave LDS partials, d_ent atomics
template <int KIND>
__global__ void __launch_bounds__(NT) cand_bwd_scalar_kernel(bool l1, float sigma, const float* __restrict__ q,
                                                             int64_t ldq, const float* __restrict__ ent,
                                                             int64_t ld_ent, const int64_t* __restrict__ cand,
                                                             int64_t ldc, int k, int d, const float* __restrict__ s,
                                                             int64_t lds, const float* __restrict__ g, int64_t ldg,
                                                             float* dq, int64_t lddq, float* d_ent, int64_t ld_dent) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* qs = sh;        // d
  float* part = sh + d;  // NW x d per-wave dq partials
  const int64_t i = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int unit = KIND == K_ROTATE ? d / 2 : d;
  for (int t = threadIdx.x; t < d; t += NT) qs[t] = q[i * ldq + t];
  for (int t = threadIdx.x; t < NW * d; t += NT) part[t] = 0.f;
  __syncthreads();
  float* pw = part + w * d;
  const int64_t* ci = cand + i * ldc;
  for (int c = w; c < k; c += NW) {
    const float gc = g[i * ldg + c];
    if (gc == 0.f) continue;
    const float inv = inv_norm<KIND>(l1, s, i * lds + c);
    const int64_t row = ci[c];
    const float* e = ent + row * ld_ent;
    float* de = d_ent ? d_ent + row * ld_dent : nullptr;
    for (int t = lane; t < unit; t += 64) {
      const float qi = KIND == K_ROTATE ? qs[t + unit] : 0.f, ei = KIND == K_ROTATE ? e[t + unit] : 0.f;
      float gr = 0.f, gi = 0.f;
      grad_q<KIND>(l1, sigma, inv, gc, qs[t], qi, e[t], ei, gr, gi);
      pw[t] += gr;
      if (KIND == K_ROTATE) pw[t + unit] += gi;
      if (de) {
        atomicAdd(de + t, KIND == K_DOT ? gc * qs[t] : -gr);
        if (KIND == K_ROTATE) atomicAdd(de + t + unit, -gi);
      }
    }
  }
  __syncthreads();
  if (dq) {
    for (int t = threadIdx.x; t < d; t += NT) {
      float v = 0.f;
#pragma unroll
      for (int u = 0; u < NW; ++u) v += part[u * d + t];
      dq[i * lddq + t] = v;
    }
  }
}

__global__ void bucket_scatter_kernel(const int64_t* __restrict__ idx, int64_t n, int64_t* cursor,
                                      int64_t* __restrict__ order) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  order[atomicAdd(reinterpret_cast<unsigned long long*>(cursor + idx[t]), 1ull)] = t;
}

// counts[idx[t]] += 1 (indexes outside [0, nbuckets) are not counted)
__global__ void bucket_count_kernel(const int64_t* __restrict__ idx, int64_t n, int64_t nbuckets, int64_t* counts) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t b = idx[t];
  if (b >= 0 && b < nbuckets) atomicAdd(reinterpret_cast<unsigned long long*>(counts + b), 1ull);
}

// Rows of ids sorted ascending inside LDS: a bitonic network over the keys id << 13 | position
// (ties keep their order: a stable sort), padded with the largest key to npad, a power of two.
// sorted[i, :] = the ids, col[i, :] = the positions they came from.
__global__ void __launch_bounds__(512) sort_rows_kernel(const int64_t* __restrict__ x, int64_t ldx, int k, int npad,
                                                        int64_t* __restrict__ sorted, int64_t* __restrict__ col) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long key[];
  const int64_t i = blockIdx.x;
  for (int t = threadIdx.x; t < npad; t += 512)
    key[t] = t < k ? ((unsigned long long)x[i * ldx + t] << 13) | (unsigned)t : ~0ull;
  __syncthreads();
  for (int size = 2; size <= npad; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < npad / 2; t += 512) {  // pair t: lo has bit `stride` clear
        const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
        const unsigned long long a = key[lo], b = key[hi];
        if ((a > b) == ((lo & size) == 0)) {
          key[lo] = b;
          key[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int t = threadIdx.x; t < k; t += 512) {
    const unsigned long long v = key[t];
    sorted[i * k + t] = (int64_t)v >> 13;
    col[i * k + t] = (int64_t)(v & 8191ull);
  }
}

// The same sort for rows of at most 2,048 ids with four consecutive keys per thread in registers:
// compare-exchanges at distance 1 and 2 stay inside a thread, distances 4 .. 128 are lane
// exchanges inside a wave (no barrier), only distances >= 256 go through LDS -- 6 of the 66 stages
// of a 2,048-key network.  blockDim.x = npad / 4 (a power of two, at most 512).  KeyT: 64-bit keys
// id << 13 | position, or 32-bit keys id << 11 | position for ids below 2^21 (half the lane
// exchanges, v_min_u32 / v_max_u32 instead of 64-bit compares and selects: 30 -> 21 us for 512
// rows of 1,025); there ids outside [0, id_bound) are clamped into it.
template <typename KeyT>
__global__ void __launch_bounds__(512) sort_rows4_kernel(const int64_t* __restrict__ x, int64_t ldx, int k, int npad,
                                                         int64_t id_bound, int64_t* __restrict__ sorted,
                                                         int64_t* __restrict__ col) {
  constexpr bool NARROW = sizeof(KeyT) == 4;
  constexpr int POS_BITS = NARROW ? 11 : 13;
  __shared__ KeyT key[2048];
  const int64_t i = blockIdx.x;
  const int t = threadIdx.x, g0 = 4 * t;
  KeyT v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int g = g0 + e;
    int64_t id = g < k ? x[i * ldx + g] : 0;
    if (NARROW) id = id < 0 ? 0 : (id >= id_bound ? id_bound - 1 : id);
    v[e] = g < k ? (KeyT)(((unsigned long long)id << POS_BITS) | (unsigned)g) : (KeyT)~0ull;
  }
  auto cx = [](KeyT& a, KeyT& b, bool up) {  // a at the lower position
    if ((a > b) == up) {
      const KeyT c = a;
      a = b;
      b = c;
    }
  };
  for (int size = 2; size <= npad; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride == 1) {
        cx(v[0], v[1], (g0 & size) == 0);
        cx(v[2], v[3], ((g0 + 2) & size) == 0);
      } else if (stride == 2) {
        cx(v[0], v[2], (g0 & size) == 0);
        cx(v[1], v[3], ((g0 + 1) & size) == 0);
      } else {
        // the partner thread holds the keys at distance `stride`: the lower position keeps the
        // smaller key of an ascending pair (positions g and g + stride lie in the same `size` block)
        const bool keep_min = ((g0 & stride) == 0) == ((g0 & size) == 0);
        KeyT o[4];
        if (stride < 256) {
          const int lane_xor = stride >> 2;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (NARROW) {
              o[e] = (KeyT)__shfl_xor((unsigned)v[e], lane_xor, 64);
            } else {
              const unsigned lo = __shfl_xor((unsigned)v[e], lane_xor, 64);
              const unsigned hi = __shfl_xor((unsigned)((unsigned long long)v[e] >> 32), lane_xor, 64);
              o[e] = (KeyT)(((unsigned long long)hi << 32) | lo);
            }
          }
        } else {
          __syncthreads();  // the previous round's reads are done
#pragma unroll
          for (int e = 0; e < 4; ++e) key[g0 + e] = v[e];
          __syncthreads();
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = key[(g0 + e) ^ stride];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = keep_min ? (v[e] < o[e] ? v[e] : o[e]) : (v[e] > o[e] ? v[e] : o[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int g = g0 + e;
    if (g < k) {
      sorted[i * k + g] = NARROW ? (int64_t)(v[e] >> POS_BITS) : ((int64_t)(unsigned long long)v[e] >> POS_BITS);
      col[i * k + g] = (int64_t)(v[e] & (KeyT)((1u << POS_BITS) - 1));
    }
  }
}

// The pairs (i, c) grouped by candidate entity, from candidate lists that are already sorted per
// row (sort_rows_kernel): a workgroup owns the entities [e0, e0 + R).  In every row its entities
// are one contiguous run, found by a binary search; the number of pairs before the run, summed over
// the rows, is where the workgroup's part of `order` starts -- so the counting sort needs no global
// counters: counts and write cursors of the R entities live in LDS.  seg_ptr[e] = first slot of
// entity e in order, order[slot] = i * k + col[i, position] (the pair in the caller's columns; the
// order inside a group is not specified).  Ids outside [0, E) are left out.
constexpr int GROUP_NT = 512, GROUP_RMAX = 1024;
__global__ void __launch_bounds__(GROUP_NT) group_sorted_rows_kernel(const int64_t* __restrict__ srt,
                                                                     const int64_t* __restrict__ col, int n, int k,
                                                                     int64_t E, int R, int64_t* __restrict__ seg_ptr,
                                                                     int64_t* __restrict__ order) {
  extern __shared__ int run_lo[];  // [n] first position of the run, then [n] its end
  __shared__ int count[GROUP_RMAX], cursor[GROUP_RMAX];
  __shared__ long long part[GROUP_NT / 64];
  int* run_hi = run_lo + n;
  const int64_t e0 = (int64_t)blockIdx.x * R, e1 = e0 + R < E ? e0 + R : E;
  const int nr = (int)(e1 - e0);
  for (int r = threadIdx.x; r < nr; r += GROUP_NT) count[r] = 0;
  __syncthreads();
  long long before = 0;
  for (int i = threadIdx.x; i < n; i += GROUP_NT) {
    const int64_t* row = srt + (int64_t)i * k;
    int a = 0, b = k;
    while (a < b) {  // first position with an id >= e0
      const int m = (a + b) >> 1;
      if (row[m] < e0) a = m + 1;
      else b = m;
    }
    int j = a;
    for (; j < k; ++j) {
      const int64_t e = row[j];
      if (e < e0 || e >= e1) break;
      atomicAdd(&count[(int)(e - e0)], 1);
    }
    run_lo[i] = a;
    run_hi[i] = j;
    before += a;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) before += __shfl_xor(before, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = before;
  __syncthreads();
  long long base = 0;
#pragma unroll
  for (int w = 0; w < GROUP_NT / 64; ++w) base += part[w];
  if (threadIdx.x < 64) {  // exclusive scan of the counts: lane l takes `per` consecutive entities
    const int per = (nr + 63) / 64, r0 = threadIdx.x * per, r1 = r0 + per < nr ? r0 + per : nr;
    int sum = 0;
    for (int r = r0; r < r1; ++r) sum += count[r];
    int incl = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off, 64);
      if ((int)threadIdx.x >= off) incl += v;
    }
    int run = incl - sum;
    for (int r = r0; r < r1; ++r) {
      cursor[r] = run;
      seg_ptr[e0 + r] = base + run;
      run += count[r];
    }
    if (threadIdx.x == 63 && e1 == E) seg_ptr[E] = base + incl;
  }
  __syncthreads();
  const int64_t total = (int64_t)n * k;
  for (int i = threadIdx.x; i < n; i += GROUP_NT) {
    const int64_t* row = srt + (int64_t)i * k;
    const int64_t* ci = col + (int64_t)i * k;
    for (int j = run_lo[i]; j < run_hi[i]; ++j) {
      const int64_t slot = base + atomicAdd(&cursor[(int)(row[j] - e0)], 1);
      if (slot < total) order[slot] = (int64_t)i * k + ci[j];
    }
  }
}

int kind_of(int model) {
  switch (model) {
    case KGE_COMPLEX:
    case KGE_DISTMULT:
    case KGE_RESCAL:
    case KGE_CP:  // the caller passes the entity-row window (cp.py:17-19) as ent
    case KGE_SIMPLE: return K_DOT;
    case KGE_TRANSE: return K_TRANSE;
    case KGE_ROTATE: return K_ROTATE;
    default: return -1;
  }
}

// chunks of 256 elements per lane row slice: 1, 2, 4 or 8 (unit <= 2048); 0 = unsupported
int nch_of(int unit) {
  const int c = (unit + 255) / 256;
  return c <= 1 ? 1 : c <= 2 ? 2 : c <= 4 ? 4 : c <= 8 ? 8 : 0;
}

template <template <int, int> class F, int KIND, typename... A>
void dispatch_nch(int nch, A&&... a) {
  switch (nch) {
    case 1: F<KIND, 1>::run(a...); break;
    case 2: F<KIND, 2>::run(a...); break;
    case 4: F<KIND, 4>::run(a...); break;
    default: F<KIND, 8>::run(a...); break;
  }
}

template <int KIND, int NCH>
struct LaunchQ {
  static void run(dim3 grid, size_t sh, hipStream_t st, bool l1, float sigma, const float* q, int64_t ldq,
                  const float* ent, int64_t ld_ent, const int64_t* cand, int64_t ldc, const int64_t* col,
                  int64_t ldcol, int k, int d, const float* s, int64_t lds, const float* g, int64_t ldg, float* dq,
                  int64_t lddq) {
    cand_bwd_q_kernel<KIND, NCH><<<grid, dim3(NT), sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, k,
                                                             d, s, lds, g, ldg, dq, lddq);
  }
};

template <int KIND, int NCH>
struct LaunchF {
  static void run(dim3 grid, hipStream_t st, bool l1, float sigma, const float* q, int64_t ldq, const float* ent,
                  int64_t ld_ent, const int64_t* cand, int64_t ldc, const int64_t* col, int64_t ldcol, int k, int d,
                  float* out, int64_t ldo) {
    cand_fwd_kernel<KIND, NCH><<<grid, dim3(NT), 0, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, k, d,
                                                          out, ldo);
  }
};

template <int KIND, int NCH>
struct LaunchE {
  static void run(dim3 grid, hipStream_t st, bool l1, float sigma, const float* q, int64_t ldq, const float* ent,
                  int64_t ld_ent, const int64_t* cand, int k, const int64_t* order, const int64_t* seg_ptr,
                  int64_t nseg, int d, const float* s, int64_t lds, const float* g, int64_t ldg, float* d_ent,
                  int64_t ld_dent) {
    cand_bwd_ent_kernel<KIND, NCH><<<grid, dim3(256), 0, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, k, order,
                                                               seg_ptr, nseg, d, s, lds, g, ldg, d_ent, ld_dent);
  }
};

}  // namespace

static int score_cand_impl(int model, float l_norm, int dir, const float* q, int64_t ldq, const float* ent,
                           int64_t ld_ent, const int64_t* cand, int64_t ldc, const int64_t* col, int64_t ldcol,
                           int64_t n, int64_t k, int d, float* out, int64_t ldo, void* stream) {
  const int kind = kind_of(model);
  KGE_REQUIRE(kind >= 0 && (dir == KGE_DIR_SP || dir == KGE_DIR_PO) && (l_norm == 1.f || l_norm == 2.f));
  KGE_REQUIRE(n >= 0 && k >= 0 && d > 0 && d <= 4096 && n < (1LL << 31) && k < (1LL << 31));
  KGE_REQUIRE(q && ent && cand && out && ldq >= d && ld_ent >= d && ldc >= k && ldo >= k);
  KGE_REQUIRE(kind != K_ROTATE || d % 2 == 0);
  if (n == 0 || k == 0) return 0;
  hipStream_t st = as_stream(stream);
  const bool l1 = l_norm == 1.f;
  const float sigma = dir == KGE_DIR_SP ? 1.f : -1.f;
  const int unit = kind == K_ROTATE ? d / 2 : d;
  const bool vec = unit % 4 == 0 && ld_ent % 4 == 0 && aligned16(ent);
  const size_t sh = (size_t)d * sizeof(float);
  const dim3 grid((unsigned)n), block(NT);
  const int nch = nch_of(unit);
  if (vec && nch && ldq % 4 == 0 && aligned16(q)) {  // rows and query slices as float4 in registers
    if (kind == K_DOT)
      dispatch_nch<LaunchF, K_DOT>(nch, grid, st, l1, sigma, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, (int)k, d, out,
                                   ldo);
    else if (kind == K_TRANSE)
      dispatch_nch<LaunchF, K_TRANSE>(nch, grid, st, l1, sigma, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, (int)k, d,
                                      out, ldo);
    else
      dispatch_nch<LaunchF, K_ROTATE>(nch, grid, st, l1, sigma, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, (int)k, d,
                                      out, ldo);
    KGE_CHECK_LAUNCH();
    return 0;
  }
  auto go = [&](auto kind_tag) {
    constexpr int K = decltype(kind_tag)::value;
    if (vec)
      cand_kernel<K, true><<<grid, block, sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, (int)k, d,
                                                    out, ldo);
    else
      cand_kernel<K, false><<<grid, block, sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, (int)k, d,
                                                     out, ldo);
  };
  if (kind == K_DOT)
    go(std::integral_constant<int, K_DOT>());
  else if (kind == K_TRANSE)
    go(std::integral_constant<int, K_TRANSE>());
  else
    go(std::integral_constant<int, K_ROTATE>());
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_score_cand(int model, float l_norm, int dir, const float* q, int64_t ldq, const float* ent,
                              int64_t ld_ent, const int64_t* cand, int64_t ldc, int64_t n, int64_t k, int d, float* out,
                              int64_t ldo, void* stream) {
  return score_cand_impl(model, l_norm, dir, q, ldq, ent, ld_ent, cand, ldc, nullptr, 0, n, k, d, out, ldo, stream);
}

extern "C" int kge_score_cand_ordered(int model, float l_norm, int dir, const float* q, int64_t ldq, const float* ent,
                                      int64_t ld_ent, const int64_t* cand, int64_t ldc, const int64_t* col,
                                      int64_t ldcol, int64_t n, int64_t k, int d, float* out, int64_t ldo,
                                      void* stream) {
  KGE_REQUIRE(col && ldcol >= k);
  return score_cand_impl(model, l_norm, dir, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, n, k, d, out, ldo, stream);
}

static int score_cand_bwd_impl(int model, float l_norm, int dir, const float* q, int64_t ldq, const float* ent,
                               int64_t ld_ent, const int64_t* cand, int64_t ldc, const int64_t* col, int64_t ldcol,
                               int64_t n, int64_t k, int d, const float* s, int64_t lds, const float* g, int64_t ldg,
                               float* dq, int64_t lddq, float* d_ent, int64_t ld_dent, void* stream) {
  const int kind = kind_of(model);
  KGE_REQUIRE(kind >= 0 && (dir == KGE_DIR_SP || dir == KGE_DIR_PO) && (l_norm == 1.f || l_norm == 2.f));
  KGE_REQUIRE(n >= 0 && k >= 0 && d > 0 && d <= 3584 && n < (1LL << 31) && k < (1LL << 31));
  KGE_REQUIRE(q && ent && cand && g && ldq >= d && ld_ent >= d && ldc >= k && ldg >= k);
  KGE_REQUIRE(!dq || lddq >= d);
  KGE_REQUIRE(!d_ent || ld_dent >= d);
  KGE_REQUIRE(kind == K_DOT || (s && lds >= k));
  KGE_REQUIRE(kind != K_ROTATE || d % 2 == 0);
  if (n == 0 || (!dq && !d_ent)) return 0;
  hipStream_t st = as_stream(stream);
  const bool l1 = l_norm == 1.f;
  const float sigma = dir == KGE_DIR_SP ? 1.f : -1.f;
  const int unit = kind == K_ROTATE ? d / 2 : d;
  const int nch = nch_of(unit);
  const dim3 grid((unsigned)n);
  // (the vector kernel's cross-wave reduction takes NW x d floats of LDS: up to the 64 KB every
  // kernel may use without asking, d <= 2048)
  if (!d_ent && nch && unit % 4 == 0 && ldq % 4 == 0 && ld_ent % 4 == 0 && aligned16(q) && aligned16(ent) &&
      (size_t)NW * d * sizeof(float) <= 65536) {
    const size_t sh = (size_t)NW * d * sizeof(float);
    if (kind == K_DOT)
      dispatch_nch<LaunchQ, K_DOT>(nch, grid, sh, st, l1, sigma, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, (int)k, d,
                                   s, lds, g, ldg, dq, lddq);
    else if (kind == K_TRANSE)
      dispatch_nch<LaunchQ, K_TRANSE>(nch, grid, sh, st, l1, sigma, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, (int)k,
                                      d, s, lds, g, ldg, dq, lddq);
    else
      dispatch_nch<LaunchQ, K_ROTATE>(nch, grid, sh, st, l1, sigma, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, (int)k,
                                      d, s, lds, g, ldg, dq, lddq);
    KGE_CHECK_LAUNCH();
    return 0;
  }
  if (col) return KGE_ERR_ALIGN;  // ordered lists are served by the vector kernel only
  const size_t sh = (size_t)(1 + NW) * d * sizeof(float);
  static std::atomic<bool> lds_ok[3][KGE_MAX_DEVICES];
  int fi = 0;
  for (const void* f : {(const void*)cand_bwd_scalar_kernel<K_DOT>, (const void*)cand_bwd_scalar_kernel<K_TRANSE>,
                        (const void*)cand_bwd_scalar_kernel<K_ROTATE>})
    if (const int e = kge_allow_lds(f, (1 + NW) * 3584 * 4, lds_ok[fi++])) return e;
  if (kind == K_DOT)
    cand_bwd_scalar_kernel<K_DOT><<<grid, dim3(NT), sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, (int)k, d, s,
                                                              lds, g, ldg, dq, lddq, d_ent, ld_dent);
  else if (kind == K_TRANSE)
    cand_bwd_scalar_kernel<K_TRANSE><<<grid, dim3(NT), sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, (int)k, d,
                                                                 s, lds, g, ldg, dq, lddq, d_ent, ld_dent);
  else
    cand_bwd_scalar_kernel<K_ROTATE><<<grid, dim3(NT), sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, (int)k, d,
                                                                 s, lds, g, ldg, dq, lddq, d_ent, ld_dent);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_score_cand_bwd(int model, float l_norm, int dir, const float* q, int64_t ldq, const float* ent,
                                  int64_t ld_ent, const int64_t* cand, int64_t ldc, int64_t n, int64_t k, int d,
                                  const float* s, int64_t lds, const float* g, int64_t ldg, float* dq, int64_t lddq,
                                  float* d_ent, int64_t ld_dent, void* stream) {
  return score_cand_bwd_impl(model, l_norm, dir, q, ldq, ent, ld_ent, cand, ldc, nullptr, 0, n, k, d, s, lds, g, ldg, dq,
                             lddq, d_ent, ld_dent, stream);
}

extern "C" int kge_score_cand_bwd_q_ordered(int model, float l_norm, int dir, const float* q, int64_t ldq,
                                            const float* ent, int64_t ld_ent, const int64_t* cand, int64_t ldc,
                                            const int64_t* col, int64_t ldcol, int64_t n, int64_t k, int d,
                                            const float* s, int64_t lds, const float* g, int64_t ldg, float* dq,
                                            int64_t lddq, void* stream) {
  KGE_REQUIRE(col && ldcol >= k && dq);
  return score_cand_bwd_impl(model, l_norm, dir, q, ldq, ent, ld_ent, cand, ldc, col, ldcol, n, k, d, s, lds, g, ldg, dq,
                             lddq, nullptr, 0, stream);
}

extern "C" int kge_score_cand_bwd_ent(int model, float l_norm, int dir, const float* q, int64_t ldq,
                                      const float* ent, int64_t ld_ent, const int64_t* cand, int64_t n, int64_t k,
                                      int d, const int64_t* order, const int64_t* seg_ptr, int64_t nseg,
                                      const float* s, int64_t lds, const float* g, int64_t ldg, float* d_ent,
                                      int64_t ld_dent, void* stream) {
  const int kind = kind_of(model);
  KGE_REQUIRE(kind >= 0 && (dir == KGE_DIR_SP || dir == KGE_DIR_PO) && (l_norm == 1.f || l_norm == 2.f));
  KGE_REQUIRE(n >= 0 && k > 0 && d > 0 && nseg >= 0 && n * k < (1LL << 62));
  KGE_REQUIRE(q && ent && cand && order && seg_ptr && g && d_ent && ldq >= d && ld_ent >= d && ldg >= k &&
              ld_dent >= d);
  KGE_REQUIRE(kind == K_DOT || (s && lds >= k));
  KGE_REQUIRE(kind != K_ROTATE || d % 2 == 0);
  const int unit = kind == K_ROTATE ? d / 2 : d;
  const int nch = nch_of(unit);
  if (!nch || unit % 4 != 0 || ldq % 4 != 0 || ld_ent % 4 != 0 || ld_dent % 4 != 0 || !aligned16(q) ||
      !aligned16(ent) || !aligned16(d_ent))
    return KGE_ERR_ALIGN;
  if (nseg == 0) return 0;
  hipStream_t st = as_stream(stream);
  const bool l1 = l_norm == 1.f;
  const float sigma = dir == KGE_DIR_SP ? 1.f : -1.f;
  const dim3 grid((unsigned)((nseg + 3) / 4));
  if (kind == K_DOT)
    dispatch_nch<LaunchE, K_DOT>(nch, grid, st, l1, sigma, q, ldq, ent, ld_ent, cand, (int)k, order, seg_ptr, nseg, d,
                                 s, lds, g, ldg, d_ent, ld_dent);
  else if (kind == K_TRANSE)
    dispatch_nch<LaunchE, K_TRANSE>(nch, grid, st, l1, sigma, q, ldq, ent, ld_ent, cand, (int)k, order, seg_ptr, nseg,
                                    d, s, lds, g, ldg, d_ent, ld_dent);
  else
    dispatch_nch<LaunchE, K_ROTATE>(nch, grid, st, l1, sigma, q, ldq, ent, ld_ent, cand, (int)k, order, seg_ptr, nseg,
                                    d, s, lds, g, ldg, d_ent, ld_dent);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_bucket_scatter(const int64_t* idx, int64_t n, int64_t* cursor, int64_t* order, void* stream) {
  KGE_REQUIRE(n >= 0 && (n == 0 || (idx && cursor && order)));
  if (n == 0) return 0;
  bucket_scatter_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream)>>>(idx, n, cursor, order);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_bucket_count(const int64_t* idx, int64_t n, int64_t nbuckets, int64_t* counts, void* stream) {
  KGE_REQUIRE(n >= 0 && nbuckets >= 0 && (n == 0 || (idx && counts)));
  if (n == 0) return 0;
  bucket_count_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream)>>>(idx, n, nbuckets, counts);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_sort_rows(const int64_t* x, int64_t ldx, int64_t n, int64_t k, int64_t id_bound, int64_t* sorted,
                             int64_t* col, void* stream) {
  KGE_REQUIRE(n >= 0 && k >= 0 && k <= 8192 && n < (1LL << 31) && ldx >= k && id_bound >= 0);
  KGE_REQUIRE(n == 0 || k == 0 || (x && sorted && col));
  if (n == 0 || k == 0) return 0;
  int npad = 2;
  while (npad < k) npad <<= 1;
  if (npad <= 2048) {
    if (npad < 4) npad = 4;
    if (id_bound > 0 && id_bound <= (1LL << 21))
      sort_rows4_kernel<unsigned><<<dim3((unsigned)n), dim3(npad / 4), 0, as_stream(stream)>>>(x, ldx, (int)k, npad,
                                                                                             id_bound, sorted, col);
    else
      sort_rows4_kernel<unsigned long long><<<dim3((unsigned)n), dim3(npad / 4), 0, as_stream(stream)>>>(
          x, ldx, (int)k, npad, id_bound, sorted, col);
    KGE_CHECK_LAUNCH();
    return 0;
  }
  sort_rows_kernel<<<dim3((unsigned)n), dim3(512), (size_t)npad * 8, as_stream(stream)>>>(x, ldx, (int)k, npad, sorted,
                                                                                          col);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_group_sorted_rows(const int64_t* srt, const int64_t* col, int64_t n, int64_t k, int64_t nbuckets,
                                     int64_t* seg_ptr, int64_t* order, void* stream) {
  KGE_REQUIRE(n >= 0 && n <= 4096 && k >= 0 && k < (1LL << 31) && nbuckets > 0 && nbuckets < (1LL << 40) && seg_ptr);
  KGE_REQUIRE(n == 0 || k == 0 || (srt && col && order));
  int64_t r = (nbuckets + 255) / 256;
  r = r < 32 ? 32 : (r > GROUP_RMAX ? GROUP_RMAX : r);
  const int64_t nblocks = (nbuckets + r - 1) / r;
  KGE_REQUIRE(nblocks < (1LL << 31));
  group_sorted_rows_kernel<<<dim3((unsigned)nblocks), dim3(GROUP_NT), (size_t)(2 * n + 1) * sizeof(int),
                             as_stream(stream)>>>(srt, col, (int)n, (int)k, nbuckets, (int)r, seg_ptr, order);
  KGE_CHECK_LAUNCH();
  return 0;
}

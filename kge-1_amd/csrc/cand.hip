// Scores of each query against its OWN candidate list -- the negative-sampling hot path
// (TrainingJobNegativeSampling "triple" implementation, train.py:868-892: score_spo over the
// B x (1 + N) triples that share (s, p) or (p, o) with a positive), with score_spo's
// per-model semantics (kge_model.py:620-637):
//   out[i, c] = score(q_i, ent[cand[i, c]])
//     dot models : <q_i, e>                                   (q = prep(s, r) / prep(r, o))
//     TransE     : -|| sigma (q_i - e) + 1e-6 ||_p            (F.pairwise_distance,
//                  sigma = +1 for sp_ queries (s+p-o'), -1 for _po (s'+p-o), transe.py:221)
//     RotatE     : + sum_k |q_ik - e_k|_C  (p=1) / sqrt(sum |.|^2) (p=2)   (rotate.py:18-50)
// Nothing is shared between rows, so the kernel is a gather: one workgroup per query row,
// the query staged in LDS, each wave streams whole candidate rows (float4 per lane, two
// rows in flight) and reduces across the wave.  4*d bytes per scored triple; the FB15K-237
// table (14,541 x 1024 x 4 = 59.6 MB) stays resident in the 256 MB MALL across rows.
//
// Backward: dq_i = sum_c g_ic d score / d q (per-wave partials in LDS, no atomics), and
// d_ent[cand[i, c]] += g_ic d score / d e (fp32 atomics: candidates repeat across rows).
#include <type_traits>

#include "common.h"

namespace {

constexpr int NT = 512, NW = NT / 64;
enum { K_DOT = 0, K_TRANSE = 1, K_ROTATE = 2 };

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Per-element contribution to the reduction for (q, e) components.  For RotatE (re, im)
// pairs are handled by the caller.
template <int KIND>
__device__ __forceinline__ float elem(float q, float e, float sigma, bool l1) {
  if (KIND == K_DOT) return q * e;
  const float df = sigma * (q - e) + 1e-6f;
  return l1 ? fabsf(df) : df * df;
}

__device__ __forceinline__ float cabs_term(float dr, float di, bool l1) {
  const float sq = fmaf(di, di, dr * dr);
  return l1 ? sqrtf(sq) : sq;
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
                                                  const int64_t* __restrict__ cand, int64_t ldc, int k, int d,
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
    if (lane == 0) {
      out[i * ldo + c] = finish<KIND>(a1, l1);
      if (c2 < k) out[i * ldo + c2] = finish<KIND>(a2, l1);
    }
  }
}

// ---------------------------------------------------------------------------- backward
template <int KIND>
__global__ void __launch_bounds__(NT) cand_bwd_kernel(bool l1, float sigma, const float* __restrict__ q, int64_t ldq,
                                                      const float* __restrict__ ent, int64_t ld_ent,
                                                      const int64_t* __restrict__ cand, int64_t ldc, int k, int d,
                                                      const float* __restrict__ s, int64_t lds,
                                                      const float* __restrict__ g, int64_t ldg, float* dq,
                                                      int64_t lddq, float* d_ent, int64_t ld_dent) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* qs = sh;               // d
  float* part = sh + d;         // NW x d per-wave dq partials
  const int64_t i = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int t = threadIdx.x; t < d; t += NT) qs[t] = q[i * ldq + t];
  for (int t = threadIdx.x; t < NW * d; t += NT) part[t] = 0.f;
  __syncthreads();
  float* pw = part + w * d;
  const int64_t* ci = cand + i * ldc;
  for (int c = w; c < k; c += NW) {
    const float gc = g[i * ldg + c];
    if (gc == 0.f) continue;
    const int64_t row = ci[c];
    const float* e = ent + row * ld_ent;
    float* de = d_ent ? d_ent + row * ld_dent : nullptr;
    if (KIND == K_DOT) {
      for (int t = lane; t < d; t += 64) {
        pw[t] += gc * e[t];
        if (de) atomicAdd(de + t, gc * qs[t]);
      }
    } else if (KIND == K_TRANSE) {
      // score = -||diff||, diff = sigma (q - e) + eps;  d/dq = -sigma * dnorm/ddiff
      const float nrm = -s[i * lds + c];  // L2 norm from the forward score
      const float inv = (!l1 && nrm > 0.f) ? 1.f / nrm : 0.f;
      for (int t = lane; t < d; t += 64) {
        const float df = sigma * (qs[t] - e[t]) + 1e-6f;
        const float dn = l1 ? (df > 0.f ? 1.f : (df < 0.f ? -1.f : 0.f)) : df * inv;
        const float gq = -gc * sigma * dn;
        pw[t] += gq;
        if (de) atomicAdd(de + t, -gq);
      }
    } else {  // RotatE: score = sum |q - e|_C (L1) or sqrt(sum |q - e|^2) (L2)
      const int h = d / 2;
      const float nrm = s[i * lds + c];
      const float inv = (!l1 && nrm > 0.f) ? 1.f / nrm : 0.f;
      for (int t = lane; t < h; t += 64) {
        const float dr = qs[t] - e[t], di = qs[t + h] - e[t + h];
        float sr, si;
        if (l1) {
          const float a = sqrtf(fmaf(di, di, dr * dr));
          const float ia = a > 0.f ? 1.f / a : 0.f;
          sr = dr * ia;
          si = di * ia;
        } else {
          sr = dr * inv;
          si = di * inv;
        }
        pw[t] += gc * sr;
        pw[t + h] += gc * si;
        if (de) {
          atomicAdd(de + t, -gc * sr);
          atomicAdd(de + t + h, -gc * si);
        }
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

int kind_of(int model) {
  switch (model) {
    case KGE_COMPLEX:
    case KGE_DISTMULT:
    case KGE_RESCAL: return K_DOT;
    case KGE_TRANSE: return K_TRANSE;
    case KGE_ROTATE: return K_ROTATE;
    default: return -1;
  }
}

}  // namespace

extern "C" int kge_score_cand(int model, float l_norm, int dir, const float* q, int64_t ldq, const float* ent,
                              int64_t ld_ent, const int64_t* cand, int64_t ldc, int64_t n, int64_t k, int d, float* out,
                              int64_t ldo, void* stream) {
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
  auto go = [&](auto kind_tag) {
    constexpr int K = decltype(kind_tag)::value;
    if (vec)
      cand_kernel<K, true><<<grid, block, sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, (int)k, d, out, ldo);
    else
      cand_kernel<K, false><<<grid, block, sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, (int)k, d, out, ldo);
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

extern "C" int kge_score_cand_bwd(int model, float l_norm, int dir, const float* q, int64_t ldq, const float* ent,
                                  int64_t ld_ent, const int64_t* cand, int64_t ldc, int64_t n, int64_t k, int d,
                                  const float* s, int64_t lds, const float* g, int64_t ldg, float* dq, int64_t lddq,
                                  float* d_ent, int64_t ld_dent, void* stream) {
  const int kind = kind_of(model);
  KGE_REQUIRE(kind >= 0 && (dir == KGE_DIR_SP || dir == KGE_DIR_PO) && (l_norm == 1.f || l_norm == 2.f));
  KGE_REQUIRE(n >= 0 && k >= 0 && d > 0 && d <= 3584 && n < (1LL << 31) && k < (1LL << 31));
  KGE_REQUIRE(q && ent && cand && g && ldq >= d && ld_ent >= d && ldc >= k && ldg >= k);
  KGE_REQUIRE(!dq || lddq >= d);
  KGE_REQUIRE(!d_ent || ld_dent >= d);
  KGE_REQUIRE(kind == K_DOT || (s && lds >= k));
  KGE_REQUIRE(kind != K_ROTATE || d % 2 == 0);
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  const bool l1 = l_norm == 1.f;
  const float sigma = dir == KGE_DIR_SP ? 1.f : -1.f;
  const size_t sh = (size_t)(1 + NW) * d * sizeof(float);
  static bool attr = false;
  if (!attr) {
    for (const void* f : {(const void*)cand_bwd_kernel<K_DOT>, (const void*)cand_bwd_kernel<K_TRANSE>,
                          (const void*)cand_bwd_kernel<K_ROTATE>}) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (1 + NW) * 3584 * 4);
      if (e != hipSuccess) return (int)e;
    }
    attr = true;
  }
  const dim3 grid((unsigned)n), block(NT);
  if (kind == K_DOT)
    cand_bwd_kernel<K_DOT><<<grid, block, sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, (int)k, d, s, lds, g,
                                                    ldg, dq, lddq, d_ent, ld_dent);
  else if (kind == K_TRANSE)
    cand_bwd_kernel<K_TRANSE><<<grid, block, sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, (int)k, d, s, lds,
                                                       g, ldg, dq, lddq, d_ent, ld_dent);
  else
    cand_bwd_kernel<K_ROTATE><<<grid, block, sh, st>>>(l1, sigma, q, ldq, ent, ld_ent, cand, ldc, (int)k, d, s, lds,
                                                       g, ldg, dq, lddq, d_ent, ld_dent);
  KGE_CHECK_LAUNCH();
  return 0;
}

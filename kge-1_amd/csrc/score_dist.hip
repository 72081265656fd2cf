// All-entities distance scoring for TransE and RotatE: VALU
// work with no MFMA.  S[i, j] = sign * dist(Q[i], T[row(j)]).
//
// The reference materialises the pairwise difference tensor (rotate.py:41-60:
// n x m x d/2 floats, several times) or goes through torch.cdist (transe.py:19-21).
// Here a 64 x 64 output tile is register-blocked 4 x 4 per thread and the K dimension is
// streamed through LDS in K-major chunks, so nothing pairwise ever leaves registers.
//   L1      : sum_k |q_k - e_k|
//   L2      : sqrt(sum_k (q_k - e_k)^2)
//   ROT_L1  : sum_k sqrt(dre_k^2 + dim_k^2)      (k over the d/2 complex components)
//   ROT_L2  : sqrt(sum_k dre_k^2 + dim_k^2)
#include "common.h"

namespace {

constexpr int TM = 64, TN = 64, KC = 32, NT = 256;
constexpr int XLD = 68;  // K-major LDS row: 64 + 4 pad (16-B aligned, fewer write conflicts)

__host__ __device__ __forceinline__ bool is_rot(int kind) { return kind >= KGE_DIST_ROT_L1; }

// Stage a [64 rows][KC] chunk of X (rows r0.., cols k0..) into Xs[KC][64] (K-major).
// For rotate kinds the chunk is of complex components: re at col k, im at col k + h.
template <bool ROT>
__device__ __forceinline__ void stage(float* xs_re, float* xs_im, const float* __restrict__ x, int64_t ldx,
                                      const int64_t* __restrict__ rowmap, int r0, int nrows, int k0, int kdim,
                                      int h) {
  const int tid = threadIdx.x;
  const int kk = tid & 31;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int rr = (tid >> 5) + 8 * r;
    const int gr = r0 + rr, gk = k0 + kk;
    float vre = 0.f, vim = 0.f;
    if (gr < nrows && gk < kdim) {
      const int64_t row = rowmap ? rowmap[gr] : (int64_t)gr;
      const float* p = x + row * ldx;
      vre = p[gk];
      if (ROT) vim = p[gk + h];
    }
    xs_re[kk * XLD + rr] = vre;
    if (ROT) xs_im[kk * XLD + rr] = vim;
  }
}

template <int KIND>
__global__ void __launch_bounds__(NT) score_dist_kernel(float sign, const float* __restrict__ q, int64_t ldq,
                                                        const float* __restrict__ t, int64_t ldt,
                                                        const int64_t* __restrict__ tidx, int n, int m, int d,
                                                        float* __restrict__ s, int64_t lds) {
  constexpr bool ROT = KIND >= KGE_DIST_ROT_L1;
  __shared__ __attribute__((aligned(16))) float qs_re[KC * XLD];
  __shared__ __attribute__((aligned(16))) float ts_re[KC * XLD];
  __shared__ __attribute__((aligned(16))) float qs_im[ROT ? KC * XLD : 4];
  __shared__ __attribute__((aligned(16))) float ts_im[ROT ? KC * XLD : 4];
  const int i0 = blockIdx.y * TM, j0 = blockIdx.x * TN;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int kdim = ROT ? d / 2 : d;
  const int h = d / 2;
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;

  for (int k0 = 0; k0 < kdim; k0 += KC) {
    stage<ROT>(qs_re, qs_im, q, ldq, nullptr, i0, n, k0, kdim, h);
    stage<ROT>(ts_re, ts_im, t, ldt, tidx, j0, m, k0, kdim, h);
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < KC; ++kk) {
      const float4 qa = *reinterpret_cast<const float4*>(qs_re + kk * XLD + ty * 4);
      const float4 ta = *reinterpret_cast<const float4*>(ts_re + kk * XLD + tx * 4);
      const float qv[4] = {qa.x, qa.y, qa.z, qa.w};
      const float tv[4] = {ta.x, ta.y, ta.z, ta.w};
      if (ROT) {
        const float4 qb = *reinterpret_cast<const float4*>(qs_im + kk * XLD + ty * 4);
        const float4 tb = *reinterpret_cast<const float4*>(ts_im + kk * XLD + tx * 4);
        const float qw[4] = {qb.x, qb.y, qb.z, qb.w};
        const float tw[4] = {tb.x, tb.y, tb.z, tb.w};
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const float dr = qv[a] - tv[b], di = qw[a] - tw[b];
            const float sq = fmaf(di, di, dr * dr);
            if (KIND == KGE_DIST_ROT_L1)
              acc[a][b] += __builtin_amdgcn_sqrtf(sq);
            else
              acc[a][b] += sq;
          }
      } else {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const float df = qv[a] - tv[b];
            if (KIND == KGE_DIST_L1)
              acc[a][b] += fabsf(df);
            else
              acc[a][b] = fmaf(df, df, acc[a][b]);
          }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int i = i0 + ty * 4 + a;
    if (i >= n) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int j = j0 + tx * 4 + b;
      if (j >= m) continue;
      float v = acc[a][b];
      if (KIND == KGE_DIST_L2 || KIND == KGE_DIST_ROT_L2) v = sqrtf(v);
      s[(int64_t)i * lds + j] = sign * v;
    }
  }
}

// Generic backward (any layout; the L2 kinds without ready weights): per 64 x 64 tile, pass 1
// recomputes the distances (needed by L2 kinds), pass 2 forms per-pair gradient weights and
// accumulates per-(row, k) partial sums in LDS, flushed to global with one atomic add per
// (row, k) per tile.  Slow (LDS atomics per pair row); float4-readable layouts take
// score_dist_bwd2.hip instead.
template <int KIND>
__global__ void __launch_bounds__(NT) score_dist_bwd_kernel(float sign, const float* __restrict__ g, int64_t ldg,
                                                            const float* __restrict__ q, int64_t ldq,
                                                            const float* __restrict__ t, int64_t ldt,
                                                            const int64_t* __restrict__ tidx, int n, int m, int d,
                                                            float* dq, int64_t lddq, float* dt, int64_t lddt) {
  constexpr bool ROT = KIND >= KGE_DIST_ROT_L1;
  constexpr bool NEED_DIST = KIND == KGE_DIST_L2 || KIND == KGE_DIST_ROT_L2;
  __shared__ __attribute__((aligned(16))) float qs_re[KC * XLD];
  __shared__ __attribute__((aligned(16))) float ts_re[KC * XLD];
  __shared__ __attribute__((aligned(16))) float qs_im[ROT ? KC * XLD : 4];
  __shared__ __attribute__((aligned(16))) float ts_im[ROT ? KC * XLD : 4];
  __shared__ float gq_re[KC * XLD], gt_re[KC * XLD];
  __shared__ float gq_im[ROT ? KC * XLD : 4], gt_im[ROT ? KC * XLD : 4];
  const int i0 = blockIdx.y * TM, j0 = blockIdx.x * TN;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int kdim = ROT ? d / 2 : d;
  const int h = d / 2;

  float w[4][4];  // per-pair weight: sign * G (L1 kinds) or sign * G / dist (L2 kinds)
  float dist[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) dist[a][b] = 0.f;
  if (NEED_DIST) {
    for (int k0 = 0; k0 < kdim; k0 += KC) {
      stage<ROT>(qs_re, qs_im, q, ldq, nullptr, i0, n, k0, kdim, h);
      stage<ROT>(ts_re, ts_im, t, ldt, tidx, j0, m, k0, kdim, h);
      __syncthreads();
      for (int kk = 0; kk < KC; ++kk)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const float dr = qs_re[kk * XLD + ty * 4 + a] - ts_re[kk * XLD + tx * 4 + b];
            float sq = dr * dr;
            if (ROT) {
              const float di = qs_im[kk * XLD + ty * 4 + a] - ts_im[kk * XLD + tx * 4 + b];
              sq = fmaf(di, di, sq);
            }
            dist[a][b] += sq;
          }
      __syncthreads();
    }
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int i = i0 + ty * 4 + a, j = j0 + tx * 4 + b;
      float gv = (i < n && j < m) ? g[(int64_t)i * ldg + j] * sign : 0.f;
      if (NEED_DIST) {
        const float dd = sqrtf(dist[a][b]);
        gv = dd > 0.f ? gv / dd : 0.f;
      }
      w[a][b] = gv;
    }

  for (int k0 = 0; k0 < kdim; k0 += KC) {
    stage<ROT>(qs_re, qs_im, q, ldq, nullptr, i0, n, k0, kdim, h);
    stage<ROT>(ts_re, ts_im, t, ldt, tidx, j0, m, k0, kdim, h);
    for (int x = threadIdx.x; x < KC * XLD; x += NT) {
      gq_re[x] = 0.f;
      gt_re[x] = 0.f;
      if (ROT) {
        gq_im[x] = 0.f;
        gt_im[x] = 0.f;
      }
    }
    __syncthreads();
    for (int kk = 0; kk < KC; ++kk) {
      float pq_re[4] = {0.f, 0.f, 0.f, 0.f}, pq_im[4] = {0.f, 0.f, 0.f, 0.f};
      float pt_re[4] = {0.f, 0.f, 0.f, 0.f}, pt_im[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const float dr = qs_re[kk * XLD + ty * 4 + a] - ts_re[kk * XLD + tx * 4 + b];
          float gr, gi = 0.f;
          if (ROT) {
            const float di = qs_im[kk * XLD + ty * 4 + a] - ts_im[kk * XLD + tx * 4 + b];
            if (KIND == KGE_DIST_ROT_L1) {
              const float am = sqrtf(fmaf(di, di, dr * dr));
              const float f = am > 0.f ? w[a][b] / am : 0.f;
              gr = f * dr;
              gi = f * di;
            } else {
              gr = w[a][b] * dr;
              gi = w[a][b] * di;
            }
          } else if (KIND == KGE_DIST_L1) {
            gr = dr > 0.f ? w[a][b] : (dr < 0.f ? -w[a][b] : 0.f);
          } else {
            gr = w[a][b] * dr;
          }
          pq_re[a] += gr;
          pt_re[b] -= gr;
          if (ROT) {
            pq_im[a] += gi;
            pt_im[b] -= gi;
          }
        }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        atomicAdd(&gq_re[kk * XLD + ty * 4 + a], pq_re[a]);
        atomicAdd(&gt_re[kk * XLD + tx * 4 + a], pt_re[a]);
        if (ROT) {
          atomicAdd(&gq_im[kk * XLD + ty * 4 + a], pq_im[a]);
          atomicAdd(&gt_im[kk * XLD + tx * 4 + a], pt_im[a]);
        }
      }
    }
    __syncthreads();
    // flush: thread -> (row, k) pairs
    for (int x0 = threadIdx.x; x0 < KC * TM; x0 += NT) {
      const int kk = x0 / TM, rr = x0 % TM;
      const int x = kk * XLD + rr;
      const int gk = k0 + kk;
      if (gk >= kdim) continue;
      const int i = i0 + rr;
      if (dq && i < n) {
        atomicAdd(dq + (int64_t)i * lddq + gk, gq_re[x]);
        if (ROT) atomicAdd(dq + (int64_t)i * lddq + gk + h, gq_im[x]);
      }
      const int j = j0 + rr;
      if (dt && j < m) {
        const int64_t row = tidx ? tidx[j] : (int64_t)j;
        atomicAdd(dt + row * lddt + gk, gt_re[x]);
        if (ROT) atomicAdd(dt + row * lddt + gk + h, gt_im[x]);
      }
    }
    __syncthreads();
  }
}

}  // namespace

#ifdef KGE_DEV_BUILD  // libkgescore_dev.so only: A/B switch between the two kernels
static int g_dist_impl = 2;  // 2: production choice, 1: always this file's kernel, 3: always the tiled kernel
extern "C" int kge_dev_dist_impl(int impl) {
  const int old = g_dist_impl;
  if (impl >= 1 && impl <= 3) g_dist_impl = impl;
  return old;
}
#else
constexpr int g_dist_impl = 2;
#endif

extern "C" int kge_score_dist(int kind, float sign, const float* q, int64_t ldq, const float* t, int64_t ldt,
                              const int64_t* tidx, int64_t n, int64_t m, int d, float* s, int64_t lds,
                              void* stream) {
  KGE_REQUIRE(n >= 0 && m >= 0 && d > 0 && n < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE(q && t && s && ldq >= d && ldt >= d && lds >= m);
  KGE_REQUIRE(kind >= KGE_DIST_L1 && kind <= KGE_DIST_ROT_L2);
  KGE_REQUIRE(!is_rot(kind) || d % 2 == 0);
  if (n == 0 || m == 0) return 0;
  KGE_REQUIRE((n + TM - 1) / TM < 65536);
  hipStream_t st = as_stream(stream);
  // The register-tiled kernel (score_dist2.hip) when the layout allows -- except for RotatE-L1,
  // whose per-pair v_sqrt and second accumulator plane run faster on this file's kernel
  // (746 vs 843 us at B = 1024, E = 14,541, d = 512; the other kinds: 358-394 vs 433-498 us).
  if (g_dist_impl == 3 || (g_dist_impl == 2 && kind != KGE_DIST_ROT_L1)) {
    const int r = kge_score_dist2(kind, sign, q, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    if (r >= 0) return r;
  }
  dim3 grid((unsigned)((m + TN - 1) / TN), (unsigned)((n + TM - 1) / TM));
  switch (kind) {
    case KGE_DIST_L1: score_dist_kernel<KGE_DIST_L1><<<grid, NT, 0, st>>>(sign, q, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds); break;
    case KGE_DIST_L2: score_dist_kernel<KGE_DIST_L2><<<grid, NT, 0, st>>>(sign, q, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds); break;
    case KGE_DIST_ROT_L1: score_dist_kernel<KGE_DIST_ROT_L1><<<grid, NT, 0, st>>>(sign, q, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds); break;
    default: score_dist_kernel<KGE_DIST_ROT_L2><<<grid, NT, 0, st>>>(sign, q, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds); break;
  }
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_score_dist_bwd(int kind, float sign, const float* g, int64_t ldg, const float* q, int64_t ldq,
                                  const float* t, int64_t ldt, const int64_t* tidx, int64_t n, int64_t m, int d,
                                  float* dq, int64_t lddq, float* dt, int64_t lddt, void* stream) {
  KGE_REQUIRE(n >= 0 && m >= 0 && d > 0 && n < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE(g && q && t && ldg >= m && ldq >= d && ldt >= d);
  KGE_REQUIRE(kind >= KGE_DIST_L1 && kind <= KGE_DIST_ROT_L2);
  KGE_REQUIRE(!is_rot(kind) || d % 2 == 0);
  if (n == 0 || m == 0 || (!dq && !dt)) return 0;
  hipStream_t st = as_stream(stream);
  // L1 kinds: the pair weights are sign * G as they stand -> the owner-computes kernels
  // (score_dist_bwd2.hip).  The L2 kinds need G / dist: callers that can hold that [n, m]
  // block use kge_score_dist_bwd_weighted; here they take the generic kernel below, which
  // recomputes the distances per tile.
  if (kind == KGE_DIST_L1 || kind == KGE_DIST_ROT_L1) {
    const int r = kge_score_dist_bwd_own(kind, sign, g, ldg, q, ldq, t, ldt, tidx, n, m, d, dq, lddq, dt, lddt, st);
    if (r >= 0) {
      if (r == 0) KGE_CHECK_LAUNCH();
      return r;
    }
  }
  KGE_REQUIRE((n + TM - 1) / TM < 65536);
  dim3 grid((unsigned)((m + TN - 1) / TN), (unsigned)((n + TM - 1) / TM));
#define KGE_DB(K) \
  score_dist_bwd_kernel<K><<<grid, NT, 0, st>>>(sign, g, ldg, q, ldq, t, ldt, tidx, (int)n, (int)m, d, dq, lddq, dt, lddt)
  switch (kind) {
    case KGE_DIST_L1: KGE_DB(KGE_DIST_L1); break;
    case KGE_DIST_L2: KGE_DB(KGE_DIST_L2); break;
    case KGE_DIST_ROT_L1: KGE_DB(KGE_DIST_ROT_L1); break;
    default: KGE_DB(KGE_DIST_ROT_L2); break;
  }
#undef KGE_DB
  KGE_CHECK_LAUNCH();
  return 0;
}

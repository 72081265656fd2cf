// All-entities distance scoring for TransE / RotatE on the VALU (no MFMA: a register-tiled,
// wavefront-reduced L1 / L2 distance kernel).
//
// S[i, j] = sign * dist(Q[i], T[row(j)]), 128 x 128 output tile per 256-thread workgroup,
// 8 x 8 outputs per thread held as 8 x 4 pairs of adjacent columns (plain scalar fp32 VALU:
// the library is built with packed fp32 instructions switched off):
//   L1      : d = q - t, acc += |d|                 (|.| as a source modifier)
//   L2      : d = q - t, acc = d * d + acc
//   ROT_L1  : dr, di, sq = dr dr + di di, acc += sqrt(sq)
//   ROT_L2  : dr, di, acc = dr dr + acc, acc = di di + acc
// Measured at B = 1024, E = 14,541, d = 512: L1 358 us, L2 360, RotatE-L2 394 (score_dist.hip's
// kernel: 498 / 478 / 433); RotatE-L1 843 vs 746 us, so kge_score_dist keeps that kind on
// score_dist.hip.
// K is staged KC = 16 columns (complex components for RotatE) at a time, K-major in LDS,
// double-buffered with the next chunk prefetched into registers (one barrier per chunk).
// A thread owns rows {4 ty .. 4 ty + 3, 64 + 4 ty ..} and columns {4 tx .., 64 + 4 tx ..}:
// the 16 lanes that share ty read 16 consecutive float4 of a K row (conflict-free), rows
// are broadcast.  Requires 16-B aligned rows, ld % 4 == 0 and kdim % 4 == 0 (the launcher
// falls back to score_dist.hip otherwise).
#include "common.h"

namespace {

constexpr int TM = 128, TN = 128, KC = 16, NT = 256;
constexpr int LD = TM + 4;  // K-major LDS row, floats

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ void __launch_bounds__(NT) score_dist2_kernel(float sign, const float* __restrict__ q, int64_t ldq,
                                                         const float* __restrict__ t, int64_t ldt,
                                                         const int64_t* __restrict__ tidx, int n, int m, int d,
                                                         float* __restrict__ s, int64_t lds) {
  constexpr bool ROT = KIND >= KGE_DIST_ROT_L1;
  constexpr int NP = ROT ? 2 : 1;  // planes: re (and im)
  // [buffer][operand q / t][plane][k][row]
  __shared__ __attribute__((aligned(16))) float xs[2][2][NP][KC * LD];
  const int tid = threadIdx.x;
  const int i0 = blockIdx.y * TM, j0 = blockIdx.x * TN;
  const int tx = tid & 15, ty = tid >> 4;
  const int kdim = ROT ? d / 2 : d;
  const int h = d / 2;
  const int nch = (kdim + KC - 1) / KC;

  // staging: thread -> row (tid & 127), float4 slots k = 8 (tid >> 7) + {0, 4} of the chunk
  const int srow = tid & (TM - 1), sk = (tid >> 7) * 8;
  const float* qrow = q + (int64_t)min(i0 + srow, n - 1) * ldq;
  int64_t trow_i = min(j0 + srow, m - 1);
  if (tidx) trow_i = tidx[trow_i];
  const float* trow = t + trow_i * ldt;
  float4 pf[2][NP][2];  // [operand][plane][slot]
  auto load = [&](int c) {
    const int k = c * KC + sk;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int kk = k + 4 * sl;
      const bool ok = kk < kdim;
      const int kc = ok ? kk : 0;
      // load from the clamped address first, select afterwards: `ok ? *p : z` compiles into a
      // load through a selected pointer (global row or a zero on the stack), i.e. flat loads
      auto ld4 = [&](const float* p) {
        const float4 v = *reinterpret_cast<const float4*>(p);
        return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
      };
      pf[0][0][sl] = ld4(qrow + kc);
      pf[1][0][sl] = ld4(trow + kc);
      if constexpr (ROT) {
        pf[0][1][sl] = ld4(qrow + h + kc);
        pf[1][1][sl] = ld4(trow + h + kc);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int op = 0; op < 2; ++op)
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          float* dst = &xs[buf][op][pl][(sk + 4 * sl) * LD + srow];
          const float4 v = pf[op][pl][sl];
          dst[0] = v.x;
          dst[LD] = v.y;
          dst[2 * LD] = v.z;
          dst[3 * LD] = v.w;
        }
  };

  f32x2 acc[8][4];
  float acc1[8][8];  // L1: scalar accumulators (the adds take |d| as a source modifier)
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      acc[a][b] = f32x2{0.f, 0.f};
      acc1[a][2 * b] = acc1[a][2 * b + 1] = 0.f;
    }

  load(0);
  store(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int cur = c & 1;
    if (c + 1 < nch) load(c + 1);
#pragma unroll 2
    for (int kk = 0; kk < KC; ++kk) {
      float qv[NP][8], tv[NP][8];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
        const float* qb = &xs[cur][0][pl][kk * LD];
        const float* tb = &xs[cur][1][pl][kk * LD];
        const float4 q0 = *reinterpret_cast<const float4*>(qb + 4 * ty);
        const float4 q1 = *reinterpret_cast<const float4*>(qb + 64 + 4 * ty);
        const float4 t0 = *reinterpret_cast<const float4*>(tb + 4 * tx);
        const float4 t1 = *reinterpret_cast<const float4*>(tb + 64 + 4 * tx);
        qv[pl][0] = q0.x; qv[pl][1] = q0.y; qv[pl][2] = q0.z; qv[pl][3] = q0.w;
        qv[pl][4] = q1.x; qv[pl][5] = q1.y; qv[pl][6] = q1.z; qv[pl][7] = q1.w;
        tv[pl][0] = t0.x; tv[pl][1] = t0.y; tv[pl][2] = t0.z; tv[pl][3] = t0.w;
        tv[pl][4] = t1.x; tv[pl][5] = t1.y; tv[pl][6] = t1.z; tv[pl][7] = t1.w;
      }
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const f32x2 qa = f32x2{qv[0][a], qv[0][a]};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const f32x2 dr = qa - f32x2{tv[0][2 * b], tv[0][2 * b + 1]};
          if constexpr (KIND == KGE_DIST_L1) {
            // |d| as a source modifier of the add (hipcc would clear the sign bits with
            // v_and_b32 and pack the adds: 2 instructions per pair instead of 1.5)
            asm("v_add_f32 %0, %0, |%1|" : "+v"(acc1[a][2 * b]) : "v"(dr.x));
            asm("v_add_f32 %0, %0, |%1|" : "+v"(acc1[a][2 * b + 1]) : "v"(dr.y));
          } else if constexpr (KIND == KGE_DIST_L2) {
            acc[a][b] = dr * dr + acc[a][b];
          } else {
            const f32x2 qi = f32x2{qv[NP - 1][a], qv[NP - 1][a]};
            const f32x2 di = qi - f32x2{tv[NP - 1][2 * b], tv[NP - 1][2 * b + 1]};
            if constexpr (KIND == KGE_DIST_ROT_L1) {
              const f32x2 sq = di * di + dr * dr;
              acc[a][b] += f32x2{__builtin_amdgcn_sqrtf(sq.x), __builtin_amdgcn_sqrtf(sq.y)};
            } else {
              acc[a][b] = dr * dr + acc[a][b];
              acc[a][b] = di * di + acc[a][b];
            }
          }
        }
      }
    }
    if (c + 1 < nch) store(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int i = i0 + (a < 4 ? 4 * ty + a : 64 + 4 * ty + a - 4);
    if (i >= n) continue;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int j = j0 + 64 * half + 4 * tx;
      float v[4] = {acc[a][2 * half].x, acc[a][2 * half].y, acc[a][2 * half + 1].x, acc[a][2 * half + 1].y};
      if constexpr (KIND == KGE_DIST_L1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc1[a][4 * half + e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (KIND == KGE_DIST_L2 || KIND == KGE_DIST_ROT_L2) v[e] = sqrtf(v[e]);
        v[e] *= sign;
      }
      float* dst = s + (int64_t)i * lds + j;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (j + e < m) dst[e] = v[e];
    }
  }
}

}  // namespace

// Launcher of the register-tiled kernel, used by kge_score_dist when the layout allows; returns
// -1 when it does not (the caller then takes score_dist.hip's kernel).
int kge_score_dist2(int kind, float sign, const float* q, int64_t ldq, const float* t, int64_t ldt,
                    const int64_t* tidx, int64_t n, int64_t m, int d, float* s, int64_t lds, hipStream_t st) {
  const int kdim = kind >= KGE_DIST_ROT_L1 ? d / 2 : d;
  if (kdim % 4 != 0 || ldq % 4 != 0 || ldt % 4 != 0 || !aligned16(q) || !aligned16(t)) return -1;
  if ((n + TM - 1) / TM >= 65536) return -1;
  dim3 grid((unsigned)((m + TN - 1) / TN), (unsigned)((n + TM - 1) / TM));
  switch (kind) {
    case KGE_DIST_L1: score_dist2_kernel<KGE_DIST_L1><<<grid, NT, 0, st>>>(sign, q, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds); break;
    case KGE_DIST_L2: score_dist2_kernel<KGE_DIST_L2><<<grid, NT, 0, st>>>(sign, q, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds); break;
    case KGE_DIST_ROT_L1: score_dist2_kernel<KGE_DIST_ROT_L1><<<grid, NT, 0, st>>>(sign, q, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds); break;
    default: score_dist2_kernel<KGE_DIST_ROT_L2><<<grid, NT, 0, st>>>(sign, q, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds); break;
  }
  KGE_CHECK_LAUNCH();
  return 0;
}

// Backward of the all-entities contraction S = Q . T^T (autograd of score_sp/score_po):
//   dQ = G . T        [n, d]  (K = m: long reduction, split over workgroups)
//   dT += G^T . Q     [m, d]  (K = n), rows scattered through tidx when given
// KGE_PREC_FP32 runs here on the exact fp32-input MFMA (v_mfma_f32_32x32x2_f32);
// KGE_PREC_BF16X3 dispatches to gemm_bwd3.hip.  Operands are staged
// into LDS K-major ([k][row]) so every fragment read is a 32-lane contiguous
// ds_read_b32 and whichever global layout an operand has is read coalesced.
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 16, NT = 256;
constexpr int A_LD = BM + 1;  // padded: transposing LDS writes stay conflict-free

// A_MODE 0: A(i, k) = a[i * lda + k]       (K contiguous: G for dQ)
// A_MODE 1: A(i, k) = a[k * lda + i]       (M contiguous: G^T for dT)
// B(k, j) = b[rowmap(k) * ldb + j]         (N contiguous: T for dQ (gathered), Q for dT)
// C_MODE 0: atomicAdd c[i * ldc + j]       (split-K partials: dQ)
// C_MODE 1: c[cmap(i) * ldc + j] += acc    (plain RMW; rows owned by one block: dT)
// C_MODE 2: atomicAdd c[cmap(i) * ldc + j] (scattered rows, duplicates possible: dT)
template <int A_MODE, int C_MODE>
__global__ void __launch_bounds__(NT, 2)
    gemm_f32_kernel(const float* __restrict__ a, int64_t lda, const float* __restrict__ b, int64_t ldb,
                    const int64_t* __restrict__ brow, float* c, int64_t ldc, const int64_t* __restrict__ crow,
                    int M, int N, int K, int kchunk) {
  __shared__ float As[BK * A_LD];
  __shared__ float Bs[BK * BN];
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  f32x16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int z = 0; z < 16; ++z) acc[x][y][z] = 0.f;

  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    // ---- stage A into As[k][i]
    if (A_MODE == 0) {
      const int kk = tid & 15;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int ii = (tid >> 4) + 16 * r;
        const int gi = m0 + ii, gk = k0 + kk;
        As[kk * A_LD + ii] = (gi < M && gk < kend) ? a[(int64_t)gi * lda + gk] : 0.f;
      }
    } else {
      const int ii = tid & 127;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int kk = (tid >> 7) + 2 * r;
        const int gi = m0 + ii, gk = k0 + kk;
        As[kk * A_LD + ii] = (gi < M && gk < kend) ? a[(int64_t)gk * lda + gi] : 0.f;
      }
    }
    // ---- stage B into Bs[k][j]
    {
      const int jj = tid & 127;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int kk = (tid >> 7) + 2 * r;
        const int gk = k0 + kk, gj = n0 + jj;
        float v = 0.f;
        if (gk < kend && gj < N) {
          const int64_t row = brow ? brow[gk] : (int64_t)gk;
          v = b[row * ldb + gj];
        }
        Bs[kk * BN + jj] = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kp = 0; kp < BK / 2; ++kp) {
      const int kk = 2 * kp + (lane >> 5);
      float av[2], bv[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        av[x] = As[kk * A_LD + wr * 64 + x * 32 + (lane & 31)];
        bv[x] = Bs[kk * BN + wc * 64 + x * 32 + (lane & 31)];
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[x], bv[y], acc[x][y], 0, 0, 0);
    }
    __syncthreads();
  }

  const int col_l = lane & 31, rh = lane >> 5;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int j = n0 + wc * 64 + y * 32 + col_l;
      if (j >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = m0 + wr * 64 + x * 32 + (r & 3) + 8 * (r >> 2) + 4 * rh;
        if (i >= M) continue;
        const float v = acc[x][y][r];
        if (C_MODE == 0) {
          atomicAdd(c + (int64_t)i * ldc + j, v);
        } else {
          const int64_t row = crow ? crow[i] : (int64_t)i;
          if (C_MODE == 1)
            c[row * ldc + j] += v;
          else
            atomicAdd(c + row * ldc + j, v);
        }
      }
    }
}

}  // namespace

extern "C" int64_t kge_score_dot_bwd_q_ws_size(int64_t n, int64_t m, int d, int precision) {
  if (precision != KGE_PREC_BF16X3 || n <= 0 || m <= 0 || d <= 0) return 0;
  const int splits = kge_bwd3_q_splits(n, m, d, kge_num_cus());
  return splits > 1 ? (int64_t)splits * n * d : 0;
}

extern "C" int kge_score_dot_bwd_q(const float* g, int64_t ldg, const float* t, int64_t ldt,
                                   const int64_t* tidx, int64_t n, int64_t m, int d, float* dq,
                                   int64_t lddq, int accumulate, int precision, void* stream) {
  return kge_score_dot_bwd_q_ws(g, ldg, t, ldt, tidx, n, m, d, dq, lddq, accumulate, precision, nullptr, 0, stream);
}

extern "C" int kge_score_dot_bwd_q_ws(const float* g, int64_t ldg, const float* t, int64_t ldt,
                                      const int64_t* tidx, int64_t n, int64_t m, int d, float* dq,
                                      int64_t lddq, int accumulate, int precision, float* ws, int64_t ws_elems,
                                      void* stream) {
  KGE_REQUIRE(n >= 0 && m >= 0 && d > 0 && n < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE((g || m == 0) && (t || m == 0) && dq && ldg >= m && ldt >= d && lddq >= d && ws_elems >= 0);
  KGE_REQUIRE(precision == KGE_PREC_FP32 || precision == KGE_PREC_BF16X3);
  hipStream_t st = as_stream(stream);
  if (m == 0 && !accumulate && n > 0) {  // empty reduction: dq = 0
    if (const int e = kge_zero_rows(dq, lddq, n, d, st)) return e;
  }
  if (n == 0 || m == 0) return 0;
  if (precision == KGE_PREC_BF16X3)
    return kge_bwd3_q(g, ldg, t, ldt, tidx, n, m, d, dq, lddq, accumulate, ws, ws_elems, kge_num_cus(), st);
  if (!accumulate) {
    if (const int e = kge_zero_rows(dq, lddq, n, d, st)) return e;
  }
  const int gm = (int)((n + BM - 1) / BM), gn = (d + BN - 1) / BN;
  // split the long K = m reduction so that the grid fills the chip (>= ~1024 blocks)
  int splits = (int)std::max<int64_t>(1, std::min<int64_t>((m + 255) / 256, 1024 / std::max(1, gm * gn)));
  int kchunk = (int)((m + splits - 1) / splits);
  kchunk = (kchunk + BK - 1) / BK * BK;
  splits = (int)((m + kchunk - 1) / kchunk);
  gemm_f32_kernel<0, 0><<<dim3(gm, gn, splits), dim3(NT), 0, st>>>(g, ldg, t, ldt, tidx, dq, lddq, nullptr,
                                                                   (int)n, d, (int)m, kchunk);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_score_dot_bwd_t(const float* g, int64_t ldg, const float* q, int64_t ldq,
                                   const int64_t* tidx, int64_t n, int64_t m, int d, float* dt,
                                   int64_t lddt, int precision, void* stream) {
  return kge_score_dot_bwd_t_ex(g, ldg, q, ldq, tidx, n, m, d, dt, lddt, 1, precision, stream);
}

extern "C" int kge_score_dot_bwd_t_ex(const float* g, int64_t ldg, const float* q, int64_t ldq,
                                      const int64_t* tidx, int64_t n, int64_t m, int d, float* dt,
                                      int64_t lddt, int accumulate, int precision, void* stream) {
  KGE_REQUIRE(n >= 0 && m >= 0 && d > 0 && n < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE(g && q && dt && ldg >= m && ldq >= d && lddt >= d);
  KGE_REQUIRE(precision == KGE_PREC_FP32 || precision == KGE_PREC_BF16X3);
  KGE_REQUIRE(accumulate || !tidx);
  if (m == 0) return 0;
  hipStream_t st = as_stream(stream);
  if (!accumulate && (n == 0 || precision == KGE_PREC_FP32)) {  // fp32 path: zero, then accumulate
    if (const int e = kge_zero_rows(dt, lddt, m, d, st)) return e;
    accumulate = 1;
  }
  if (n == 0) return 0;
  if (precision == KGE_PREC_BF16X3) return kge_bwd3_t(g, ldg, q, ldq, tidx, n, m, d, dt, lddt, accumulate, st);
  const int gm = (int)((m + BM - 1) / BM), gn = (d + BN - 1) / BN;
  // C[j][k] = sum_i G[i][j] Q[i][k]: A = G^T (M contiguous), B = Q
  if (tidx)
    gemm_f32_kernel<1, 2><<<dim3(gm, gn, 1), dim3(NT), 0, st>>>(g, ldg, q, ldq, nullptr, dt, lddt, tidx, (int)m,
                                                                d, (int)n, (int)n);
  else
    gemm_f32_kernel<1, 1><<<dim3(gm, gn, 1), dim3(NT), 0, st>>>(g, ldg, q, ldq, nullptr, dt, lddt, nullptr,
                                                                (int)m, d, (int)n, (int)n);
  KGE_CHECK_LAUNCH();
  return 0;
}

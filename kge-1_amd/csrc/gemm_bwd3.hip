// bf16x3 backward of the all-entities contraction S = Q . T^T (engine.precision bf16x3):
//   dQ  = G . T        [n, d]   K = m (entities), split over workgroups, atomic partials
//   dT += G^T . Q      [m, d]   K = n (queries), rows owned (RMW) or scattered (atomics)
// Same numerics as the forward (hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_bf16, fp32
// accumulation), ~8x the fp32-input MFMA rate of gemm_bwd.hip.
//
// Operands are fp32 in HBM and split to bf16 hi / lo while staging.  One "unit" is one
// operand row x 8 consecutive k: 8 strided scalar loads (G has a leading dimension m that
// is generally not a multiple of 4, so no vector loads), one 16-B LDS write per plane into
// the same XOR-swizzled [row][k] image the forward kernel reads conflict-free.  Threads
// map consecutive rows to consecutive lanes when the row index is the contiguous one
// (G^T, Q, T), so every load instruction of a wave reads 256 contiguous bytes.
// Tiles: 256 (rows of C) x 128 (columns of C = embedding dims), 8 waves of 64 x 64,
// BK = 32 double-buffered, register prefetch; 1-D grid remapped so the column tiles of
// one row panel (and the row panels of one K chunk) share an XCD's L2.
#include "common.h"

namespace {

constexpr int BM = 256, BN = 128, BK = 32, NT = 512, WN = 2;
constexpr int PLANE_A = BM * BK * 2, PLANE_B = BN * BK * 2;
constexpr int STAGE = 2 * PLANE_A + 2 * PLANE_B;  // 48 KB
constexpr int A_UNITS = BM * (BK / 8) / NT;       // 2
static_assert(BN * (BK / 8) == NT, "one B unit per thread");

__device__ __forceinline__ int sw_off(int row, int slot) {
  return row * 64 + ((slot ^ ((row >> 2) & 3)) << 4);
}

__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& h, bf16x8& l) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 x = (__bf16)v[e];
    h[e] = x;
    l[e] = (__bf16)(v[e] - (float)x);
  }
}

// C[i, j] (+)= sum_{k in chunk} A(i, k) * B(k, j)
//   A_T = false: A(i, k) = a[i * lda + k]     (G for dQ)
//   A_T = true : A(i, k) = a[k * lda + i]     (G^T for dT)
//   B(k, j) = b[brow(k) * ldb + j]            (T gathered through tidx for dQ; Q for dT)
// C_MODE 0: atomicAdd c[i * ldc + j]; 1: c[i * ldc + j] += v; 2: atomicAdd c[crow[i] * ldc + j];
// 3: c[i * ldc + j] = v (K not split: one block owns the element)
template <bool A_T, int C_MODE, bool GATHER>
__global__ void __launch_bounds__(NT, 1)
    gemm3_kernel(const float* __restrict__ a, int64_t lda, const float* __restrict__ b, int64_t ldb,
                 const int64_t* __restrict__ brow, float* c, int64_t ldc, const int64_t* __restrict__ crow, int M,
                 int N, int K, int kchunk, int nmt, int nnt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const int frow = lane & 31, fh = lane >> 5;

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = tile % nnt, rest = tile / nnt;
  const int mt = rest % nmt, z = rest / nmt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kbeg = z * kchunk, kend = min(K, kbeg + kchunk);
  if (kbeg >= kend) return;
  const int nst = (kend - kbeg + BK - 1) / BK;

  // Unit geometry.  Rows past M / columns past N read a clamped valid row and produce
  // accumulator rows / columns that are never stored, so only k needs masking (tail stage).
  // When k is the strided index (G^T, Q, T) it is wave-uniform: the row base goes to SGPRs
  // and each load is saddr + 32-bit lane offset, no per-load 64-bit VALU address math.
  int a_r[A_UNITS], a_ks[A_UNITS];
#pragma unroll
  for (int u = 0; u < A_UNITS; ++u) {
    const int id = tid + u * NT;
    a_r[u] = A_T ? id % BM : id / (BK / 8);
    a_ks[u] = A_T ? __builtin_amdgcn_readfirstlane(id / BM) : id % (BK / 8);
  }
  const int b_r = tid % BN, b_ks = __builtin_amdgcn_readfirstlane(tid / BN);  // one B unit per thread
  const unsigned b_off = (unsigned)min(n0 + b_r, N - 1);
  unsigned a_off[A_UNITS];  // A_T: lane column offset
  const float* a_ptr[A_UNITS];  // !A_T: lane row pointer at k = 0
#pragma unroll
  for (int u = 0; u < A_UNITS; ++u) {
    const int gr = min(m0 + a_r[u], M - 1);
    a_off[u] = (unsigned)gr;
    a_ptr[u] = a + (int64_t)gr * lda + a_ks[u] * 8;
  }

  // Branch-free loads (k clamped into the chunk): a load whose result is merged from two
  // control-flow paths makes the compiler wait for it right away, exposing the latency.
  // Out-of-chunk k are zeroed when the registers are written to LDS (store), one stage later.
  float ra[A_UNITS][8], rb[8];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < A_UNITS; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = min(k0 + a_ks[u] * 8 + e, kend - 1);
        ra[u][e] = A_T ? (a + (int64_t)k * lda)[a_off[u]] : a_ptr[u][k - a_ks[u] * 8];
      }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = min(k0 + b_ks * 8 + e, kend - 1);
      const int64_t row = GATHER ? brow[k] : (int64_t)k;
      rb[e] = (b + row * ldb)[b_off];
    }
  };
  auto store = [&](unsigned char* st, int k0) {
    unsigned char* ahi = st;
    unsigned char* alo = st + PLANE_A;
    unsigned char* bhi = st + 2 * PLANE_A;
    unsigned char* blo = bhi + PLANE_B;
    bf16x8 h, l;
    const int lim = kend - k0;  // k offsets >= lim are outside the chunk
#pragma unroll
    for (int u = 0; u < A_UNITS; ++u) {
#pragma unroll
      for (int e = 0; e < 8; ++e) ra[u][e] = a_ks[u] * 8 + e < lim ? ra[u][e] : 0.f;
      split8(ra[u], h, l);
      *reinterpret_cast<bf16x8*>(ahi + sw_off(a_r[u], a_ks[u])) = h;
      *reinterpret_cast<bf16x8*>(alo + sw_off(a_r[u], a_ks[u])) = l;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) rb[e] = b_ks * 8 + e < lim ? rb[e] : 0.f;
    split8(rb, h, l);
    *reinterpret_cast<bf16x8*>(bhi + sw_off(b_r, b_ks)) = h;
    *reinterpret_cast<bf16x8*>(blo + sw_off(b_r, b_ks)) = l;
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[x][y][q] = 0.f;

  auto compute = [&](const unsigned char* cur) {
    const unsigned char* ahi = cur;
    const unsigned char* alo = cur + PLANE_A;
    const unsigned char* bhi = cur + 2 * PLANE_A;
    const unsigned char* blo = bhi + PLANE_B;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int slot = ks * 2 + fh;
      bf16x8 b_h[2], b_l[2];
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        const int rb_ = wc * 64 + y * 32 + frow;
        b_h[y] = *reinterpret_cast<const bf16x8*>(bhi + sw_off(rb_, slot));
        b_l[y] = *reinterpret_cast<const bf16x8*>(blo + sw_off(rb_, slot));
      }
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int ra_ = wr * 64 + x * 32 + frow;
        const bf16x8 a_h = *reinterpret_cast<const bf16x8*>(ahi + sw_off(ra_, slot));
        const bf16x8 a_l = *reinterpret_cast<const bf16x8*>(alo + sw_off(ra_, slot));
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_l, b_h[y], acc[x][y], 0, 0, 0);
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, b_l[y], acc[x][y], 0, 0, 0);
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, b_h[y], acc[x][y], 0, 0, 0);
        }
      }
    }
  };

  load(kbeg);
  store(smem, kbeg);
  if (nst > 1) load(kbeg + BK);
  __syncthreads();
  int st = 0;
  for (; st + 2 < nst; ++st) {
    store(smem + ((st + 1) & 1) * STAGE, kbeg + (st + 1) * BK);
    load(kbeg + (st + 2) * BK);
    // keep the prefetch loads ahead of the MFMAs (left alone, the scheduler sinks them to
    // the end of the stage and the next store waits on their full latency)
    __builtin_amdgcn_sched_barrier(0);
    compute(smem + (st & 1) * STAGE);
    __syncthreads();
  }
  if (st + 1 < nst) {
    store(smem + ((st + 1) & 1) * STAGE, kbeg + (st + 1) * BK);
    compute(smem + (st & 1) * STAGE);
    __syncthreads();
    ++st;
  }
  compute(smem + (st & 1) * STAGE);

  const int rh = lane >> 5;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int j = n0 + wc * 64 + y * 32 + frow;
      if (j >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = m0 + wr * 64 + x * 32 + (r & 3) + 8 * (r >> 2) + 4 * rh;
        if (i >= M) continue;
        const float v = acc[x][y][r];
        if (C_MODE == 0) {
          atomicAdd(c + (int64_t)i * ldc + j, v);
        } else if (C_MODE == 1) {
          c[(int64_t)i * ldc + j] += v;
        } else if (C_MODE == 3) {
          c[(int64_t)i * ldc + j] = v;
        } else if (C_MODE == 4) {
          c[((int64_t)z * M + i) * ldc + j] = v;
        } else {
          atomicAdd(c + crow[i] * ldc + j, v);
        }
      }
    }
}

// ---------------------------------------------------------------------------------------
// Vectorised variant for 16-B-aligned operands with leading dimensions % 4 == 0 -- the G
// written by kge_softmax_xent into padded rows, T and Q.  Operands whose reduction index k
// is their ROW index (G^T for dT; T and Q as B) are staged in their natural [k][col] layout:
// float4 global loads along the contiguous column, 8-B bf16x4 LDS writes, and the MFMA
// fragments (8 consecutive k of one column per lane) are assembled by the gfx950
// transposing read ds_read_b64_tr_b16 (two per fragment).  [k][col] rows are XOR-swizzled
// in 64-B chunks by (k & 3), so the four rows of one transposed read hit four different
// bank ranges.  G for dQ (k = its column) keeps the [row][k] image of the forward kernel.
// Requires: N % 4 == 0, lda >= round_up(M, 4) (A_T) -- pad columns are read into
// accumulator rows that are never stored.

typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4v lds_bf16x4;

// byte offset of column `col` (multiple of 4) of k-row `k` in a [k][COLS] bf16 image
template <int COLS>
__device__ __forceinline__ int kc_off(int k, int col) {
  return k * (COLS * 2) + ((((col >> 5) ^ (k & 3))) << 6) + (col & 31) * 2;
}

// fragment of a 32x32x16 operand whose 32 rows are columns c0 .. c0+31 of a [k][COLS] image,
// k = k0 .. k0+15: lane l gets (column c0 + (l & 31), k = k0 + 8 (l >> 5) + j), j = 0..7
template <int COLS>
__device__ __forceinline__ bf16x8 tr_frag(const unsigned char* img, int c0, int k0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int kb = k0 + 8 * (g >> 1) + q, col = c0 + 16 * (g & 1) + 4 * p;
  const bf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + kc_off<COLS>(kb, col)));
  const bf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + kc_off<COLS>(kb + 4, col)));
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[j] = lo[j];
    f[4 + j] = hi[j];
  }
  return f;
}

__device__ __forceinline__ void split4(const float4& v, bf16x4& h, bf16x4& l) { split_bf16x4_pk(v, h, l); }

template <bool A_T, int C_MODE, bool GATHER>
__global__ void __launch_bounds__(NT, 1)
    gemm3v_kernel(const float* __restrict__ a, int64_t lda, const float* __restrict__ b, int64_t ldb,
                  const int64_t* __restrict__ brow, float* c, int64_t ldc, const int64_t* __restrict__ crow, int M,
                  int N, int K, int kchunk, int nmt, int nnt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const int frow = lane & 31, fh = lane >> 5;

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = tile % nnt, rest = tile / nnt;
  const int mt = rest % nmt, z = rest / nmt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kbeg = z * kchunk, kend = min(K, kbeg + kchunk);
  if (kbeg >= kend) return;
  const int nst = (kend - kbeg + BK - 1) / BK;

  // ---- A units.  A_T: 4 k-rows x 4 columns (one per thread, k-quad = wave: uniform).
  //      K-contig: 1 row x 4 k (four per thread).
  constexpr int AU = A_T ? 1 : 4;
  int a_row[AU], a_kq[AU];
  const float* a_src[AU];
  const int Mp = (M + 3) & ~3;
#pragma unroll
  for (int u = 0; u < AU; ++u) {
    if (A_T) {
      a_row[u] = (tid & 63) * 4;                                 // column group of G (rows of C)
      a_kq[u] = __builtin_amdgcn_readfirstlane(tid >> 6);        // k-quad 0..7
      a_src[u] = a + min(m0 + a_row[u], Mp - 4);
    } else {
      const int id = tid + u * NT;
      a_row[u] = id >> 3;
      a_kq[u] = id & 7;
      a_src[u] = a + (int64_t)min(m0 + a_row[u], M - 1) * lda;
    }
  }
  // ---- B units: 4 k-rows x 4 columns, threads 256..511 (waves 4-7)
  const bool b_unit = tid >= NT / 2;
  const int bt = tid & (NT / 2 - 1);
  const int b_col = (bt & 31) * 4, b_kq = bt >> 5;
  const float* b_src = b + min(n0 + b_col, N - 4);

  float4 ra[A_T ? 4 : AU], rb[4];
  auto load = [&](int k0) {
    if (A_T) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = min(k0 + a_kq[0] * 4 + e, kend - 1);
        ra[e] = *reinterpret_cast<const float4*>(a_src[0] + (int64_t)k * lda);
      }
    } else {
#pragma unroll
      for (int u = 0; u < AU; ++u) {
        const int k = min(k0 + a_kq[u] * 4, (int)lda - 4);
        ra[u] = *reinterpret_cast<const float4*>(a_src[u] + k);
      }
    }
    if (b_unit) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = min(k0 + b_kq * 4 + e, kend - 1);
        const int64_t row = GATHER ? brow[k] : (int64_t)k;
        rb[e] = *reinterpret_cast<const float4*>(b_src + row * ldb);
      }
    }
  };
  constexpr int A_PLANE = BM * BK * 2, B_PLANE = BN * BK * 2;
  auto zero_past = [](float4 v, int kk, int lim) {  // zero elements whose k offset >= lim
    return kk < lim ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto store = [&](unsigned char* st, int k0) {
    unsigned char* ahi = st;
    unsigned char* alo = st + A_PLANE;
    unsigned char* bhi = st + 2 * A_PLANE;
    unsigned char* blo = bhi + B_PLANE;
    const int lim = kend - k0;
    bf16x4 h, l;
    if (A_T) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kk = a_kq[0] * 4 + e;
        split4(zero_past(ra[e], kk, lim), h, l);
        *reinterpret_cast<bf16x4*>(ahi + kc_off<BM>(kk, a_row[0])) = h;
        *reinterpret_cast<bf16x4*>(alo + kc_off<BM>(kk, a_row[0])) = l;
      }
    } else {
#pragma unroll
      for (int u = 0; u < AU; ++u) {
        const int kk = a_kq[u] * 4;
        float4 v = ra[u];
        v.x = kk + 0 < lim ? v.x : 0.f;
        v.y = kk + 1 < lim ? v.y : 0.f;
        v.z = kk + 2 < lim ? v.z : 0.f;
        v.w = kk + 3 < lim ? v.w : 0.f;
        split4(v, h, l);
        const int off = sw_off(a_row[u], a_kq[u] >> 1) + (a_kq[u] & 1) * 8;
        *reinterpret_cast<bf16x4*>(ahi + off) = h;
        *reinterpret_cast<bf16x4*>(alo + off) = l;
      }
    }
    if (b_unit) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kk = b_kq * 4 + e;
        split4(zero_past(rb[e], kk, lim), h, l);
        *reinterpret_cast<bf16x4*>(bhi + kc_off<BN>(kk, b_col)) = h;
        *reinterpret_cast<bf16x4*>(blo + kc_off<BN>(kk, b_col)) = l;
      }
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[x][y][q] = 0.f;

  auto compute = [&](const unsigned char* cur) {
    const unsigned char* ahi = cur;
    const unsigned char* alo = cur + A_PLANE;
    const unsigned char* bhi = cur + 2 * A_PLANE;
    const unsigned char* blo = bhi + B_PLANE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 b_h[2], b_l[2];
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        const int c0 = wc * 64 + y * 32;
        b_h[y] = tr_frag<BN>(bhi, c0, ks * 16, lane);
        b_l[y] = tr_frag<BN>(blo, c0, ks * 16, lane);
      }
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        bf16x8 a_h, a_l;
        if (A_T) {
          const int r0 = wr * 64 + x * 32;
          a_h = tr_frag<BM>(ahi, r0, ks * 16, lane);
          a_l = tr_frag<BM>(alo, r0, ks * 16, lane);
        } else {
          const int ra_ = wr * 64 + x * 32 + frow;
          a_h = *reinterpret_cast<const bf16x8*>(ahi + sw_off(ra_, ks * 2 + fh));
          a_l = *reinterpret_cast<const bf16x8*>(alo + sw_off(ra_, ks * 2 + fh));
        }
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_l, b_h[y], acc[x][y], 0, 0, 0);
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, b_l[y], acc[x][y], 0, 0, 0);
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, b_h[y], acc[x][y], 0, 0, 0);
        }
      }
    }
  };

  load(kbeg);
  store(smem, kbeg);
  if (nst > 1) load(kbeg + BK);
  __syncthreads();
  int st = 0;
  for (; st + 2 < nst; ++st) {
    store(smem + ((st + 1) & 1) * STAGE, kbeg + (st + 1) * BK);
    load(kbeg + (st + 2) * BK);
    __builtin_amdgcn_sched_barrier(0);
    compute(smem + (st & 1) * STAGE);
    __syncthreads();
  }
  if (st + 1 < nst) {
    store(smem + ((st + 1) & 1) * STAGE, kbeg + (st + 1) * BK);
    compute(smem + (st & 1) * STAGE);
    __syncthreads();
    ++st;
  }
  compute(smem + (st & 1) * STAGE);

  const int rh = lane >> 5;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int j = n0 + wc * 64 + y * 32 + frow;
      if (j >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = m0 + wr * 64 + x * 32 + (r & 3) + 8 * (r >> 2) + 4 * rh;
        if (i >= M) continue;
        const float v = acc[x][y][r];
        if (C_MODE == 0) {
          atomicAdd(c + (int64_t)i * ldc + j, v);
        } else if (C_MODE == 1) {
          c[(int64_t)i * ldc + j] += v;
        } else if (C_MODE == 3) {
          c[(int64_t)i * ldc + j] = v;
        } else if (C_MODE == 4) {  // this K chunk's partial slab (summed by slab_sum_kernel)
          c[((int64_t)z * M + i) * ldc + j] = v;
        } else {
          atomicAdd(c + crow[i] * ldc + j, v);
        }
      }
    }
}

// out[i, j] (+)= sum over z = 0 .. splits-1 of slab[z][i][j], in z order: the split-K sum of
// the dQ GEMM without float atomics (which run at ~1.3 TB/s of added bytes chip-wide,
// MI355X_MICROARCH.md 'Global float atomics', and sum in arrival order) -- deterministic.
__global__ void __launch_bounds__(256) slab_sum_kernel(const float* __restrict__ slab, int splits, int64_t M, int N,
                                                       float* __restrict__ out, int64_t ldo, int accumulate) {
  const int n4 = N / 4;
  const int64_t total = M * n4;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / n4;
    const int j = (int)(e - i * n4) * 4;
    float4 acc = accumulate ? *reinterpret_cast<const float4*>(out + i * ldo + j) : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int z = 0; z < splits; ++z) {
      const float4 v = *reinterpret_cast<const float4*>(slab + (z * M + i) * N + j);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    *reinterpret_cast<float4*>(out + i * ldo + j) = acc;
  }
}

// x[i, 0 .. d) = 0 for i < n (a fill kernel rather than hipMemset2DAsync, so that a caller may
// capture the launch sequence into a HIP graph).
__global__ void __launch_bounds__(256) zero_rows_kernel(float* __restrict__ x, int64_t ldx, int64_t n, int d) {
  const int64_t total = n * d;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x)
    x[(e / d) * ldx + e % d] = 0.f;
}

int zero_rows(float* x, int64_t ldx, int64_t n, int d, hipStream_t st) { return kge_zero_rows(x, ldx, n, d, st); }

template <bool A_T, int C_MODE, bool GATHER, bool VEC>
int launch(const float* a, int64_t lda, const float* b, int64_t ldb, const int64_t* brow, float* c, int64_t ldc,
           const int64_t* crow, int64_t M, int64_t N, int64_t K, int splits, hipStream_t st) {
  const void* fn = VEC ? (const void*)gemm3v_kernel<A_T, C_MODE, GATHER> : (const void*)gemm3_kernel<A_T, C_MODE, GATHER>;
  static std::atomic<bool> lds_ok[KGE_MAX_DEVICES];
  if (const int e = kge_allow_lds(fn, 2 * STAGE, lds_ok)) return e;
  const int nmt = (int)((M + BM - 1) / BM), nnt = (int)((N + BN - 1) / BN);
  int kchunk = (int)((K + splits - 1) / splits);
  kchunk = (kchunk + BK - 1) / BK * BK;
  splits = (int)((K + kchunk - 1) / kchunk);
  const int64_t blocks = (int64_t)nmt * nnt * splits;
  if (blocks > 0x7fffffff) return KGE_ERR_ARG;
  if (VEC)
    gemm3v_kernel<A_T, C_MODE, GATHER><<<dim3((unsigned)blocks), dim3(NT), 2 * STAGE, st>>>(
        a, lda, b, ldb, brow, c, ldc, crow, (int)M, (int)N, (int)K, kchunk, nmt, nnt);
  else
    gemm3_kernel<A_T, C_MODE, GATHER><<<dim3((unsigned)blocks), dim3(NT), 2 * STAGE, st>>>(
        a, lda, b, ldb, brow, c, ldc, crow, (int)M, (int)N, (int)K, kchunk, nmt, nnt);
  KGE_CHECK_LAUNCH();
  return 0;
}

bool vec_ok(const float* g, int64_t ldg, int64_t m, const float* x, int64_t ldx, int d) {
  return aligned16(g) && ldg % 4 == 0 && ldg >= ((m + 3) & ~3LL) && aligned16(x) && ldx % 4 == 0 && d % 4 == 0 &&
         d >= 4 && m >= 4;
}

}  // namespace

int kge_zero_rows(float* x, int64_t ldx, int64_t n, int d, hipStream_t st) {
  if (n <= 0 || d <= 0) return 0;
  const int blocks = (int)std::min<int64_t>((n * d + 255) / 256, 4096);
  zero_rows_kernel<<<dim3(blocks), dim3(256), 0, st>>>(x, ldx, n, d);
  KGE_CHECK_LAUNCH();
  return 0;
}

// K splits of the dQ GEMM: enough that the grid covers the CUs once (one wave of
// 1-block-per-CU tiles)
int kge_bwd3_q_splits(int64_t n, int64_t m, int d, int cus) {
  const int64_t tiles = ((n + BM - 1) / BM) * ((d + BN - 1) / BN);
  const int64_t by_k = std::max<int64_t>(1, (m + 8 * BK - 1) / (8 * BK));
  const int64_t asked = std::max<int64_t>(1, std::min<int64_t>(by_k, cus / std::max<int64_t>(1, tiles)));
  // launch() rounds the K chunk up to whole BK stages, which can leave fewer chunks than asked
  // (14,541 rows in 32 chunks -> 480-row chunks -> 31 of them): return the number of chunks that
  // actually run, because that is how many slabs get written and must be summed.  The rounding is
  // idempotent (c = round_up(ceil(K / s)) and s' = ceil(K / c) give round_up(ceil(K / s')) = c),
  // so launch() arrives at the same chunk size from the returned count.
  int64_t kchunk = (m + asked - 1) / asked;
  kchunk = (kchunk + BK - 1) / BK * BK;
  return (int)std::max<int64_t>(1, (m + kchunk - 1) / kchunk);
}

// Called from kge_score_dot_bwd_q / _t (gemm_bwd.hip) for KGE_PREC_BF16X3.  With a workspace
// of splits * n * d floats (and vectorisable operands) the K chunks write partial slabs that
// slab_sum_kernel adds in a fixed order; otherwise the chunks add into dq with float atomics
// (dq zero-filled first unless accumulating).
int kge_bwd3_q(const float* g, int64_t ldg, const float* t, int64_t ldt, const int64_t* tidx, int64_t n,
               int64_t m, int d, float* dq, int64_t lddq, int accumulate, float* ws, int64_t ws_elems, int cus,
               hipStream_t st) {
  const int splits = kge_bwd3_q_splits(n, m, d, cus);
  if (vec_ok(g, ldg, m, t, ldt, d) && splits > 1 && ws && ws_elems >= (int64_t)splits * n * d && lddq % 4 == 0 &&
      aligned16(dq) && aligned16(ws)) {
    const int e = tidx ? launch<false, 4, true, true>(g, ldg, t, ldt, tidx, ws, d, nullptr, n, d, m, splits, st)
                       : launch<false, 4, false, true>(g, ldg, t, ldt, nullptr, ws, d, nullptr, n, d, m, splits, st);
    if (e) return e;
    const int64_t total = n * (d / 4);
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, (int64_t)cus * 4);
    slab_sum_kernel<<<dim3(blocks), dim3(256), 0, st>>>(ws, splits, n, d, dq, lddq, accumulate);
    KGE_CHECK_LAUNCH();
    return 0;
  }
  if (vec_ok(g, ldg, m, t, ldt, d) && splits == 1) {  // K not split: every dQ element has one owner
    if (accumulate)
      return tidx ? launch<false, 1, true, true>(g, ldg, t, ldt, tidx, dq, lddq, nullptr, n, d, m, 1, st)
                  : launch<false, 1, false, true>(g, ldg, t, ldt, nullptr, dq, lddq, nullptr, n, d, m, 1, st);
    return tidx ? launch<false, 3, true, true>(g, ldg, t, ldt, tidx, dq, lddq, nullptr, n, d, m, 1, st)
                : launch<false, 3, false, true>(g, ldg, t, ldt, nullptr, dq, lddq, nullptr, n, d, m, 1, st);
  }
  if (!accumulate) {
    if (const int e = zero_rows(dq, lddq, n, d, st)) return e;
  }
  if (vec_ok(g, ldg, m, t, ldt, d)) {
    if (tidx) return launch<false, 0, true, true>(g, ldg, t, ldt, tidx, dq, lddq, nullptr, n, d, m, splits, st);
    return launch<false, 0, false, true>(g, ldg, t, ldt, nullptr, dq, lddq, nullptr, n, d, m, splits, st);
  }
  if (tidx) return launch<false, 0, true, false>(g, ldg, t, ldt, tidx, dq, lddq, nullptr, n, d, m, splits, st);
  return launch<false, 0, false, false>(g, ldg, t, ldt, nullptr, dq, lddq, nullptr, n, d, m, splits, st);
}

int kge_bwd3_t(const float* g, int64_t ldg, const float* q, int64_t ldq, const int64_t* tidx, int64_t n,
               int64_t m, int d, float* dt, int64_t lddt, int accumulate, hipStream_t st) {
  if (vec_ok(g, ldg, m, q, ldq, d)) {
    if (tidx) return launch<true, 2, false, true>(g, ldg, q, ldq, nullptr, dt, lddt, tidx, m, d, n, 1, st);
    if (!accumulate) return launch<true, 3, false, true>(g, ldg, q, ldq, nullptr, dt, lddt, nullptr, m, d, n, 1, st);
    return launch<true, 1, false, true>(g, ldg, q, ldq, nullptr, dt, lddt, nullptr, m, d, n, 1, st);
  }
  if (tidx) return launch<true, 2, false, false>(g, ldg, q, ldq, nullptr, dt, lddt, tidx, m, d, n, 1, st);
  if (!accumulate) return launch<true, 3, false, false>(g, ldg, q, ldq, nullptr, dt, lddt, nullptr, m, d, n, 1, st);
  return launch<true, 1, false, false>(g, ldg, q, ldq, nullptr, dt, lddt, nullptr, m, d, n, 1, st);
}

// ---------------------------------------------------------------------------------------
// kge_score_dot_bwd_q_noalloc: the dQ GEMM for callers that cannot allocate (HIP graph
// capture, serving loops).  The split-K partial slabs go to this file-scope device array
// instead of a caller workspace.  Its size covers every shape on a device of up to 256 CUs:
// splits <= CUs / tiles and tiles >= (n / BM) (d / BN), so splits * n * d <= 256 * BM * BN.
// Each GPU the library runs on holds its own copy (at its own address) until the process
// ends; every call on a GPU shares it, so calls that overlap on one GPU (two streams) race.
// Nothing in it needs clearing between calls: every slab element that slab_sum_kernel reads
// is written by the GEMM of the same call.
constexpr int64_t SCRATCH_ELEMS = (int64_t)256 * BM * BN;  // 8 Mi floats = 32 MiB
static __device__ __align__(256) float scratch[SCRATCH_ELEMS];

namespace {
std::atomic<float*> scratch_ptr[KGE_MAX_DEVICES];  // device address of `scratch`, per device

// The array's name is a host-side stand-in, not a device address: resolve it once per device,
// with that device current, and hand kernels the resolved pointer only.
int scratch_address(float** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  if (dev < 0 || dev >= KGE_MAX_DEVICES) return KGE_ERR_ARG;
  float* p = scratch_ptr[dev].load(std::memory_order_acquire);
  if (!p) {
    void* sym = nullptr;
    e = hipGetSymbolAddress(&sym, HIP_SYMBOL(scratch));
    if (e != hipSuccess) return (int)e;
    if (!sym) return (int)hipErrorInvalidSymbol;
    p = static_cast<float*>(sym);
    scratch_ptr[dev].store(p, std::memory_order_release);
  }
  *out = p;
  return 0;
}
}  // namespace

extern "C" int kge_score_dot_bwd_q_noalloc(const float* g, int64_t ldg, const float* t, int64_t ldt,
                                           const int64_t* tidx, int64_t n, int64_t m, int d, float* dq,
                                           int64_t lddq, int accumulate, void* stream) {
  KGE_REQUIRE(n >= 0 && m >= 0 && d > 0 && n < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE((g || m == 0) && (t || m == 0) && dq && ldg >= m && ldt >= d && lddq >= d);  // m == 0: g, t unread
  hipStream_t st = as_stream(stream);
  if (n == 0) return 0;
  if (m == 0) return accumulate ? 0 : zero_rows(dq, lddq, n, d, st);
  if (!vec_ok(g, ldg, m, t, ldt, d) || lddq % 4 != 0 || !aligned16(dq)) return KGE_ERR_ALIGN;
  const int cus = kge_num_cus();
  const int splits = kge_bwd3_q_splits(n, m, d, cus);
  const int64_t need = splits > 1 ? (int64_t)splits * n * d : 0;
  if (need > SCRATCH_ELEMS) return KGE_ERR_SCRATCH;
  float* ws = nullptr;
  if (need > 0) {
    if (const int e = scratch_address(&ws)) return e;
  }
  return kge_bwd3_q(g, ldg, t, ldt, tidx, n, m, d, dq, lddq, accumulate, ws, need > 0 ? SCRATCH_ELEMS : 0, cus, st);
}

#ifdef KGE_DEV_BUILD  // libkgescore_dev.so only
// Dev-only variants for scripts/dev/tune_bwd.py (not in include/kgescore.h): 0 = dQ as shipped
// (split-K atomics), 1 = dQ with plain stores (wrong sums: prices the atomics), 2 = dT
// written (C_MODE 3), 3 = dT read-modify-write (C_MODE 1).
extern "C" int kge_dev_bwd3(int variant, const float* g, int64_t ldg, const float* x, int64_t ldx, int64_t n,
                            int64_t m, int d, float* c, int64_t ldc, int splits, void* stream) {
  hipStream_t st = as_stream(stream);
  if (!vec_ok(g, ldg, m, x, ldx, d)) return KGE_ERR_ALIGN;
  switch (variant) {
    case 0: return launch<false, 0, false, true>(g, ldg, x, ldx, nullptr, c, ldc, nullptr, n, d, m, splits, st);
    case 1: return launch<false, 3, false, true>(g, ldg, x, ldx, nullptr, c, ldc, nullptr, n, d, m, splits, st);
    case 2: return launch<true, 3, false, true>(g, ldg, x, ldx, nullptr, c, ldc, nullptr, m, d, n, 1, st);
    case 3: return launch<true, 1, false, true>(g, ldg, x, ldx, nullptr, c, ldc, nullptr, m, d, n, 1, st);
    default: return KGE_ERR_ARG;
  }
}
#endif  // KGE_DEV_BUILD

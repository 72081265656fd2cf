// All-entities contraction S = Q . T^T for the bilinear scorers (ComplEx, DistMult,
// RESCAL): the hot kernel of score_sp / score_po.
//
// Shape: Q [n, d] (prepared query rows), T [m, d] (entity table rows, optionally
// gathered through tidx), S [n, m] fp32.  Both operands are K-contiguous, so every MFMA
// fragment is one 16-byte LDS read.
//
// Two precisions:
//   KGE_PREC_BF16X3 -- each fp32 operand is split into bf16 hi + lo while it is staged
//     into LDS; the product is hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_bf16
//     (fp32 accumulate).  Representation error <= 2^-16 relative per operand, dropped
//     lo*lo term <= 2^-16 |q||e|: ~4e-6 of the row max at d = 512, inside the 1e-4
//     contract, and bit-exact whenever the inputs have <= 16 significant bits (dyadic
//     fixtures).  3 bf16 passes run at 3/16 of the cost of the fp32 MFMA.
//   KGE_PREC_FP32 -- v_mfma_f32_32x32x2_f32: an exact f32 FMA chain (different
//     summation order than the reference's sgemm, same rounding class).
//
// Tiling: 256 threads = 4 waves (2 x 2), block tile 128 queries x 128 entities, wave
// tile 64 x 64 = 2 x 2 MFMA 32x32 accumulators; K staged 32 fp32 columns at a time
// with a register prefetch of the next stage overlapping the MFMAs of the current one.
// Block ids are remapped XCD-aware so the n/128 query tiles that share one entity panel
// run on one XCD and read that panel from its L2 (the Q rows, 2 MB at B=1024/d=512,
// stay L2-resident everywhere).
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;

// bf16 LDS image: [row][32 bf16] = 64-B rows, 16-B slots XOR-swizzled by (row>>2)&3 so
// that the ds_read_b128 lane groups of a 32x32x16 fragment read are conflict-free.
__device__ __forceinline__ int sw_off(int row, int slot) {  // byte offset
  return row * 64 + ((slot ^ ((row >> 2) & 3)) << 4);
}

// fp32 LDS image: [row][32 + 4 pad] floats (144-B rows: conflict-free ds_read_b128).
constexpr int F32_LD = BK + 4;

struct StageRegs {
  float4 a[4];
  float4 b[4];
};

template <bool VEC>
__device__ __forceinline__ float4 load4(const float* row, int k, int d) {
  if (VEC) {
    if (k < d) return *reinterpret_cast<const float4*>(row + k);
    return make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
    float4 v;
    v.x = (k + 0 < d) ? row[k + 0] : 0.f;
    v.y = (k + 1 < d) ? row[k + 1] : 0.f;
    v.z = (k + 2 < d) ? row[k + 2] : 0.f;
    v.w = (k + 3 < d) ? row[k + 3] : 0.f;
    return v;
  }
}

template <int PREC, bool VEC>
__global__ void __launch_bounds__(NT, 2)
    score_dot_kernel(const float* __restrict__ q, int64_t ldq, const float* __restrict__ t,
                     int64_t ldt, const int64_t* __restrict__ tidx, int n, int m, int d,
                     float* __restrict__ s, int64_t lds, int n_row_tiles) {
  // LDS: bf16x3 -> 4 planes of [128][32] bf16 (8 KB each); fp32 -> 2 x [128][36] floats.
  constexpr int LDS_BYTES = (PREC == KGE_PREC_BF16X3) ? 4 * BM * BK * 2 : 2 * BM * F32_LD * 4;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[LDS_BYTES];

  const int nblocks = gridDim.x;
  const int L = xcd_remap(blockIdx.x, nblocks);
  const int tile_m = L % n_row_tiles;  // query tile
  const int tile_n = L / n_row_tiles;  // entity tile
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  // per-thread global rows for staging: row = (tid >> 3) + 32 * i, col = (tid & 7) * 4
  const int ld_row = tid >> 3, ld_col = (tid & 7) * 4;
  const float* arow[4];
  const float* brow[4];
  bool aval[4], bval[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qi = m0 + ld_row + 32 * i;
    aval[i] = qi < n;
    arow[i] = q + (int64_t)(aval[i] ? qi : 0) * ldq;
    const int ej = n0 + ld_row + 32 * i;
    bval[i] = ej < m;
    const int64_t er = bval[i] ? (tidx ? tidx[ej] : (int64_t)ej) : 0;
    brow[i] = t + er * ldt;
  }

  auto load_stage = [&](StageRegs& r, int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      r.a[i] = aval[i] ? load4<VEC>(arow[i], k0 + ld_col, d) : make_float4(0.f, 0.f, 0.f, 0.f);
      r.b[i] = bval[i] ? load4<VEC>(brow[i], k0 + ld_col, d) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int z = 0; z < 16; ++z) acc[x][y][z] = 0.f;

  StageRegs regs;
  load_stage(regs, 0);
  const int nstages = (d + BK - 1) / BK;

  for (int st = 0; st < nstages; ++st) {
    // ---- write the staged registers into LDS
    if (PREC == KGE_PREC_BF16X3) {
      unsigned char* ahi = lds_raw;
      unsigned char* alo = lds_raw + BM * BK * 2;
      unsigned char* bhi = lds_raw + 2 * BM * BK * 2;
      unsigned char* blo = lds_raw + 3 * BM * BK * 2;
      const int slot = ld_col >> 3, half = (ld_col >> 2) & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = ld_row + 32 * i;
        const int off = sw_off(row, slot) + half * 8;
        bf16x4 h, l;
        split_bf16x4(regs.a[i], h, l);
        *reinterpret_cast<bf16x4*>(ahi + off) = h;
        *reinterpret_cast<bf16x4*>(alo + off) = l;
        split_bf16x4(regs.b[i], h, l);
        *reinterpret_cast<bf16x4*>(bhi + off) = h;
        *reinterpret_cast<bf16x4*>(blo + off) = l;
      }
    } else {
      float* as = reinterpret_cast<float*>(lds_raw);
      float* bs = as + BM * F32_LD;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = ld_row + 32 * i;
        *reinterpret_cast<float4*>(as + row * F32_LD + ld_col) = regs.a[i];
        *reinterpret_cast<float4*>(bs + row * F32_LD + ld_col) = regs.b[i];
      }
    }
    __syncthreads();
    if (st + 1 < nstages) load_stage(regs, (st + 1) * BK);  // in flight during the MFMAs

    // ---- MFMAs on the staged tile
    if (PREC == KGE_PREC_BF16X3) {
      const unsigned char* ahi = lds_raw;
      const unsigned char* alo = lds_raw + BM * BK * 2;
      const unsigned char* bhi = lds_raw + 2 * BM * BK * 2;
      const unsigned char* blo = lds_raw + 3 * BM * BK * 2;
      const int frow = lane & 31, fh = lane >> 5;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int slot = ks * 2 + fh;
        bf16x8 a_h[2], a_l[2], b_h[2], b_l[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          const int ra = wr * 64 + x * 32 + frow;
          a_h[x] = *reinterpret_cast<const bf16x8*>(ahi + sw_off(ra, slot));
          a_l[x] = *reinterpret_cast<const bf16x8*>(alo + sw_off(ra, slot));
          const int rb = wc * 64 + x * 32 + frow;
          b_h[x] = *reinterpret_cast<const bf16x8*>(bhi + sw_off(rb, slot));
          b_l[x] = *reinterpret_cast<const bf16x8*>(blo + sw_off(rb, slot));
        }
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y) {
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_l[x], b_h[y], acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h[x], b_l[y], acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h[x], b_h[y], acc[x][y], 0, 0, 0);
          }
      }
    } else {
      const float* as = reinterpret_cast<const float*>(lds_raw);
      const float* bs = as + BM * F32_LD;
      const int frow = lane & 31, fh = lane >> 5;
      // lane half fh covers k in [16 fh, 16 fh + 16): one MFMA (K = 2) sums k and k + 16
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) {
        float4 av[2], bv[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          av[x] = *reinterpret_cast<const float4*>(as + (wr * 64 + x * 32 + frow) * F32_LD + fh * 16 + kq * 4);
          bv[x] = *reinterpret_cast<const float4*>(bs + (wc * 64 + x * 32 + frow) * F32_LD + fh * 16 + kq * 4);
        }
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y) {
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[x].x, bv[y].x, acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[x].y, bv[y].y, acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[x].z, bv[y].z, acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[x].w, bv[y].w, acc[x][y], 0, 0, 0);
          }
      }
    }
    __syncthreads();
  }

  // ---- epilogue: C[row][col], row = (r&3) + 8(r>>2) + 4(lane>>5), col = lane&31
  const int col_l = lane & 31, rh = lane >> 5;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int j = n0 + wc * 64 + y * 32 + col_l;
      if (j >= m) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = m0 + wr * 64 + x * 32 + (r & 3) + 8 * (r >> 2) + 4 * rh;
        if (i < n) s[(int64_t)i * lds + j] = acc[x][y][r];
      }
    }
}

template <int PREC>
int launch(const float* q, int64_t ldq, const float* t, int64_t ldt, const int64_t* tidx, int64_t n,
           int64_t m, int d, float* s, int64_t lds, hipStream_t st) {
  const int nrt = (int)((n + BM - 1) / BM);
  const int nct = (int)((m + BN - 1) / BN);
  const int64_t nb = (int64_t)nrt * nct;
  if (nb > 0x7fffffff) return KGE_ERR_ARG;
  const bool vec = (d % 4 == 0) && (ldq % 4 == 0) && (ldt % 4 == 0) && aligned16(q) && aligned16(t);
  if (vec)
    score_dot_kernel<PREC, true><<<dim3((unsigned)nb), dim3(NT), 0, st>>>(q, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds, nrt);
  else
    score_dot_kernel<PREC, false><<<dim3((unsigned)nb), dim3(NT), 0, st>>>(q, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds, nrt);
  KGE_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int kge_score_dot(const float* q, int64_t ldq, const float* t, int64_t ldt, const int64_t* tidx,
                             int64_t n, int64_t m, int d, float* s, int64_t lds, int precision, void* stream) {
  KGE_REQUIRE(n >= 0 && m >= 0 && d > 0 && n < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE(q && t && s && ldq >= d && ldt >= d && lds >= m);
  if (n == 0 || m == 0) return 0;
  hipStream_t st = as_stream(stream);
  if (precision == KGE_PREC_BF16X3) return launch<KGE_PREC_BF16X3>(q, ldq, t, ldt, tidx, n, m, d, s, lds, st);
  if (precision == KGE_PREC_FP32) return launch<KGE_PREC_FP32>(q, ldq, t, ldt, tidx, n, m, d, s, lds, st);
  return KGE_ERR_ARG;
}

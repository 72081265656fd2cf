// Persistent bf16x3 contraction S = Q . T^T: every workgroup loops over output tiles, so the
// fp32 score stores of tile t (the dominant HBM traffic: 4 B per scored triple) drain while
// tile t+1 is loaded and multiplied, instead of all tiles storing at once at the end.
//
// Per tile: Q arrives pre-split as bf16 hi / lo planes, the entity rows are split on the
// fly; K is staged 32 fp32 columns at a time into a double-buffered, XOR-swizzled LDS
// image; one barrier per stage; 32x32x16 bf16 MFMA, hi*hi + hi*lo + lo*hi.
// Tile order is XCD-grouped: the workgroups that share an XCD take consecutive tiles, i.e.
// the query tiles of one entity panel, so each panel is read from HBM once per XCD.
#include "common.h"

namespace {

constexpr int BK = 32;

__device__ __forceinline__ int sw_off(int row, int slot) {
  return row * 64 + ((slot ^ ((row >> 2) & 3)) << 4);
}

template <int BM, int BN, int WM, int WN>
struct PCfg {
  static constexpr int NT = 64 * WM * WN;
  static constexpr int TM = BM / WM / 32;
  static constexpr int TN = BN / WN / 32;
  static constexpr int PLANE_A = BM * BK * 2;
  static constexpr int PLANE_B = BN * BK * 2;
  static constexpr int STAGE = 2 * PLANE_A + 2 * PLANE_B;
  static constexpr int A_PER_T = BM * 4 / NT;
  static constexpr int B_PER_T = BN * 8 / NT;
  static_assert(BM * 4 % NT == 0 && BN * 8 % NT == 0, "staging");
  static_assert(BM % (32 * WM) == 0 && BN % (32 * WN) == 0, "tile");
};

typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));  // 4-B-aligned float4

template <int BM, int BN, int WM, int WN, bool EPI = false>
__global__ void __launch_bounds__(64 * WM * WN, 1)
    score_dot_persist_kernel(const __bf16* __restrict__ qhi, const __bf16* __restrict__ qlo, int64_t ldq,
                             const float* __restrict__ t, int64_t ldt, const int64_t* __restrict__ tidx, int n,
                             int m, int d, float* __restrict__ s, int64_t lds, int nrt, int ntiles) {
  using C = PCfg<BM, BN, WM, WN>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const int frow = lane & 31, fh = lane >> 5;
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, per_xcd = G >> 3, local = blockIdx.x >> 3;
  const int nst = (d + BK - 1) / BK;

  for (int it = 0;; ++it) {
    const int tile = it * G + xcd * per_xcd + local;
    if (tile >= ntiles) break;
    const int m0 = (tile % nrt) * BM, n0 = (tile / nrt) * BN;

    const __bf16* a_hi[C::A_PER_T];
    const __bf16* a_lo[C::A_PER_T];
    int a_off[C::A_PER_T];
    unsigned a_mk[C::A_PER_T];
#pragma unroll
    for (int i = 0; i < C::A_PER_T; ++i) {
      const int c = tid + i * C::NT;
      const int row = c >> 2, slot = c & 3;
      const int qi = m0 + row;
      a_mk[i] = qi < n ? 0xffffffffu : 0u;
      const int64_t base = (int64_t)(qi < n ? qi : 0) * ldq + slot * 8;
      a_hi[i] = qhi + base;
      a_lo[i] = qlo + base;
      a_off[i] = sw_off(row, slot);
    }
    const float* b_src[C::B_PER_T];
    int b_off[C::B_PER_T], b_col[C::B_PER_T];
    bool b_ok[C::B_PER_T];
#pragma unroll
    for (int i = 0; i < C::B_PER_T; ++i) {
      const int f = tid + i * C::NT;
      const int row = f >> 3, col = (f & 7) * 4;
      const int ej = n0 + row;
      b_ok[i] = ej < m;
      const int64_t er = b_ok[i] ? (tidx ? tidx[ej] : (int64_t)ej) : 0;
      b_src[i] = t + er * ldt + col;
      b_col[i] = col;
      b_off[i] = sw_off(row, col >> 3) + ((col >> 2) & 1) * 8;
    }
    uint4 ra_hi[C::A_PER_T], ra_lo[C::A_PER_T], rb[C::B_PER_T];
    auto load = [&](int k0) {
#pragma unroll
      for (int i = 0; i < C::A_PER_T; ++i) {
        ra_hi[i] = *reinterpret_cast<const uint4*>(a_hi[i] + k0);
        ra_lo[i] = *reinterpret_cast<const uint4*>(a_lo[i] + k0);
      }
#pragma unroll
      for (int i = 0; i < C::B_PER_T; ++i)
        rb[i] = *reinterpret_cast<const uint4*>(b_src[i] + min(k0, d - 4 - b_col[i]));
    };
    auto store = [&](unsigned char* st, int k0) {
      unsigned char* ahi = st;
      unsigned char* alo = st + C::PLANE_A;
      unsigned char* bhi = st + 2 * C::PLANE_A;
      unsigned char* blo = bhi + C::PLANE_B;
#pragma unroll
      for (int i = 0; i < C::A_PER_T; ++i) {
        const unsigned mk = a_mk[i];
        *reinterpret_cast<uint4*>(ahi + a_off[i]) =
            make_uint4(ra_hi[i].x & mk, ra_hi[i].y & mk, ra_hi[i].z & mk, ra_hi[i].w & mk);
        *reinterpret_cast<uint4*>(alo + a_off[i]) =
            make_uint4(ra_lo[i].x & mk, ra_lo[i].y & mk, ra_lo[i].z & mk, ra_lo[i].w & mk);
      }
#pragma unroll
      for (int i = 0; i < C::B_PER_T; ++i) {
        const unsigned mk = (b_ok[i] && k0 + b_col[i] < d) ? 0xffffffffu : 0u;
        const float4 v = make_float4(__uint_as_float(rb[i].x & mk), __uint_as_float(rb[i].y & mk),
                                     __uint_as_float(rb[i].z & mk), __uint_as_float(rb[i].w & mk));
        bf16x4 h, l;
        split_bf16x4(v, h, l);
        *reinterpret_cast<bf16x4*>(bhi + b_off[i]) = h;
        *reinterpret_cast<bf16x4*>(blo + b_off[i]) = l;
      }
    };

    f32x16 acc[C::TM][C::TN];
#pragma unroll
    for (int x = 0; x < C::TM; ++x)
#pragma unroll
      for (int y = 0; y < C::TN; ++y)
#pragma unroll
        for (int z = 0; z < 16; ++z) acc[x][y][z] = 0.f;

    auto compute = [&](const unsigned char* cur) {
      const unsigned char* ahi = cur;
      const unsigned char* alo = cur + C::PLANE_A;
      const unsigned char* bhi = cur + 2 * C::PLANE_A;
      const unsigned char* blo = bhi + C::PLANE_B;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int slot = ks * 2 + fh;
        bf16x8 b_h[C::TN], b_l[C::TN];
#pragma unroll
        for (int y = 0; y < C::TN; ++y) {
          const int rb_ = wc * (BN / WN) + y * 32 + frow;
          b_h[y] = *reinterpret_cast<const bf16x8*>(bhi + sw_off(rb_, slot));
          b_l[y] = *reinterpret_cast<const bf16x8*>(blo + sw_off(rb_, slot));
        }
#pragma unroll
        for (int x = 0; x < C::TM; ++x) {
          const int ra = wr * (BM / WM) + x * 32 + frow;
          const bf16x8 a_h = *reinterpret_cast<const bf16x8*>(ahi + sw_off(ra, slot));
          const bf16x8 a_l = *reinterpret_cast<const bf16x8*>(alo + sw_off(ra, slot));
#pragma unroll
          for (int y = 0; y < C::TN; ++y) {
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_l, b_h[y], acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, b_l[y], acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, b_h[y], acc[x][y], 0, 0, 0);
          }
        }
      }
    };

    load(0);
    store(smem, 0);
    if (nst > 1) load(BK);
    __syncthreads();
    int st = 0;
    for (; st + 2 < nst; ++st) {
      store(smem + ((st + 1) & 1) * C::STAGE, (st + 1) * BK);
      load((st + 2) * BK);
      compute(smem + (st & 1) * C::STAGE);
      __syncthreads();
    }
    if (st + 1 < nst) {
      store(smem + ((st + 1) & 1) * C::STAGE, (st + 1) * BK);
      compute(smem + (st & 1) * C::STAGE);
      __syncthreads();
      ++st;
    }
    compute(smem + (st & 1) * C::STAGE);

    const int col_l = lane & 31, rh = lane >> 5;
    if (EPI) {
      // Row-vector epilogue: each 32x32 accumulator tile (a column per lane) is transposed
      // through a wave-private 4 KB LDS scratch and stored as whole-row float4s -- 4
      // global_store_dwordx4 per lane instead of 16 dword stores; the tail of the kernel is
      // store-issue-bound.  Score rows (leading dim m, odd in general) are only 4-B aligned:
      // gfx950 / HSA declares unaligned global access (the compiler emits dwordx4 for an
      // align-4 float4), so no per-row realignment is needed.
      __syncthreads();  // every wave is done with the stage buffers: reuse as scratch
      float* scr = reinterpret_cast<float*>(smem) + wave * 32 * 32;
      const int rr = lane >> 3, cc = (lane & 7) * 4;
#pragma unroll
      for (int x = 0; x < C::TM; ++x)
#pragma unroll
        for (int y = 0; y < C::TN; ++y) {
#pragma unroll
          for (int r = 0; r < 16; ++r) scr[((r & 3) + 8 * (r >> 2) + 4 * rh) * 32 + col_l] = acc[x][y][r];
          const int i0 = m0 + wr * (BM / WM) + x * 32, j = n0 + wc * (BN / WN) + y * 32 + cc;
#pragma unroll
          for (int pass = 0; pass < 4; ++pass) {
            const int row = pass * 8 + rr;
            const float4 v = *reinterpret_cast<const float4*>(scr + row * 32 + cc);
            const int i = i0 + row;
            if (i >= n) continue;
            float* dst = s + (int64_t)i * lds + j;
            if (j + 3 < m) {
              *reinterpret_cast<f32x4u*>(dst) = f32x4u{v.x, v.y, v.z, v.w};
            } else {
              if (j < m) dst[0] = v.x;
              if (j + 1 < m) dst[1] = v.y;
              if (j + 2 < m) dst[2] = v.z;
            }
          }
        }
    } else {
#pragma unroll
      for (int x = 0; x < C::TM; ++x)
#pragma unroll
        for (int y = 0; y < C::TN; ++y) {
          const int j = n0 + wc * (BN / WN) + y * 32 + col_l;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int i = m0 + wr * (BM / WM) + x * 32 + (r & 3) + 8 * (r >> 2) + 4 * rh;
            if (i < n && j < m) s[(int64_t)i * lds + j] = acc[x][y][r];
          }
        }
    }
    __syncthreads();  // LDS of this tile is free for the next tile's prologue
  }
}

template <int BM, int BN, int WM, int WN, bool EPI = false>
int launch_persist(const __bf16* qhi, const __bf16* qlo, int64_t ldq, const float* t, int64_t ldt,
                   const int64_t* tidx, int64_t n, int64_t m, int d, float* s, int64_t lds, int per_cu,
                   hipStream_t st) {
  using C = PCfg<BM, BN, WM, WN>;
  const int nrt = (int)((n + BM - 1) / BM);
  const int64_t ntiles = (int64_t)nrt * ((m + BN - 1) / BN);
  if (ntiles > 0x7fffffff) return KGE_ERR_ARG;
  const size_t shmem = 2 * C::STAGE;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)score_dot_persist_kernel<BM, BN, WM, WN, EPI>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  int grid = kge_num_cus() * per_cu;
  grid = (int)std::min<int64_t>(grid, (ntiles + 7) / 8 * 8);
  grid = std::max(8, grid / 8 * 8);
  score_dot_persist_kernel<BM, BN, WM, WN, EPI><<<dim3(grid), dim3(C::NT), shmem, st>>>(
      qhi, qlo, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds, nrt, (int)ntiles);
  KGE_CHECK_LAUNCH();
  return 0;
}

__global__ void split_rows_kernel(const float* __restrict__ x, int64_t ldx, int n, int d, __bf16* __restrict__ hi,
                                  __bf16* __restrict__ lo, int64_t ldo) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)n * ldo) return;
  const int64_t i = idx / ldo;
  const int k = (int)(idx - i * ldo);
  const float v = k < d ? x[i * ldx + k] : 0.f;
  __bf16 h, l;
  split_bf16(v, h, l);
  hi[idx] = h;
  lo[idx] = l;
}

}  // namespace

extern "C" int kge_split_rows(const float* x, int64_t ldx, int64_t n, int d, void* hi, void* lo, int64_t ldo,
                              void* stream) {
  KGE_REQUIRE(n >= 0 && d > 0 && x && hi && lo && ldx >= d && ldo >= d && ldo % 8 == 0);
  if (n == 0) return 0;
  const int64_t total = n * ldo;
  split_rows_kernel<<<dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream)>>>(
      x, ldx, (int)n, d, (__bf16*)hi, (__bf16*)lo, ldo);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_score_dot_split(const void* qhi, const void* qlo, int64_t ldq, const float* t, int64_t ldt,
                                   const int64_t* tidx, int64_t n, int64_t m, int d, float* s, int64_t lds,
                                   void* stream) {
  KGE_REQUIRE(n >= 0 && m >= 0 && d >= 4 && n < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE(qhi && qlo && t && s && lds >= m && ldt >= d);
  KGE_REQUIRE(ldq % 8 == 0 && ldq >= ((d + 31) / 32) * 32);
  if (d % 4 != 0 || ldt % 4 != 0 || !aligned16(t) || !aligned16(qhi) || !aligned16(qlo)) return KGE_ERR_ALIGN;
  if (n == 0 || m == 0) return 0;
  hipStream_t st = as_stream(stream);
  const __bf16* h = (const __bf16*)qhi;
  const __bf16* l = (const __bf16*)qlo;
  if (n > 128) return launch_persist<256, 256, 2, 4, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 1, st);
  return launch_persist<128, 256, 2, 4, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 1, st);
}

extern "C" int kge_dev_score_dot_persist(int variant, const void* qhi, const void* qlo, int64_t ldq,
                                         const float* t, int64_t ldt, const int64_t* tidx, int64_t n, int64_t m,
                                         int d, float* s, int64_t lds, void* stream) {
  KGE_REQUIRE(n > 0 && m > 0 && d >= 4 && ldq % 8 == 0 && ldq >= ((d + 31) / 32) * 32);
  KGE_REQUIRE(d % 4 == 0 && ldt % 4 == 0 && aligned16(t) && aligned16(qhi) && aligned16(qlo));
  hipStream_t st = as_stream(stream);
  const __bf16* h = (const __bf16*)qhi;
  const __bf16* l = (const __bf16*)qlo;
  switch (variant) {
    case 0: return launch_persist<256, 128, 4, 2>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 1, st);
    case 1: return launch_persist<128, 256, 2, 4>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 1, st);
    case 2: return launch_persist<128, 128, 2, 2>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 2, st);
    case 3: return launch_persist<128, 128, 2, 2>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 1, st);
    case 4: return launch_persist<256, 256, 2, 4>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 1, st);
    case 5: return launch_persist<256, 128, 4, 2>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 2, st);
    case 6: return launch_persist<128, 128, 2, 2>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 3, st);
    case 7: return launch_persist<256, 256, 2, 4, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 1, st);
    case 8: return launch_persist<128, 256, 2, 4, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, 1, st);
    default: return KGE_ERR_ARG;
  }
}

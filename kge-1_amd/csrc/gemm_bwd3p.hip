// bf16x3 backward GEMMs of the all-entities contraction S = Q . T^T on PRE-SPLIT operand
// planes (engine.precision bf16x3, fused-loss path):
//   dQ = G . T        [n, d]   K = m (entities), split over workgroups into partial slabs
//   dT = G^T . Q      [m, d]   K = n (queries)
// G arrives as bf16 hi / lo planes written by the loss kernel (kge_softmax_*_planes: row i of
// the score buffer holds the hi plane in its first half and the lo plane in its second), Q as
// the hi / lo planes the forward contraction already used.  Same numerics as the forward
// kernel and as gemm_bwd3.hip (hi*hi + hi*lo + lo*hi on bf16 MFMA, fp32 accumulation; the split
// of G happens once in the loss kernel instead of once per tile that reads it).
//
// What this buys over gemm_bwd3.hip: operands that are already bf16 planes are staged by
// LDS-DMA (global_load_lds_dwordx4) -- no register staging, no split VALU, no masks: padding
// rows / columns of the planes are zero by contract -- so the dT kernel issues no VALU work at
// all between its MFMAs and the dQ kernel only the split of the entity rows (as the forward).
//   dQ: A = G planes in the forward's [row][k] image (ds_read_b128 fragments); B = entity rows
//       (fp32, k = row index): each thread loads two consecutive rows x 4 columns, so a bf16
//       PAIR along k comes out of the paired split directly (ds_write_b32 into the [col][k]
//       image); hand-counted vmcnt as in score_dot3.hip.
//   dT: A = G planes, B = Q planes, both with k = row index: staged in their natural [k][col]
//       layout and read with the transposing ds_read_b64_tr_b16 (two per 16x16x32 fragment).
// Tiles 256 x 128 (8 waves of 64 x 64 = 4 x 4 MFMA 16x16x32), BK = 32, double-buffered LDS
// (96 KB), one barrier per stage, one tile per workgroup.
#include "mfma16.h"

namespace {

constexpr int BK = KGE_BK;
constexpr int BM = 256, BN = 128, WM = 4, WN = 2, NT = 512, NW = 8;
constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // 4 x 4 tiles of 16 x 16 per wave
constexpr int WCOLS = BN / WN;                       // 64
constexpr int SCR_LD = WCOLS + 4;
constexpr int PLANE_A = BM * BK * 2, PLANE_B = BN * BK * 2;
constexpr int STAGE = 2 * PLANE_A + 2 * PLANE_B;  // 48 KB
constexpr int A_G = BM / 16 / NW;                 // 1-KB A chunks per plane per wave (dQ)

typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4v lds_bf16x4;

// Epilogue shared by both kernels: each wave passes its 16 x 64 accumulator bands through a
// padded LDS scratch and stores 256-B row segments (float4 per lane), scaled by `alpha`,
// optionally added to what is there.  rows / cols: valid extent of the output; ldc % 4 == 0.
__device__ __forceinline__ void store_tile(const f32x4 (&acc)[TM][TN], unsigned char* smem, int wave, int lane,
                                           int wr, int wc, float* c, int64_t ldc, int r0, int c0, int rows, int cols,
                                           float alpha, bool accumulate) {
  const int fr = lane & 15, fs = lane >> 4;
  float* scr = reinterpret_cast<float*>(smem) + wave * 16 * SCR_LD;
  constexpr int LPR = WCOLS / 4;  // 16 lanes per scratch row
#pragma unroll
  for (int x = 0; x < TM; ++x) {
#pragma unroll
    for (int y = 0; y < TN; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[(4 * fs + r) * SCR_LD + y * 16 + fr] = acc[x][y][r];
    const int i0 = r0 + wr * (BM / WM) + x * 16;
#pragma unroll
    for (int pass = 0; pass < (16 * LPR) / 64; ++pass) {
      const int g = pass * 64 + lane;
      const int row = g / LPR, c4 = g % LPR;
      const int i = i0 + row, j = c0 + wc * WCOLS + c4 * 4;
      float4 v = *reinterpret_cast<const float4*>(scr + row * SCR_LD + c4 * 4);
      if (i >= rows || j >= cols) continue;  // cols % 4 == 0: a float4 is in or out as a whole
      float* dst = c + (int64_t)i * ldc + j;
      v.x *= alpha;
      v.y *= alpha;
      v.z *= alpha;
      v.w *= alpha;
      if (accumulate) {
        const float4 o = *reinterpret_cast<const float4*>(dst);
        v.x += o.x;
        v.y += o.y;
        v.z += o.z;
        v.w += o.w;
      }
      *reinterpret_cast<float4*>(dst) = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// dQ partial slabs: slab[z][i][j] = sum_{e in K chunk z} G[i, e] * T[e, j]
// ghi / glo: G planes, row stride ldgp (bf16 elements), columns [K, round_up(K, 32)) zero.
// GROUP: the three MFMAs of a band issued as three runs over y with one A fragment held per run
// (instead of three per accumulator in turn): same order per accumulator, bit-identical.
template <bool PIPE, bool GROUP>
__global__ void __launch_bounds__(NT, 1)
    bwd3p_q_kernel(const __bf16* __restrict__ ghi, const __bf16* __restrict__ glo, int64_t ldgp,
                   const float* __restrict__ t, int64_t ldt, int n, int N, int K, int kchunk, int nrt, int nct,
                   float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int fr = lane & 15, fs = lane >> 4;
  const unsigned smem_base = lds_addr(smem);
  const int64_t lo_off = glo - ghi;

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int ct = tile % nct, rest = tile / nct;
  const int mt = rest % nrt, z = rest / nrt;
  const int m0 = mt * BM, n0 = ct * BN;
  const int kb = z * kchunk, kend = min(K, kb + kchunk);
  const int nst = (kend - kb + BK - 1) / BK;  // >= 1 by construction of the grid

  // A planes by LDS-DMA (the forward's image): wave-instruction c fills rows 16c .. 16c+15 of
  // a plane; rows past n read row n-1 (never stored).
  const __bf16* ga[A_G];
#pragma unroll
  for (int i = 0; i < A_G; ++i) {
    const int row = (wave * A_G + i) * 16 + (lane >> 2);
    const int slot = (lane & 3) ^ sw16_swz(row);
    ga[i] = ghi + (int64_t)min(m0 + row, n - 1) * ldgp + kb + slot * 8;
  }
  // B: thread -> k pair kp (rows kb + k0 + 2 kp, +1) x 4 columns 4 c4 .. 4 c4 + 3.  Lanes are
  // 8 k pairs x 8 column quads: a wave-instruction reads 8 rows x 128 contiguous bytes.
  const int kp = (lane & 7) + 8 * (wave & 1), c4 = (lane >> 3) + 8 * (wave >> 1);
  const int b_colg = min(n0 + 4 * c4, N - 4);  // columns past N are never stored
  const float* b_base = t + b_colg;
  int b_off[4];  // LDS byte offset of (image row 4 c4 + j, k pair kp)
#pragma unroll
  for (int j = 0; j < 4; ++j) b_off[j] = sw16_off(4 * c4 + j, kp >> 2) + (kp & 3) * 4;
  u32x4 rv[2];

#define KGE_WAIT_VM(N) asm volatile("s_waitcnt vmcnt(%2)" : "+v"(rv[0]), "+v"(rv[1]) : "i"(N) : "memory")
  auto glds_a = [&](int buf, int k0) {
    const unsigned base = smem_base + buf * STAGE;
#pragma unroll
    for (int i = 0; i < A_G; ++i) {
      const unsigned c = (unsigned)(wave * A_G + i) * 1024u;
      glds16_asm(ga[i] + k0, base + c);
      glds16_asm(ga[i] + lo_off + k0, base + PLANE_A + c);
    }
  };
  auto load_b = [&](int k0) {  // rows past K read row K-1: the G planes are zero there
    const int e0 = min(kb + k0 + 2 * kp, K - 1), e1 = min(kb + k0 + 2 * kp + 1, K - 1);
    rv[0] = gload16_asm(b_base + (int64_t)e0 * ldt);
    rv[1] = gload16_asm(b_base + (int64_t)e1 * ldt);
  };
  auto store_b = [&](unsigned char* stg) {
    unsigned char* bhi = stg + 2 * PLANE_A;
    unsigned char* blo = bhi + PLANE_B;
    const float a0 = __uint_as_float(rv[0].x), a1 = __uint_as_float(rv[0].y), a2 = __uint_as_float(rv[0].z),
                a3 = __uint_as_float(rv[0].w);
    const float b0 = __uint_as_float(rv[1].x), b1 = __uint_as_float(rv[1].y), b2 = __uint_as_float(rv[1].z),
                b3 = __uint_as_float(rv[1].w);
    bf16x4 h, l;
    split_bf16x4_pk(make_float4(a0, b0, a1, b1), h, l);  // (k, k+1) of column 0 | of column 1
    uint2 hw = __builtin_bit_cast(uint2, h), lw = __builtin_bit_cast(uint2, l);
    *reinterpret_cast<unsigned*>(bhi + b_off[0]) = hw.x;
    *reinterpret_cast<unsigned*>(blo + b_off[0]) = lw.x;
    *reinterpret_cast<unsigned*>(bhi + b_off[1]) = hw.y;
    *reinterpret_cast<unsigned*>(blo + b_off[1]) = lw.y;
    split_bf16x4_pk(make_float4(a2, b2, a3, b3), h, l);
    hw = __builtin_bit_cast(uint2, h);
    lw = __builtin_bit_cast(uint2, l);
    *reinterpret_cast<unsigned*>(bhi + b_off[2]) = hw.x;
    *reinterpret_cast<unsigned*>(blo + b_off[2]) = lw.x;
    *reinterpret_cast<unsigned*>(bhi + b_off[3]) = hw.y;
    *reinterpret_cast<unsigned*>(blo + b_off[3]) = lw.y;
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int x = 0; x < TM; ++x)
#pragma unroll
    for (int y = 0; y < TN; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 b_h[TN], b_l[TN];
  auto compute_b = [&](const unsigned char* cur) {
    const unsigned char* bhi = cur + 2 * PLANE_A;
    const unsigned char* blo = bhi + PLANE_B;
#pragma unroll
    for (int y = 0; y < TN; ++y) {
      const int rb_ = wc * WCOLS + y * 16 + fr;
      b_h[y] = *reinterpret_cast<const bf16x8*>(bhi + sw16_off(rb_, fs));
      b_l[y] = *reinterpret_cast<const bf16x8*>(blo + sw16_off(rb_, fs));
    }
  };
  auto compute_x = [&](const unsigned char* cur, int x0, int x1) {
    const unsigned char* ahi = cur;
    const unsigned char* alo = cur + PLANE_A;
#pragma unroll
    for (int x = x0; x < x1; ++x) {
      const int ra = wr * (BM / WM) + x * 16 + fr;
      const bf16x8 a_h = *reinterpret_cast<const bf16x8*>(ahi + sw16_off(ra, fs));
      const bf16x8 a_l = *reinterpret_cast<const bf16x8*>(alo + sw16_off(ra, fs));
#pragma unroll
      for (int y = 0; y < TN; ++y) {
        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_l, b_h[y], acc[x][y], 0, 0, 0);
        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_h, b_l[y], acc[x][y], 0, 0, 0);
        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_h, b_h[y], acc[x][y], 0, 0, 0);
      }
    }
  };

  glds_a(0, 0);
  load_b(0);
  KGE_WAIT_VM(0);
  store_b(smem);
  load_b(min(1, nst - 1) * BK);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // One barrier per stage; the stage body is branch-free (the last stage re-stages its own K
  // chunk into the idle buffer) so that every path keeps the same in-flight counts: per stage a
  // wave issues 2 A_G DMAs (stage st + 1), then 2 register loads (stage st + 2).
  if constexpr (PIPE) {
    // The same loop software-pipelined inside each wave (as the forward kernel's): A fragments
    // fetched a band ahead, the last band held across the barrier while the next stage's first
    // fragments arrive, the split of the entity rows inside band 1.
    bf16x8 ah[2], al[2];
    auto read_a = [&](const unsigned char* stg, int x, int slot) {
      const int ra = wr * (BM / WM) + x * 16 + fr;
      ah[slot] = *reinterpret_cast<const bf16x8*>(stg + sw16_off(ra, fs));
      al[slot] = *reinterpret_cast<const bf16x8*>(stg + PLANE_A + sw16_off(ra, fs));
    };
    auto read_b = [&](const unsigned char* stg, int y) {
      const int rb_ = wc * WCOLS + y * 16 + fr;
      b_h[y] = *reinterpret_cast<const bf16x8*>(stg + 2 * PLANE_A + sw16_off(rb_, fs));
      b_l[y] = *reinterpret_cast<const bf16x8*>(stg + 2 * PLANE_A + PLANE_B + sw16_off(rb_, fs));
    };
    auto mfma3 = [&](int x, int y, int slot) {
      acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[slot], b_h[y], acc[x][y], 0, 0, 0);
      acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[slot], b_l[y], acc[x][y], 0, 0, 0);
      acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[slot], b_h[y], acc[x][y], 0, 0, 0);
    };
    static_assert(TM % 2 == 0 && TM >= 4, "held band in fragment slot 1");
    read_a(smem, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int y = 0; y < TN; ++y) {
      read_b(smem, y);
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int st = 0; st < nst; ++st) {
      const int nb = (st + 1) & 1;
      const unsigned char* cur = smem + (st & 1) * STAGE;
      unsigned char* nxt = smem + nb * STAGE;
      const int k1 = min(st + 1, nst - 1) * BK;
      glds_a(nb, k1);
#pragma unroll
      for (int x = 0; x < TM - 1; ++x) {
        read_a(cur, x + 1, (x + 1) & 1);
        if (x == 1) {
          KGE_WAIT_VM(2 * A_G);  // B(st + 1) has landed
          store_b(nxt);
          load_b(min(st + 2, nst - 1) * BK);
        }
        if constexpr (GROUP) {
#pragma unroll
          for (int y = 0; y < TN; ++y)
            acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[x & 1], b_h[y], acc[x][y], 0, 0, 0);
#pragma unroll
          for (int y = 0; y < TN; ++y)
            acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[x & 1], b_l[y], acc[x][y], 0, 0, 0);
#pragma unroll
          for (int y = 0; y < TN; ++y)
            acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[x & 1], b_h[y], acc[x][y], 0, 0, 0);
        } else {
#pragma unroll
          for (int y = 0; y < TN; ++y) mfma3(x, y, x & 1);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      KGE_WAIT_VM(2);  // A(st + 1) has landed
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      read_a(nxt, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (GROUP) {
        constexpr int HS = (TM - 1) & 1;
#pragma unroll
        for (int y = 0; y < TN; ++y)
          acc[TM - 1][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[HS], b_h[y], acc[TM - 1][y], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int y = 0; y < TN; ++y) {
          acc[TM - 1][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[HS], b_l[y], acc[TM - 1][y], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          const int rb_ = wc * WCOLS + y * 16 + fr;
          b_l[y] = *reinterpret_cast<const bf16x8*>(nxt + 2 * PLANE_A + PLANE_B + sw16_off(rb_, fs));
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int y = 0; y < TN; ++y) {
          acc[TM - 1][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[HS], b_h[y], acc[TM - 1][y], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          const int rb_ = wc * WCOLS + y * 16 + fr;
          b_h[y] = *reinterpret_cast<const bf16x8*>(nxt + 2 * PLANE_A + sw16_off(rb_, fs));
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int y = 0; y < TN; ++y) {
          mfma3(TM - 1, y, (TM - 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
          read_b(nxt, y);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  } else
  for (int st = 0; st < nst; ++st) {
    const int nb = (st + 1) & 1;
    const unsigned char* cur = smem + (st & 1) * STAGE;
    const int k1 = min(st + 1, nst - 1) * BK;
    glds_a(nb, k1);
    compute_b(cur);
    compute_x(cur, 0, 1);
    KGE_WAIT_VM(2 * A_G);  // B(st + 1) has landed
    store_b(smem + nb * STAGE);
    load_b(min(st + 2, nst - 1) * BK);
    compute_x(cur, 1, TM);
    KGE_WAIT_VM(2);  // A(st + 1) has landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  KGE_WAIT_VM(0);
#undef KGE_WAIT_VM

  __syncthreads();  // stage buffers free: per-wave epilogue scratch
  store_tile(acc, smem, wave, lane, wr, wc, slab + (int64_t)z * n * N, N, m0, n0, n, N, 1.f, false);
}

// out[i, j] (+)= alpha * sum_z slab[z][i][j], in z order (deterministic; no float atomics)
__global__ void __launch_bounds__(256) slab_sum_kernel(const float* __restrict__ slab, int splits, int64_t M, int N,
                                                       float* __restrict__ out, int64_t ldo, int accumulate,
                                                       const float* __restrict__ alpha_ptr) {
  const float alpha = alpha_ptr ? *alpha_ptr : 1.f;
  const int n4 = N / 4;
  const int64_t total = M * n4;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / n4;
    const int j = (int)(e - i * n4) * 4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int z = 0; z < splits; ++z) {
      const float4 v = *reinterpret_cast<const float4*>(slab + (z * M + i) * N + j);
      a.x += v.x;
      a.y += v.y;
      a.z += v.z;
      a.w += v.w;
    }
    a.x *= alpha;
    a.y *= alpha;
    a.z *= alpha;
    a.w *= alpha;
    if (accumulate) {
      const float4 o = *reinterpret_cast<const float4*>(out + i * ldo + j);
      a.x += o.x;
      a.y += o.y;
      a.z += o.z;
      a.w += o.w;
    }
    *reinterpret_cast<float4*>(out + i * ldo + j) = a;
  }
}

// ---------------------------------------------------------------------------------------
// dT[e, c] (+)= alpha * sum_i G[i, e] * Q[i, c]       e in [0, M), c in [0, N), i in [0, K)
// Both operands are bf16 planes whose reduction index is their ROW index: staged by LDS-DMA
// in their natural [k][col] layout, fragments assembled by ds_read_b64_tr_b16.  Rows
// [K, round_up(K, 32)) of all four planes are zero by contract.
//
// [k][COLS] image: 16-B chunk cc = col >> 3 = (q << 2) | (h << 1) | w of k-row k sits at chunk
// position ((q ^ (k & 3)) << 2) | ((h ^ ((k >> 3) & 1)) << 1) | w: the four k-rows and the two
// k-octets that the 32 lanes of one transposing-read cycle address then cover 32 distinct
// 8-B bank pairs (row pitches are multiples of 256 B, so without it they would all collide).
template <int COLS>
__device__ __forceinline__ int kc16_off(int k, int col) {
  const int cc = col >> 3;
  const int pos = ((((cc >> 2) ^ (k & 3)) << 2) | ((((cc >> 1) & 1) ^ ((k >> 3) & 1)) << 1) | (cc & 1));
  return k * (COLS * 2) + pos * 16 + (col & 7) * 2;
}

// 16x16x32 operand fragment whose 16 rows are columns c0 .. c0+15 of a [k][COLS] image:
// lane l gets (column c0 + (l & 15), k = 8 (l >> 4) + j), j = 0 .. 7
template <int COLS>
__device__ __forceinline__ bf16x8 tr_frag16(const unsigned char* img, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int k = 8 * g + q, col = c0 + 4 * p;
  const bf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + kc16_off<COLS>(k, col)));
  const bf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + kc16_off<COLS>(k + 4, col)));
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[j] = lo[j];
    f[4 + j] = hi[j];
  }
  return f;
}

// NSTG LDS stage buffers: 2 = the next stage's transfers are in flight during a stage's MFMAs;
// 3 = the next two stages' (144 KB of LDS), which covers HBM latency when the G planes are not
// resident in the memory-side cache.
template <int NSTG, bool GROUP>
__global__ void __launch_bounds__(NT, 1)
    bwd3p_t_kernel(const __bf16* __restrict__ ghi, const __bf16* __restrict__ glo, int64_t ldgp, int64_t gcols,
                   const __bf16* __restrict__ qhi, const __bf16* __restrict__ qlo, int64_t ldqp, int64_t qcols,
                   int M, int N, int Kpad, int nct, float* __restrict__ dt, int64_t lddt, int accumulate,
                   const float* __restrict__ alpha_ptr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const unsigned smem_base = lds_addr(smem);
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int ct = tile % nct, mt = tile / nct;
  const int m0 = mt * BM, n0 = ct * BN;
  const int nst = Kpad / BK;

  // DMA sources.  A: 16 wave-instructions per plane (two 512-B k-rows each), two per wave;
  // B: 8 per plane (four 256-B k-rows each), one per wave.  Columns past the plane's width
  // read its last chunk (they feed accumulator rows / columns that are never stored).
  const __bf16* a_src[2];
  unsigned a_dst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int inst = wave * 2 + i;
    const int k = 2 * inst + (lane >> 5), pos = lane & 31;
    const int cc = ((((pos >> 2) ^ (k & 3)) << 2) | ((((pos >> 1) & 1) ^ ((k >> 3) & 1)) << 1) | (pos & 1));
    a_src[i] = ghi + (int64_t)k * ldgp + min((int64_t)m0 + 8 * cc, gcols - 8);
    a_dst[i] = (unsigned)inst * 1024u;
  }
  const __bf16* b_src;
  {
    const int k = 4 * wave + (lane >> 4), pos = lane & 15;
    const int cc = ((((pos >> 2) ^ (k & 3)) << 2) | ((((pos >> 1) & 1) ^ ((k >> 3) & 1)) << 1) | (pos & 1));
    b_src = qhi + (int64_t)k * ldqp + min((int64_t)n0 + 8 * cc, qcols - 8);
  }
  const unsigned b_dst = (unsigned)wave * 1024u;
  const int64_t glo_off = glo - ghi, qlo_off = qlo - qhi;
  auto stage = [&](int buf, int st) {
    const unsigned base = smem_base + buf * STAGE;
    const int64_t ka = (int64_t)st * BK * ldgp, kq = (int64_t)st * BK * ldqp;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      glds16_asm(a_src[i] + ka, base + a_dst[i]);
      glds16_asm(a_src[i] + glo_off + ka, base + PLANE_A + a_dst[i]);
    }
    glds16_asm(b_src + kq, base + 2 * PLANE_A + b_dst);
    glds16_asm(b_src + qlo_off + kq, base + 2 * PLANE_A + PLANE_B + b_dst);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int x = 0; x < TM; ++x)
#pragma unroll
    for (int y = 0; y < TN; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const unsigned char* cur) {
    const unsigned char* ahi = cur;
    const unsigned char* alo = cur + PLANE_A;
    const unsigned char* bhi = cur + 2 * PLANE_A;
    const unsigned char* blo = bhi + PLANE_B;
    bf16x8 b_h[TN], b_l[TN];
#pragma unroll
    for (int y = 0; y < TN; ++y) {
      b_h[y] = tr_frag16<BN>(bhi, wc * WCOLS + y * 16, lane);
      b_l[y] = tr_frag16<BN>(blo, wc * WCOLS + y * 16, lane);
    }
#pragma unroll
    for (int x = 0; x < TM; ++x) {
      const bf16x8 a_h = tr_frag16<BM>(ahi, wr * (BM / WM) + x * 16, lane);
      const bf16x8 a_l = tr_frag16<BM>(alo, wr * (BM / WM) + x * 16, lane);
      if constexpr (GROUP) {
#pragma unroll
        for (int y = 0; y < TN; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_l, b_h[y], acc[x][y], 0, 0, 0);
#pragma unroll
        for (int y = 0; y < TN; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_h, b_l[y], acc[x][y], 0, 0, 0);
#pragma unroll
        for (int y = 0; y < TN; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_h, b_h[y], acc[x][y], 0, 0, 0);
      } else {
#pragma unroll
        for (int y = 0; y < TN; ++y) {
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_l, b_h[y], acc[x][y], 0, 0, 0);
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_h, b_l[y], acc[x][y], 0, 0, 0);
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_h, b_h[y], acc[x][y], 0, 0, 0);
        }
      }
    }
  };

  // Every vector-memory operation of the loop is an LDS-DMA issued from inline asm: the stage
  // st + 1 transfers are issued before stage st's MFMAs and waited for (vmcnt(0)) after them.
  if constexpr (NSTG == 3) {
    // Three buffers, branch-free: iteration st issues the transfers of stage st + 2 (the last K
    // chunk again once there is none: it lands in a buffer nobody reads any more) into the
    // buffer that stage st - 1 was read from, and waits until at most those 6 instructions are
    // outstanding -- vector-memory operations retire in order, so stage st + 1 has landed.
    stage(0, 0);
    stage(1, min(1, nst - 1));
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    int cur = 0, nxt2 = 2;  // buffer of stage st, buffer for stage st + 2
    for (int st = 0; st < nst; ++st) {
      stage(nxt2, min(st + 2, nst - 1));
      compute(smem + cur * STAGE);
      asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      nxt2 = cur;
      cur = cur == 2 ? 0 : cur + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the redundant tail transfers target LDS too
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int st = 0; st < nst; ++st) {
      if (st + 1 < nst) stage((st + 1) & 1, st + 1);  // uniform branch; no register loads in flight
      compute(smem + (st & 1) * STAGE);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  const float alpha = alpha_ptr ? *alpha_ptr : 1.f;
  store_tile(acc, smem, wave, lane, wr, wc, dt, lddt, m0, n0, M, N, alpha, accumulate != 0);
}

int g_bwdp_pipe = 1;    // dev builds can switch the dQ kernel back to its plain loop (kge_dev_bwdp_pipe)
int g_bwdp_stages = 3;  // ... and the dE kernel back to two LDS stage buffers (kge_dev_bwdp_stages)
int g_bwdp_group = 3;   // ... bit 0: dQ, bit 1: dE with the grouped MFMA order; 0: accumulator by accumulator (kge_dev_bwdp_group)

int splits_q(int64_t n, int64_t m, int d, int cus) {
  const int64_t tiles = ((n + BM - 1) / BM) * ((d + BN - 1) / BN);
  const int64_t by_k = std::max<int64_t>(1, (m + 8 * BK - 1) / (8 * BK));
  return (int)std::max<int64_t>(1, std::min<int64_t>(by_k, cus / std::max<int64_t>(1, tiles)));
}

void chunking(int64_t K, int& splits, int& kchunk) {
  kchunk = (int)((K + splits - 1) / splits);
  kchunk = (kchunk + BK - 1) / BK * BK;
  splits = (int)((K + kchunk - 1) / kchunk);
}

}  // namespace

extern "C" int64_t kge_score_dot_bwd_q_planes_ws_size(int64_t n, int64_t m, int d) {
  if (n <= 0 || m <= 0 || d <= 0) return 0;
  int splits = splits_q(n, m, d, kge_num_cus()), kchunk;
  chunking(m, splits, kchunk);
  return (int64_t)splits * n * d;
}

extern "C" int kge_score_dot_bwd_q_planes(const void* g_hi, const void* g_lo, int64_t ldgp, const float* t,
                                          int64_t ldt, int64_t n, int64_t m, int d, float* dq, int64_t lddq,
                                          int accumulate, const float* gscale, float* ws, int64_t ws_elems,
                                          void* stream) {
  KGE_REQUIRE(n > 0 && m > 0 && d >= 4 && n < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE(g_hi && g_lo && t && dq && ws && ldt >= d && lddq >= d);
  const int64_t mp = (m + BK - 1) / BK * BK;
  const int64_t lo_off = (const __bf16*)g_lo - (const __bf16*)g_hi;
  // each plane holds round_up(m, 32) columns (zero past m) and must not overlap the other
  KGE_REQUIRE(ldgp >= mp && (lo_off >= mp || lo_off <= -mp));
  if (d % 4 != 0 || ldt % 4 != 0 || lddq % 4 != 0 || ldgp % 8 != 0 || lo_off % 8 != 0 || !aligned16(g_hi) ||
      !aligned16(t) || !aligned16(dq) || !aligned16(ws))
    return KGE_ERR_ALIGN;
  int splits = splits_q(n, m, d, kge_num_cus()), kchunk;
  chunking(m, splits, kchunk);
  KGE_REQUIRE(ws_elems >= (int64_t)splits * n * d);
  hipStream_t st = as_stream(stream);
  static std::atomic<bool> lds_ok[KGE_MAX_DEVICES];
  static std::atomic<bool> lds_ok_plain[KGE_MAX_DEVICES];
  static std::atomic<bool> lds_ok_group[KGE_MAX_DEVICES];
  const bool pipe = g_bwdp_pipe != 0, group = pipe && (g_bwdp_group & 1);
  if (const int e = group  ? kge_allow_lds((const void*)bwd3p_q_kernel<true, true>, 2 * STAGE, lds_ok_group)
                    : pipe ? kge_allow_lds((const void*)bwd3p_q_kernel<true, false>, 2 * STAGE, lds_ok)
                           : kge_allow_lds((const void*)bwd3p_q_kernel<false, false>, 2 * STAGE, lds_ok_plain))
    return e;
  const int nrt = (int)((n + BM - 1) / BM), nct = (d + BN - 1) / BN;
  const int64_t blocks = (int64_t)nrt * nct * splits;
  if (blocks > 0x7fffffff) return KGE_ERR_ARG;
  auto kern = group ? bwd3p_q_kernel<true, true> : pipe ? bwd3p_q_kernel<true, false> : bwd3p_q_kernel<false, false>;
  kern<<<dim3((unsigned)blocks), dim3(NT), 2 * STAGE, st>>>((const __bf16*)g_hi, (const __bf16*)g_lo, ldgp, t, ldt, (int)n,
                                                            d, (int)m, kchunk, nrt, nct, ws);
  KGE_CHECK_LAUNCH();
  const int64_t total = n * (d / 4);
  const int sblocks = (int)std::min<int64_t>((total + 255) / 256, (int64_t)kge_num_cus() * 4);
  slab_sum_kernel<<<dim3(sblocks), dim3(256), 0, st>>>(ws, splits, n, d, dq, lddq, accumulate, gscale);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_score_dot_bwd_t_planes(const void* g_hi, const void* g_lo, int64_t ldgp, const void* q_hi,
                                          const void* q_lo, int64_t ldqp, int64_t n_pad, int64_t m, int d, float* dt,
                                          int64_t lddt, int accumulate, const float* gscale, void* stream) {
  KGE_REQUIRE(n_pad > 0 && n_pad % BK == 0 && m > 0 && d >= 8 && n_pad < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE(g_hi && g_lo && q_hi && q_lo && dt && lddt >= d);
  const int64_t glo = (const __bf16*)g_lo - (const __bf16*)g_hi, qlo = (const __bf16*)q_lo - (const __bf16*)q_hi;
  const int64_t gcols = (m + 7) / 8 * 8, qcols = (d + 7) / 8 * 8;  // plane widths read (zero past m / d)
  KGE_REQUIRE(ldgp >= gcols && ldqp >= qcols);
  if (d % 4 != 0 || lddt % 4 != 0 || ldgp % 8 != 0 || ldqp % 8 != 0 || glo % 8 != 0 || qlo % 8 != 0 ||
      !aligned16(g_hi) || !aligned16(q_hi) || !aligned16(dt))
    return KGE_ERR_ALIGN;
  hipStream_t st = as_stream(stream);
  static std::atomic<bool> lds_ok[KGE_MAX_DEVICES];
  static std::atomic<bool> lds_ok2[KGE_MAX_DEVICES];
  static std::atomic<bool> lds_ok_group[KGE_MAX_DEVICES];
  const bool three = g_bwdp_stages == 3, group = three && (g_bwdp_group & 2);
  if (const int e = group   ? kge_allow_lds((const void*)bwd3p_t_kernel<3, true>, 3 * STAGE, lds_ok_group)
                    : three ? kge_allow_lds((const void*)bwd3p_t_kernel<3, false>, 3 * STAGE, lds_ok)
                            : kge_allow_lds((const void*)bwd3p_t_kernel<2, false>, 2 * STAGE, lds_ok2))
    return e;
  const int nrt = (int)((m + BM - 1) / BM), nct = (d + BN - 1) / BN;
  const int64_t blocks = (int64_t)nrt * nct;
  if (blocks > 0x7fffffff) return KGE_ERR_ARG;
  auto kern = group ? bwd3p_t_kernel<3, true> : three ? bwd3p_t_kernel<3, false> : bwd3p_t_kernel<2, false>;
  kern<<<dim3((unsigned)blocks), dim3(NT), (three ? 3 : 2) * STAGE, st>>>(
      (const __bf16*)g_hi, (const __bf16*)g_lo, ldgp, gcols, (const __bf16*)q_hi, (const __bf16*)q_lo, ldqp, qcols,
      (int)m, d, (int)n_pad, nct, dt, lddt, accumulate, gscale);
  KGE_CHECK_LAUNCH();
  return 0;
}

#ifdef KGE_DEV_BUILD  // libkgescore_dev.so only
extern "C" void kge_dev_bwdp_pipe(int on) { g_bwdp_pipe = on; }
extern "C" void kge_dev_bwdp_stages(int n) { g_bwdp_stages = n == 2 ? 2 : 3; }
extern "C" void kge_dev_bwdp_group(int mask) { g_bwdp_group = mask & 3; }
#endif

// Persistent bf16x3 contraction S = Q . T^T (the production score_sp / score_po kernel):
// workgroups loop over output tiles (one tile per CU at the C2 shape).
//
// Per tile: Q arrives pre-split as bf16 hi / lo planes and is staged by LDS-DMA
// (global_load_lds_dwordx4); the entity rows are loaded into registers and split on the
// fly.  K is staged 32 columns at a time into a double-buffered, XOR-swizzled LDS image;
// one barrier per stage; 16x16x32 bf16 MFMA, hi*hi + hi*lo + lo*hi (measured 7 % faster
// than the 32x32x16 form of the same kernel: the chip holds a higher clock on the 16x16
// shape, MI355X_MICROARCH 'DVFS give-back' item 7).  Row-vector epilogue through LDS.
// Tile order is XCD-grouped: the workgroups that share an XCD take consecutive tiles, i.e.
// the query tiles of one entity panel, so each panel is read from HBM once per XCD.
#include "mfma16.h"

namespace {

constexpr int BK = KGE_BK;

template <int BM, int BN, int WM, int WN>
struct PCfg {
  static constexpr int NT = 64 * WM * WN;
  static constexpr int PLANE_A = BM * BK * 2;
  static constexpr int PLANE_B = BN * BK * 2;
  static constexpr int STAGE = 2 * PLANE_A + 2 * PLANE_B;
  static constexpr int B_PER_T = (BN * 8 + NT - 1) / NT;  // float4 slots per thread (last may idle)
  static_assert(BM % (16 * WM) == 0 && BN % (16 * WN) == 0, "tile");
};

// ---------------------------------------------------------------------------------------
// v_mfma_f32_16x16x32_bf16: one MFMA covers the whole BK = 32 stage, per wave
// (BM/WM/16) x (BN/WN/16) tiles of 16 x 16 (f32x4 accumulators); LDS image, inline-asm VMEM
// helpers: mfma16.h.  Epilogue: the four 16 x 16 tiles of a 16-row band go through a padded
// LDS scratch and leave as 256-B row segments of float4 stores.

// ABL: dev-only ablation / probe switches (kge_dev_score_dot_persist): 1 = no score stores,
// 2 = no staging after the prologue, 4 = per-workgroup clock probe written to row n of s,
// 8 = no barrier inside the K loop (timing only: the waves race on the LDS image),
// 16 / 32 = no query DMA / no entity staging, 64 = every panel reads rows 0 .. 63, 128 = the last
// round fills XCD after XCD, 256 = the three MFMAs of an accumulator in turn (see the loop).
// PIPE: the K loop software-pipelined inside each wave (see the loop): same barriers, same
// in-flight counts, same MFMA order per accumulator (bit-identical scores).
//
// RANK (the evaluation job's contraction): the scores never leave the registers.  The epilogue
// compares each accumulator with its row's true score and writes a 2-bit CODE per entry instead
// of the fp32 score -- 0: below the true score (also: the true column itself, columns past m),
// 1: above, 2: equal, 3: within the row's refinement band of the true score (to be rescored
// exactly by the ranking kernel) -- 16 codes per 32-bit word, 1/16 of the score block's bytes.
// Word layout of a row: word (j / 64) * 4 + (j % 16) / 4 holds column j's code at bit
// 8 * ((j % 64) / 16) + 2 * (j % 4)  (kge_rank_code_of in rank.hip decodes it).
struct RankEpi {
  // rows [0, n_a) are query batch A, rows [n_a, n) batch B: each brings its true scores and the
  // global column of its true entry
  const float* true_score_a;
  const int64_t* true_idx_a;
  const float* true_score_b;
  const int64_t* true_idx_b;
  int n_a;
  const float* band;        // [n] |score - true| <= band -> code 3 (negative: never)
  int64_t c0;               // global column of this table's row 0
  unsigned* codes;          // [n, ldc]
  int64_t ldc;              // words per row: ceil(m / 256) * 16
};

// The lane id computed where it is called (volatile asm: never hoisted out of a loop and kept in
// a register, or spilled, across it).
__device__ __forceinline__ int lane_id_here() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

template <int BM, int BN, int WM, int WN, int ABL = 0, bool PIPE = false, bool RANK = false>
__global__ void __launch_bounds__(64 * WM * WN, 1)
    score_dot_persist16_kernel(const __bf16* __restrict__ qhi, const __bf16* __restrict__ qlo, int64_t ldq,
                               const float* __restrict__ t, int64_t ldt, const int64_t* __restrict__ tidx, int n,
                               int m, int d, float* __restrict__ s, int64_t lds, int nrt, int ntiles,
                               const RankEpi re) {
  static_assert(!RANK || (PIPE && BN == 256 && WN == 4), "the code words assume transposed accumulators, 64-column waves");
  using C = PCfg<BM, BN, WM, WN>;
  constexpr int NW = C::NT / 64;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // 16 x 16 tiles per wave
  constexpr int WCOLS = BN / WN;                         // wave tile width
  constexpr int SCR_LD = WCOLS + 4;                      // padded scratch row (floats)
  constexpr int A_G = BM / 16 / NW;                      // 1-KB A chunks per plane per wave
  constexpr int XS = TM / 4 > 0 ? TM / 4 : 1;            // bands computed before the staging block
  static_assert((BM / 16) % NW == 0, "A chunks");
  static_assert(C::B_PER_T == 8 || C::B_PER_T == 4 || C::B_PER_T == 2, "KGE_WAIT_VM names the B registers");
  static_assert(WN > 1, "x-outer band loop");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int fr = lane & 15, fs = lane >> 4;
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, per_xcd = G >> 3, local = blockIdx.x >> 3;
  const int nst = (d + BK - 1) / BK;
  const unsigned smem_base = lds_addr(smem);
  const int64_t lo_off = qlo - qhi;
  const uint64_t t_clk0 = (ABL & 4) ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t t_rt0 = (ABL & 4) ? __builtin_amdgcn_s_memrealtime() : 0;
  uint64_t t_loop0 = 0, t_loop1 = 0;  // dev probe: K loop entry / exit of the last tile

  for (int it = 0;; ++it) {
    // Round `it` covers tiles [it G, it G + count): XCD x takes the x-th eighth of them,
    // consecutive tiles (the query tiles of one entity panel) staying on one XCD.  A last,
    // partial round is spread evenly too: 228 tiles on 256 CUs leave 3-4 CUs idle on EVERY XCD
    // (and use all eight L2s and fabric ports) instead of 28 on one.
    int tile;
    if constexpr (ABL & 128) {  // dev: the last round fills XCD after XCD
      tile = it * G + xcd * per_xcd + local;
      if (tile >= ntiles) break;
    } else {
      const int base = it * G;
      if (base >= ntiles) break;
      const int count = min(G, ntiles - base);
      const int lo = (int)((int64_t)xcd * count / 8), hi = (int)((int64_t)(xcd + 1) * count / 8);
      if (local >= hi - lo) break;  // only in the last round: no later tile either
      tile = base + lo + local;
    }
    const int m0 = (tile % nrt) * BM, n0 = (tile / nrt) * BN;

    // A planes by LDS-DMA: wave-instruction c fills rows 16c .. 16c+15 of a plane (64 B
    // each, lane-linear destination), so the 16x16x32 read swizzle goes on the source
    // address.  Rows past n read row n-1: their scores are never stored.
    // RANK: the thread coordinates of the prologue are taken behind an opaque asm, so that the
    // per-slot row numbers derived from them are recomputed per tile instead of being kept
    // (spilled) across the K loop, whose registers that variant has no room to share
    int tid_t = tid;
    if constexpr (RANK) {  // the thread id anew (wave is scalar, the lane id comes from mbcnt)
      tid_t = wave * 64 + lane_id_here();
    }
    const int lane_t = tid_t & 63;
    const __bf16* ga[A_G];
#pragma unroll
    for (int i = 0; i < A_G; ++i) {
      const int row = (wave * A_G + i) * 16 + (lane_t >> 2);
      const int slot = (lane_t & 3) ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3);
      ga[i] = qhi + (int64_t)min(m0 + row, n - 1) * ldq + slot * 8;
    }
    // B (entity rows, fp32) through registers: float4 f of the stage = row f / 8, cols 4 (f % 8)
    // slot i of thread tid: row tid / 8 + i NT / 8, columns 4 (tid % 8) .. +3; NT / 8 is a
    // multiple of 16 rows, so the swizzle term is the same for every slot
    static_assert(C::NT % 128 == 0, "B slot stride");
    const float* b_src[C::B_PER_T];
    constexpr bool B_RAGGED = BN * 8 % C::NT != 0;  // the last slot of some threads idles
    const bool b_last = !B_RAGGED || tid_t + (C::B_PER_T - 1) * C::NT < BN * 8;
    const int b_col = (tid_t & 7) * 4;
    const int b_off0 = sw16_off(tid_t >> 3, b_col >> 3) + ((b_col >> 2) & 1) * 8;
#pragma unroll
    for (int i = 0; i < C::B_PER_T; ++i) {
      const int row = min((tid_t >> 3) + i * (C::NT / 8), BN - 1);
      const int ej = n0 + row;  // rows past m read row 0: their scores are never stored
      const int64_t er = ej < m ? ((!RANK && tidx) ? tidx[ej] : (int64_t)ej) : 0;
      b_src[i] = t + ((ABL & 64) ? (er & 63) : er) * ldt + b_col;  // dev 64: every panel reads rows 0 .. 63
    }
    u32x4 rv[C::B_PER_T];

    // Every VMEM operation of the K loop is inline asm, counted by hand: per stage a wave
    // issues 2 A_G DMAs (stage st + 1), then B_PER_T register loads (stage st + 2).
#define KGE_WAIT_VM(N)                                                                                   \
  do {                                                                                                   \
    if constexpr (C::B_PER_T == 8)                                                                       \
      asm volatile("s_waitcnt vmcnt(%8)"                                                                 \
                   : "+v"(rv[0]), "+v"(rv[1]), "+v"(rv[2]), "+v"(rv[3]), "+v"(rv[4]), "+v"(rv[5]),       \
                     "+v"(rv[6]), "+v"(rv[7])                                                            \
                   : "i"(N)                                                                              \
                   : "memory");                                                                          \
    else if constexpr (C::B_PER_T == 4)                                                                  \
      asm volatile("s_waitcnt vmcnt(%4)" : "+v"(rv[0]), "+v"(rv[1]), "+v"(rv[2]), "+v"(rv[3]) : "i"(N) : "memory"); \
    else                                                                                                 \
      asm volatile("s_waitcnt vmcnt(%2)" : "+v"(rv[0]), "+v"(rv[C::B_PER_T - 1]) : "i"(N) : "memory");  \
  } while (0)
    auto glds_a = [&](int buf, int k0) {
      const unsigned base = smem_base + buf * C::STAGE;
#pragma unroll
      for (int i = 0; i < A_G; ++i) {
        const unsigned c = (unsigned)(wave * A_G + i) * 1024u;
        glds16_asm(ga[i] + k0, base + c);
        glds16_asm(ga[i] + lo_off + k0, base + C::PLANE_A + c);
      }
    };
    auto load_b = [&](int k0) {
#pragma unroll
      for (int i = 0; i < C::B_PER_T; ++i) rv[i] = gload16_asm(b_src[i] + min(k0, d - 4 - b_col));
    };
    // split fp32 -> bf16 hi / lo into the LDS image; only the K-tail stage masks (the
    // branch is wave-uniform)
    auto store_b = [&](unsigned char* stg, int k0) {
      unsigned char* bhi = stg + 2 * C::PLANE_A;
      unsigned char* blo = bhi + C::PLANE_B;
      const bool tail = k0 + BK > d;
      const unsigned mk = (!tail || k0 + b_col < d) ? 0xffffffffu : 0u;
      auto put = [&](bool masked) {
#pragma unroll
        for (int i = 0; i < C::B_PER_T; ++i) {
          float4 v = make_float4(__uint_as_float(rv[i].x), __uint_as_float(rv[i].y), __uint_as_float(rv[i].z),
                                 __uint_as_float(rv[i].w));
          if (masked)
            v = make_float4(__uint_as_float(rv[i].x & mk), __uint_as_float(rv[i].y & mk),
                            __uint_as_float(rv[i].z & mk), __uint_as_float(rv[i].w & mk));
          bf16x4 h, l;
          split_bf16x4_pk(v, h, l);
          if (i == C::B_PER_T - 1 && !b_last) continue;
          *reinterpret_cast<bf16x4*>(bhi + b_off0 + i * (C::NT / 8) * 64) = h;
          *reinterpret_cast<bf16x4*>(blo + b_off0 + i * (C::NT / 8) * 64) = l;
        }
      };
      if (tail)  // wave-uniform
        put(true);
      else
        put(false);
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int x = 0; x < TM; ++x)
#pragma unroll
      for (int y = 0; y < TN; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

    bf16x8 b_h[TN], b_l[TN];
    auto compute_b = [&](const unsigned char* cur) {
      const unsigned char* bhi = cur + 2 * C::PLANE_A;
      const unsigned char* blo = bhi + C::PLANE_B;
#pragma unroll
      for (int y = 0; y < TN; ++y) {
        const int rb_ = wc * WCOLS + y * 16 + fr;
        b_h[y] = *reinterpret_cast<const bf16x8*>(bhi + sw16_off(rb_, fs));
        b_l[y] = *reinterpret_cast<const bf16x8*>(blo + sw16_off(rb_, fs));
      }
    };
    auto compute_x = [&](const unsigned char* cur, int x0, int x1) {
      const unsigned char* ahi = cur;
      const unsigned char* alo = cur + C::PLANE_A;
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
    store_b(smem, 0);
    if (nst > 1) load_b(BK);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ABL & 4) t_loop0 = __builtin_amdgcn_s_memtime();
    if constexpr (PIPE) {
      // Inside a wave nothing but the matrix pipe should ever be waited for, so every LDS read
      // is issued a band (12 MFMAs) before its use: band x + 1's A fragments while band x runs,
      // and across the barrier the last band of a stage is held back -- its operands are in
      // registers -- and runs while the next stage's first fragments are fetched (each B
      // fragment is replaced as soon as the held band has used it).  The split of the entity
      // rows is spread, one float4 slot at a time, over the bands from XS on, each slot's
      // register load for stage st + 2 issued right behind it.
      // MFMA order inside a band: three runs over the band's TN accumulators -- lo(query) x
      // hi(entity), hi x lo, hi x hi -- so that one query fragment stays on the matrix pipe's
      // operand port for TN instructions in a row and consecutive MFMAs never share an
      // accumulator.  Per accumulator the three products still arrive in that order, so the
      // scores are bit-identical to issuing them accumulator by accumulator (ABL & 256, dev);
      // measured 0.5-2.5 % faster on this power-limited part.
      static_assert(TM >= 4 && TM % 2 == 0 && !B_RAGGED && (ABL & 8) == 0, "band pipeline");
      constexpr int PXS = TM >= 8 ? 2 : 1;      // first band that stages
      constexpr int PNB = TM - 1 - PXS;         // bands that stage
      bf16x8 ah[2], al[2];
      auto read_a = [&](const unsigned char* stg, int x, int slot) {
        const int ra = wr * (BM / WM) + x * 16 + fr;
        ah[slot] = *reinterpret_cast<const bf16x8*>(stg + sw16_off(ra, fs));
        al[slot] = *reinterpret_cast<const bf16x8*>(stg + C::PLANE_A + sw16_off(ra, fs));
      };
      auto read_b = [&](const unsigned char* stg, int y) {
        const int rb_ = wc * WCOLS + y * 16 + fr;
        b_h[y] = *reinterpret_cast<const bf16x8*>(stg + 2 * C::PLANE_A + sw16_off(rb_, fs));
        b_l[y] = *reinterpret_cast<const bf16x8*>(stg + 2 * C::PLANE_A + C::PLANE_B + sw16_off(rb_, fs));
      };
      // the entity fragment goes first: the 16 x 16 result comes out transposed (same sums, bit
      // for bit), a lane holding four CONSECUTIVE entities of one query row -- the epilogue
      // then moves whole float4s through its LDS scratch
      auto mfma3 = [&](int x, int y, int slot) {
        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b_h[y], al[slot], acc[x][y], 0, 0, 0);
        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b_l[y], ah[slot], acc[x][y], 0, 0, 0);
        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b_h[y], ah[slot], acc[x][y], 0, 0, 0);
      };
      // same issue order as at the end of the loop body: the waits at the loop head then only
      // cover what the first MFMAs need
      read_a(smem, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int y = 0; y < TN; ++y) {
        read_b(smem, y);
        __builtin_amdgcn_sched_barrier(0);
      }
      for (int st = 0; st < nst; ++st) {
        const int nb = (st + 1) & 1;
        const unsigned char* cur = smem + (st & 1) * C::STAGE;
        unsigned char* nxt = smem + nb * C::STAGE;
        const int k1 = min(st + 1, nst - 1) * BK;
        const int koff = min(min(st + 2, nst - 1) * BK, d - 4 - b_col);
        const unsigned mk = (k1 + b_col < d) ? 0xffffffffu : 0u;  // zero past the K tail
        // dev ablations (timing only): 2 = no staging at all, 16 = no A DMA, 32 = no B staging
        if constexpr (!(ABL & (2 | 16))) glds_a(nb, k1);
#pragma unroll
        for (int x = 0; x < TM - 1; ++x) {
          read_a(cur, x + 1, (x + 1) & 1);
          if (x == PXS && !(ABL & (2 | 32))) KGE_WAIT_VM((ABL & 16) ? 0 : 2 * A_G);  // B(st + 1) has landed
#pragma unroll
          for (int i = 0; i < C::B_PER_T; ++i) {
            if (PXS + i * PNB / C::B_PER_T != x || (ABL & (2 | 32))) continue;
            const float4 v = make_float4(__uint_as_float(rv[i].x & mk), __uint_as_float(rv[i].y & mk),
                                         __uint_as_float(rv[i].z & mk), __uint_as_float(rv[i].w & mk));
            bf16x4 h, l;
            split_bf16x4_pk(v, h, l);
            *reinterpret_cast<bf16x4*>(nxt + 2 * C::PLANE_A + b_off0 + i * (C::NT / 8) * 64) = h;
            *reinterpret_cast<bf16x4*>(nxt + 2 * C::PLANE_A + C::PLANE_B + b_off0 + i * (C::NT / 8) * 64) = l;
            rv[i] = gload16_asm(b_src[i] + koff);
          }
          if constexpr (!(ABL & 256)) {  // one query fragment held over the band's four accumulators
#pragma unroll
            for (int y = 0; y < TN; ++y)
              acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b_h[y], al[x & 1], acc[x][y], 0, 0, 0);
#pragma unroll
            for (int y = 0; y < TN; ++y)
              acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b_l[y], ah[x & 1], acc[x][y], 0, 0, 0);
#pragma unroll
            for (int y = 0; y < TN; ++y)
              acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b_h[y], ah[x & 1], acc[x][y], 0, 0, 0);
          } else {
#pragma unroll
            for (int y = 0; y < TN; ++y) mfma3(x, y, x & 1);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        KGE_WAIT_VM((ABL & 32) ? 0 : C::B_PER_T);  // A(st + 1) has landed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        read_a(nxt, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(ABL & 256)) {
          constexpr int HS = (TM - 1) & 1;
#pragma unroll
          for (int y = 0; y < TN; ++y)
            acc[TM - 1][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b_h[y], al[HS], acc[TM - 1][y], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int y = 0; y < TN; ++y) {
            acc[TM - 1][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b_l[y], ah[HS], acc[TM - 1][y], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            const int rb_ = wc * WCOLS + y * 16 + fr;
            b_l[y] = *reinterpret_cast<const bf16x8*>(nxt + 2 * C::PLANE_A + C::PLANE_B + sw16_off(rb_, fs));
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int y = 0; y < TN; ++y) {
            acc[TM - 1][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b_h[y], ah[HS], acc[TM - 1][y], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            const int rb_ = wc * WCOLS + y * 16 + fr;
            b_h[y] = *reinterpret_cast<const bf16x8*>(nxt + 2 * C::PLANE_A + sw16_off(rb_, fs));
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
    // One barrier per stage.  Stage st + 1 is staged into the other buffer between the first
    // XS bands of stage st's MFMAs and the rest (measured: 8 % over staging ahead of them).
    // The stage body is branch-free: the last stage re-stages its own K chunk into the idle
    // buffer, so every path keeps the same in-flight counts and the B registers stay put --
    // with a conditional wait, hipcc copied the registers of loads still in flight at the
    // merge and reused them (a rare memory fault under multi-tile schedules).
    for (int st = 0; st < nst; ++st) {
      const int nb = (st + 1) & 1;
      const unsigned char* cur = smem + (st & 1) * C::STAGE;
      const int k1 = min(st + 1, nst - 1) * BK;
      if constexpr (!(ABL & 2)) glds_a(nb, k1);
      compute_b(cur);
      compute_x(cur, 0, XS);
      if constexpr (!(ABL & 2)) {
        KGE_WAIT_VM(2 * A_G);  // B(st + 1) has landed
        store_b(smem + nb * C::STAGE, k1);
        load_b(min(st + 2, nst - 1) * BK);
      }
      compute_x(cur, XS, TM);
      KGE_WAIT_VM(C::B_PER_T);  // A(st + 1) has landed
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (!(ABL & 8)) __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    KGE_WAIT_VM(0);
#undef KGE_WAIT_VM
    if (ABL & 4) t_loop1 = __builtin_amdgcn_s_memtime();

    if constexpr (RANK) {
      // transposed accumulators: acc[x][y][r] = row (lane & 15) of band x, column 16 y + 4 fs + r
      // of this wave's 64 columns; one code word per lane and band.  The lane coordinates are
      // re-derived behind an opaque asm so that nothing of the epilogue's address arithmetic is
      // hoisted out of the tile loop and kept alive across the K loop (no register to spare there);
      // the lane id itself comes from mbcnt, not from a register kept since kernel entry.
      const int lane_e = lane_id_here();
      const int fr_e = lane_e & 15, fs_e = lane_e >> 4;
      const int jw = n0 + wc * WCOLS;  // first column of the wave (a multiple of 64)
      auto row_info = [&](int x, float& ts, float& bd, int& tjr) {
        const int ic = min(m0 + wr * (BM / WM) + x * 16 + fr_e, n - 1);
        const bool in_a = ic < re.n_a;
        const float v = in_a ? re.true_score_a[ic] : re.true_score_b[ic - re.n_a];
        ts = v == v ? v : -INFINITY;
        bd = re.band[ic];
        const int64_t tj = (in_a ? re.true_idx_a[ic] : re.true_idx_b[ic - re.n_a]) - re.c0 - jw;  // wave-relative
        tjr = (tj >= 0 && tj < WCOLS) ? (int)tj : -1;
      };
      float ts_n, bd_n;
      int tj_n;
      row_info(0, ts_n, bd_n, tj_n);
#pragma unroll
      for (int x = 0; x < TM; ++x) {
        const float ts = ts_n, bd = bd_n;
        const int tjr = tj_n;
        if (x + 1 < TM) row_info(x + 1, ts_n, bd_n, tj_n);
        unsigned word = 0;
        if (__builtin_expect(__any(__builtin_fabsf(ts) == INFINITY), 0)) {
          // a row whose true score is infinite (or was NaN): comparisons as they are written down
#pragma unroll
          for (int y = 0; y < TN; ++y) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = acc[x][y][r];
              v = v == v ? v : -INFINITY;
              unsigned code = (v > ts) ? 1u : ((v == ts) ? 2u : 0u);
              code = (__builtin_fabsf(v - ts) <= bd) ? 3u : code;
              word |= code << (8 * y + 2 * r);
            }
          }
        } else {
          // A finite true score: "inside the band" is |v - ts| <= bd, and v == ts lies inside every
          // band >= 0, so a refined row needs no equality test; an unrefined row (bd < 0) takes
          // the band 0, whose members ARE the ties -- their code 3 is turned into 2 below.  A NaN
          // score fails both comparisons (code 0, as -inf would), an infinite one is outside any band.
          const float bd0 = bd < 0.f ? 0.f : bd;
#pragma unroll
          for (int y = 0; y < TN; ++y) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = acc[x][y][r];
              unsigned code = (v > ts) ? (1u << (8 * y + 2 * r)) : 0u;
              code = (__builtin_fabsf(v - ts) <= bd0) ? (3u << (8 * y + 2 * r)) : code;
              word |= code;
            }
          }
          if (bd < 0.f) word ^= word & (word >> 1) & 0x55555555u;  // 3 -> 2
        }
        // the true column and the columns past m carry code 0
        if (tjr >= 0 && ((tjr >> 2) & 3) == fs_e) word &= ~(3u << (8 * (tjr >> 4) + 2 * (tjr & 3)));
        if (m - jw < WCOLS) {
#pragma unroll
          for (int y = 0; y < TN; ++y) {
            const int rem = m - jw - (y * 16 + 4 * fs_e);  // columns 16 y + 4 fs + r with r >= rem lie past m
            const unsigned keep = rem >= 4 ? 0xFFu : (rem <= 0 ? 0u : ((1u << (2 * rem)) - 1u));
            word &= ~(0xFFu << (8 * y)) | (keep << (8 * y));
          }
        }
        const int i = m0 + wr * (BM / WM) + x * 16 + fr_e;
        if (i < n) re.codes[(int64_t)i * re.ldc + (jw >> 6) * 4 + fs_e] = word;
      }
      __syncthreads();  // every wave has read its last K stage: the next tile's prologue may overwrite LDS
      continue;
    }
    // epilogue: C/D of 16x16 -- lane holds column (lane & 15), rows 4 (lane >> 4) + r
    __syncthreads();  // stage buffers free: per-wave scratch of 16 rows x WCOLS (+4) floats
    float* scr = reinterpret_cast<float*>(smem) + wave * 16 * SCR_LD;
    constexpr int LPR = WCOLS / 4;  // lanes per scratch row (float4 each)
#pragma unroll
    for (int x = 0; x < TM; ++x) {
#pragma unroll
      for (int y = 0; y < TN; ++y) {
        if constexpr (PIPE) {  // transposed accumulators: row (lane & 15), columns 4 (lane >> 4) .. + 3
          *reinterpret_cast<f32x4*>(scr + fr * SCR_LD + y * 16 + 4 * fs) = acc[x][y];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) scr[(4 * fs + r) * SCR_LD + y * 16 + fr] = acc[x][y][r];
        }
      }
      const int i0 = m0 + wr * (BM / WM) + x * 16;
#pragma unroll
      for (int pass = 0; pass < (16 * LPR + 63) / 64; ++pass) {
        const int g = pass * 64 + lane;  // float4 g of the band: row g / LPR, column 4 (g % LPR)
        const int row = g / LPR, c4 = g % LPR;
        const int i = i0 + row;
        if ((16 * LPR) % 64 != 0 && g >= 16 * LPR) continue;
        const float4 v = *reinterpret_cast<const float4*>(scr + row * SCR_LD + c4 * 4);
        const int j = n0 + wc * WCOLS + c4 * 4;
        if (i >= n) continue;
        float* dst = s + (int64_t)i * lds + j;
        if (ABL & 1) {
          if (v.x == 1234.5f) dst[0] = v.y;  // keep the values live, store (almost) nothing
        } else if (j + 3 < m) {
          *reinterpret_cast<f32x4u*>(dst) = f32x4u{v.x, v.y, v.z, v.w};
        } else {
          if (j < m) dst[0] = v.x;
          if (j + 1 < m) dst[1] = v.y;
          if (j + 2 < m) dst[2] = v.z;
        }
      }
    }
    __syncthreads();  // LDS of this tile is free for the next tile's prologue
  }
  if ((ABL & 4) && tid == 0) {  // dev: shader clocks and 100-MHz ticks spent by this workgroup
    const uint64_t c = __builtin_amdgcn_s_memtime() - t_clk0, r = __builtin_amdgcn_s_memrealtime() - t_rt0;
    s[(int64_t)n * lds + 2 * blockIdx.x] = (float)c;  // the caller allocates rows n, n + 1
    s[(int64_t)n * lds + 2 * blockIdx.x + 1] = (float)r;
    s[(int64_t)(n + 1) * lds + 2 * blockIdx.x] = (float)(t_loop0 - t_clk0);
    s[(int64_t)(n + 1) * lds + 2 * blockIdx.x + 1] = (float)(t_loop1 - t_clk0);
  }
}

template <int BM, int BN, int WM, int WN, int ABL = 0, bool PIPE = false, bool RANK = false>
int launch_persist16(const __bf16* qhi, const __bf16* qlo, int64_t ldq, const float* t, int64_t ldt,
                     const int64_t* tidx, int64_t n, int64_t m, int d, float* s, int64_t lds, hipStream_t st,
                     const RankEpi re = RankEpi{}) {
  using C = PCfg<BM, BN, WM, WN>;
  const int nrt = (int)((n + BM - 1) / BM);
  const int64_t ntiles = (int64_t)nrt * ((m + BN - 1) / BN);
  if (ntiles > 0x7fffffff) return KGE_ERR_ARG;
  const size_t shmem = 2 * C::STAGE;
  static std::atomic<bool> lds_ok[KGE_MAX_DEVICES];
  if (const int e = kge_allow_lds((const void*)score_dot_persist16_kernel<BM, BN, WM, WN, ABL, PIPE, RANK>, (int)shmem,
                                  lds_ok))
    return e;
  int grid = kge_num_cus();
  grid = (int)std::min<int64_t>(grid, (ntiles + 7) / 8 * 8);
  grid = std::max(8, grid / 8 * 8);
  score_dot_persist16_kernel<BM, BN, WM, WN, ABL, PIPE, RANK><<<dim3(grid), dim3(C::NT), shmem, st>>>(
      qhi, qlo, ldq, t, ldt, tidx, (int)n, (int)m, d, s, lds, nrt, (int)ntiles, re);
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

#ifdef KGE_DEV_BUILD
static int g_dot3_pipe = 1;
extern "C" void kge_dev_dot3_pipe(int on) { g_dot3_pipe = on; }
#endif

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
#ifdef KGE_DEV_BUILD  // A/B against the XCD-after-XCD last round (2) and the plain K loop (0)
  if (g_dot3_pipe == 2) {
    if (n > 128) return launch_persist16<256, 256, 2, 4, 128, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    return launch_persist16<128, 256, 2, 4, 128, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
  }
  if (g_dot3_pipe == 3) {  // the three MFMAs of each accumulator in turn
    if (n > 128) return launch_persist16<256, 256, 2, 4, 256, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    return launch_persist16<128, 256, 2, 4, 256, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
  }
  if (!g_dot3_pipe) {
    if (n > 128) return launch_persist16<256, 256, 2, 4>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    return launch_persist16<128, 256, 2, 4>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
  }
#endif
  // 256- or 128-row tiles (bit-identical scores): the workgroups take whole rounds of tiles and a
  // partial last round costs a full tile time, so the cheaper of the two schedules is chosen --
  // a 128-row tile measures 0.55 of a 256-row tile (its MFMA work is half, its entity staging the
  // same).  E.g. 512 x 40,943: 320 tiles = 2 rounds vs 640 half tiles = 3 rounds * 0.55.
  const int64_t slots = std::max(8, kge_num_cus() / 8 * 8);
  const int64_t panels = (m + 255) / 256;
  const double cost256 = (double)((((n + 255) / 256) * panels + slots - 1) / slots);
  const double cost128 = 0.55 * (double)((((n + 127) / 128) * panels + slots - 1) / slots);
  if (n > 128 && cost256 <= cost128)
    return launch_persist16<256, 256, 2, 4, 0, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
  return launch_persist16<128, 256, 2, 4, 0, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
}

extern "C" int64_t kge_rank_codes_ld(int64_t m) { return m <= 0 ? 0 : (m + 255) / 256 * 16; }

extern "C" int kge_score_dot_split_rank(const void* qhi, const void* qlo, int64_t ldq, const float* t, int64_t ldt,
                                        int64_t n_a, int64_t n_b, int64_t m, int d, const float* true_score_a,
                                        const int64_t* true_idx_a, const float* true_score_b,
                                        const int64_t* true_idx_b, const float* band, int64_t c0, void* codes,
                                        int64_t ldc, void* stream) {
  const int64_t n = n_a + n_b;
  KGE_REQUIRE(n_a >= 0 && n_b >= 0 && m >= 0 && d >= 4 && n < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE(qhi && qlo && t && ldt >= d && band && codes && ldc >= kge_rank_codes_ld(m));
  KGE_REQUIRE((n_a == 0 || (true_score_a && true_idx_a)) && (n_b == 0 || (true_score_b && true_idx_b)));
  KGE_REQUIRE(ldq % 8 == 0 && ldq >= ((d + 31) / 32) * 32);
  if (d % 4 != 0 || ldt % 4 != 0 || !aligned16(t) || !aligned16(qhi) || !aligned16(qlo)) return KGE_ERR_ALIGN;
  if (n == 0 || m == 0) return 0;
  hipStream_t st = as_stream(stream);
  const __bf16* h = (const __bf16*)qhi;
  const __bf16* l = (const __bf16*)qlo;
  const RankEpi re{true_score_a, true_idx_a, true_score_b, true_idx_b, (int)n_a, band, c0, (unsigned*)codes, ldc};
  // tile height as in kge_score_dot_split (the code words do not depend on it)
  const int64_t slots = std::max(8, kge_num_cus() / 8 * 8);
  const int64_t panels = (m + 255) / 256;
  const double cost256 = (double)((((n + 255) / 256) * panels + slots - 1) / slots);
  const double cost128 = 0.55 * (double)((((n + 127) / 128) * panels + slots - 1) / slots);
  if (n > 128 && cost256 <= cost128)
    return launch_persist16<256, 256, 2, 4, 0, true, true>(h, l, ldq, t, ldt, nullptr, n, m, d, nullptr, 0, st, re);
  return launch_persist16<128, 256, 2, 4, 0, true, true>(h, l, ldq, t, ldt, nullptr, n, m, d, nullptr, 0, st, re);
}

#ifdef KGE_DEV_BUILD  // libkgescore_dev.so only: ablation / probe variants for scripts/dev
extern "C" int kge_dev_score_dot_persist(int variant, const void* qhi, const void* qlo, int64_t ldq,
                                         const float* t, int64_t ldt, const int64_t* tidx, int64_t n, int64_t m,
                                         int d, float* s, int64_t lds, void* stream) {
  KGE_REQUIRE(n > 0 && m > 0 && d >= 4 && ldq % 8 == 0 && ldq >= ((d + 31) / 32) * 32);
  KGE_REQUIRE(d % 4 == 0 && ldt % 4 == 0 && aligned16(t) && aligned16(qhi) && aligned16(qlo));
  hipStream_t st = as_stream(stream);
  const __bf16* h = (const __bf16*)qhi;
  const __bf16* l = (const __bf16*)qlo;
  switch (variant) {
    case 0: return launch_persist16<256, 256, 2, 4>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 1: return launch_persist16<128, 256, 2, 4>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 11: return launch_persist16<256, 256, 2, 4, 1>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 12: return launch_persist16<256, 256, 2, 4, 2>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 13: return launch_persist16<256, 256, 2, 4, 3>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 14: return launch_persist16<256, 256, 2, 4, 4>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 18: return launch_persist16<256, 256, 2, 4, 8>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 19: return launch_persist16<256, 256, 2, 4, 11>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    // one wave per SIMD, 128 x 128 wave tiles (accumulators in AGPRs)
    case 20: return launch_persist16<256, 256, 2, 2>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 24: return launch_persist16<256, 256, 2, 2, 4>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    // K loop software-pipelined inside each wave
    case 30: return launch_persist16<256, 256, 2, 4, 0, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 31: return launch_persist16<128, 256, 2, 4, 0, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 34: return launch_persist16<256, 256, 2, 4, 4, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    // one wave per SIMD, 128 x 128 wave tiles, pipelined
    case 35: return launch_persist16<256, 256, 2, 2, 0, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 36: return launch_persist16<256, 256, 2, 2, 4, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 37: return launch_persist16<256, 256, 2, 4, 128, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 38: return launch_persist16<256, 256, 2, 4, 128 + 4, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 41: return launch_persist16<256, 256, 2, 4, 1, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 42: return launch_persist16<256, 256, 2, 4, 2, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 43: return launch_persist16<256, 256, 2, 4, 3, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 44: return launch_persist16<256, 256, 2, 4, 16, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 45: return launch_persist16<256, 256, 2, 4, 32, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 46: return launch_persist16<256, 256, 2, 4, 64, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 51: return launch_persist16<256, 256, 2, 4, 5, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 52: return launch_persist16<256, 256, 2, 4, 6, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 53: return launch_persist16<256, 256, 2, 4, 7, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    // 128 x 128 tiles, four waves, 64 KB of LDS: two workgroups (of two launches on two streams) fit a CU
    // the three MFMAs of each accumulator in turn (the order before the grouped one)
    case 70: return launch_persist16<256, 256, 2, 4, 256, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 60: return launch_persist16<128, 128, 2, 2, 0, true>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    case 61: return launch_persist16<128, 128, 2, 2>(h, l, ldq, t, ldt, tidx, n, m, d, s, lds, st);
    default: return KGE_ERR_ARG;
  }
}
#endif  // KGE_DEV_BUILD

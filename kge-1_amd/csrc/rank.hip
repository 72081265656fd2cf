// Entity-ranking counts and rank histograms (EntityRankingJob, entity_ranking.py:139-216,
// 469-551; eval.py:148-171).
//
// Raw counts take one coalesced pass over the score row.  Filtering is applied as a
// correction over the (short) per-query filter lists instead of materialising dense
// +inf label chunks (entity_ranking.py:428-467): an entry j in the filter set F_i moves
// from its raw value v_j to -inf, so
//   greater_filt = greater_raw - [v_j > t] ,  ties_filt = ties_raw - [v_j == t] + [t == -inf]
// summed over the unique filtered j inside the chunk (the true entity excluded).  That is
// exactly `scores - labels` followed by NaN -> -inf and the two comparisons, including
// the -inf / NaN corner cases.
#include "common.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float clean(float v) { return (v != v) ? -INFINITY : v; }

__device__ __forceinline__ void block_sum2(int64_t& a, int64_t& b, int64_t* sm) {
  // wave reduce then LDS
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    sm[wave] = a;
    sm[8 + wave] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t x = 0, y = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      x += sm[w];
      y += sm[8 + w];
    }
    a = x;
    b = y;
  }
}

__global__ void __launch_bounds__(NT) rank_counts_kernel(const float* __restrict__ s, int64_t lds, int64_t n,
                                                         int64_t m, int64_t c0, const int64_t* __restrict__ true_idx,
                                                         const float* __restrict__ true_score,
                                                         const int64_t* __restrict__ f_ptr,
                                                         const int64_t* __restrict__ f_col,
                                                         const int64_t* __restrict__ t_ptr,
                                                         const int64_t* __restrict__ t_col, int64_t* greater,
                                                         int64_t* ties) {
  __shared__ int64_t sm[16];
  const int64_t i = blockIdx.x;
  const float t = clean(true_score[i]);
  const int64_t tj = true_idx[i] - c0;  // true column inside the chunk (if 0 <= tj < m)
  const float* row = s + i * lds;
  auto value = [&](int64_t j) -> float { return clean(j == tj ? t : row[j]); };

  int64_t gt = 0, eq = 0;
  for (int64_t j = threadIdx.x; j < m; j += NT) {
    const float v = value(j);
    gt += v > t;
    eq += v == t;
  }
  block_sum2(gt, eq, sm);
  if (threadIdx.x == 0) {
    greater[i] += gt;
    ties[i] += eq;
  }
  __syncthreads();

  const int nrank = t_ptr ? 2 : 1;
  int64_t dgt_f = 0, deq_f = 0;
  for (int r = 0; r < nrank; ++r) {
    const int64_t* ptr = r == 0 ? f_ptr : t_ptr;
    const int64_t* col = r == 0 ? f_col : t_col;
    int64_t dgt = 0, deq = 0;
    if (ptr) {
      const int64_t b = ptr[i], e = ptr[i + 1];
      for (int64_t x = b + threadIdx.x; x < e; x += NT) {
        const int64_t j = col[x] - c0;
        if (j < 0 || j >= m || j == tj) continue;
        const float v = value(j);
        dgt -= v > t;
        deq -= v == t;
        deq += (t == -INFINITY);  // the filtered entry is now -inf
      }
    }
    block_sum2(dgt, deq, sm);
    if (threadIdx.x == 0) {
      dgt_f += dgt;
      deq_f += deq;
      greater[(1 + r) * n + i] += gt + dgt_f;
      ties[(1 + r) * n + i] += eq + deq_f;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// Stacked ranking pass: rows [0, n_a) belong to query batch A (e.g. the (s, p, ?) queries of
// an evaluation batch), rows [n_a, n) to batch B (the (?, p, o) queries); each batch brings
// its own true column / true score / filter-list pointers, the list columns are shared.
// Optionally finishes the job in the same launch (rank per tie policy + histogram), and
// optionally REFINES scores that came from a reduced-precision contraction: an entry whose
// score lies within  band_i = band_rel * |q_i| * max_j |t_j|  of the true score is rescored
// as the correctly rounded fp32 value of the exact dot product of the fp32 query row and
// the fp32 candidate row (fp64 accumulation, fixed order) before it is compared.  Entries
// outside the band are on the same side of the true score as their exact value whenever the
// contraction's error is below the band, so the counts equal those of exact scoring.
struct RankPart {
  const int64_t* true_idx;
  const float* true_score;
  const int64_t* f_ptr;
  const int64_t* t_ptr;
};

struct RankRowsArgs {
  const float* s;
  const unsigned* codes;  // CODES kernels: the contraction's 2-bit codes instead of scores
  int64_t ldc;
  int codes_vec;  // code rows start on 16-byte boundaries: a row is read four words at a time
  int64_t lds, n_a, n, m, c0;
  RankPart part[2];
  const int64_t* f_col;
  const int64_t* t_col;
  int64_t* greater;
  int64_t* ties;
  int accumulate;
  int tie;  // < 0: counts only
  int64_t* ranks;
  float* hist;
  int64_t hist_len, rows_per_hist;
  const float* q;  // null: no refinement
  int64_t ldq;
  const float* t;  // row j of the chunk = t + j * ldt
  int64_t ldt;
  int d;
  float band_rel;
  const float* t_norm_max;
};

// Correctly rounded fp32 values of the exact dot products of the fp32 row a with up to U fp32
// rows b[u], computed by ONE WAVE in a fixed order per product (lane l accumulates the float4
// chunks l, l + 64, ... in fp64, then a butterfly sum): every lane returns the same values,
// and each value depends on (a, b[u], d) only -- not on U or on the other rows.  U products at
// a time keep U row loads in flight.
template <int U>
__device__ __forceinline__ void exact_dots_wave(const float* __restrict__ a, const float* const (&b)[U], int d,
                                                float (&out)[U]) {
  const int lane = threadIdx.x & 63;
  double acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = 0.0;
  for (int k = 4 * lane; k < d; k += 256) {
    const float4 x = *reinterpret_cast<const float4*>(a + k);
    float4 y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) y[u] = *reinterpret_cast<const float4*>(b[u] + k);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc[u] = fma((double)x.x, (double)y[u].x, acc[u]);
      acc[u] = fma((double)x.y, (double)y[u].y, acc[u]);
      acc[u] = fma((double)x.z, (double)y[u].z, acc[u]);
      acc[u] = fma((double)x.w, (double)y[u].w, acc[u]);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] += __shfl_xor(acc[u], off, 64);
#pragma unroll
  for (int u = 0; u < U; ++u) out[u] = (float)acc[u];
}

constexpr int EV_CAP = 8 * NT;  // near-tie ring: one scan step pushes at most 8 entries per thread

// The 2-bit code of column j in a row of code words written by the ranking contraction
// (kge_score_dot_split_rank): word (j / 64) * 4 + (j % 16) / 4, bit 8 * ((j % 64) / 16) + 2 * (j % 4).
__device__ __forceinline__ unsigned kge_rank_code_of(const unsigned* __restrict__ crow, int64_t j) {
  const unsigned w = crow[(j >> 6) * 4 + ((j & 15) >> 2)];
  return (w >> (8 * ((j & 63) >> 4) + 2 * (j & 3))) & 3u;
}

// CODES: the row comes as 2-bit codes (0 below / not a competitor, 1 above, 2 equal, 3 inside the
// refinement band) instead of scores; the band test has been made by the contraction's epilogue,
// the exact rescoring of the code-3 entries happens here (REFINE must be set when any can occur).
template <bool VEC, bool REFINE, bool CODES = false>
__global__ void __launch_bounds__(NT) rank_rows_kernel(const RankRowsArgs a) {
  __shared__ int64_t sm[16];
  __shared__ float fsm[NT / 64];
  __shared__ int ev[REFINE ? EV_CAP : 1];
  __shared__ unsigned ev_total;
  const int64_t i = blockIdx.x;
  const int side = i >= a.n_a;
  const int64_t li = side ? i - a.n_a : i;
  const RankPart& P = a.part[side];
  const float t = clean(P.true_score[li]);
  const int64_t tj = P.true_idx[li] - a.c0;
  const float* row = CODES ? nullptr : a.s + i * a.lds;
  const unsigned* crow = CODES ? a.codes + i * a.ldc : nullptr;
  const int64_t m = a.m;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;

  float band = -1.f;  // no score satisfies |v - t| <= band
  const float* qrow = nullptr;
  if (REFINE) {
    qrow = a.q + i * a.ldq;
    float ss = 0.f;
    if (!CODES) {  // the codes already say which entries lie inside the band
      for (int k = threadIdx.x; k < a.d; k += NT) ss += qrow[k] * qrow[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
      if (lane == 0) fsm[wave] = ss;
    }
    if (threadIdx.x == 0) ev_total = 0;
    __syncthreads();
    if (!CODES) {
      ss = 0.f;
      for (int w = 0; w < NT / 64; ++w) ss += fsm[w];
      band = a.band_rel * sqrtf(ss) * a.t_norm_max[0];
    }
  }

  // Counting one entry: the true column takes the true score; a score inside the band is
  // deferred to the ring (REFINE) and counted after it has been rescored.
  int64_t gt = 0, eq = 0;
  int pushed = 0;  // this thread deferred an entry since the last drain
  auto count = [&](int64_t j, float v, int sign) {
    if (j == tj) v = t;
    else if (REFINE && fabsf(v - t) <= band) {
      ev[atomicAdd(&ev_total, 1u) % EV_CAP] = (int)j;
      pushed = 1;
      return;
    }
    v = clean(v);
    gt += sign * (v > t);
    eq += sign * (v == t);
  };
  // the same for a column given by its code (never the true column: its code is 0)
  auto count_code = [&](int64_t j, unsigned code, int sign) {
    if (code == 3u) {
      if (REFINE) {
        ev[atomicAdd(&ev_total, 1u) % EV_CAP] = (int)j;
        pushed = 1;
      }
      return;
    }
    gt += sign * (int)(code == 1u);
    eq += sign * (int)(code == 2u);
  };
  // Rescore and count the entries pushed since `done` (block-uniform control flow): wave w
  // takes entries w, w + 4, ...; its lane 0 owns the counts.  Returns the new `done`.
  auto drain = [&](unsigned done, int sign) -> unsigned {
    // the barrier makes the pushes visible and tells every thread alike whether there are any
    // (ev_total itself may already be moving again when a slower thread would read it)
    const int any = __syncthreads_or(pushed);
    pushed = 0;
    if (!any) return done;
    const unsigned total = ev_total;  // stable: nobody pushes before the barrier below
    // wave w takes entries w, w + 4, ...: four at a time (four row loads in flight) while it has
    // at least two left -- a round's idle slots recompute its first entry (same cache lines) and
    // are not counted -- then a last single one
    constexpr int U = 4, NWV = NT / 64;
    unsigned x0 = done + wave;
    for (; x0 + NWV < total; x0 += U * NWV) {
      const float* rows_[U];
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const unsigned x = x0 + u * NWV < total ? x0 + u * NWV : x0;
        rows_[u] = a.t + (int64_t)ev[x % EV_CAP] * a.ldt;
      }
      exact_dots_wave<U>(qrow, rows_, a.d, v);
      if (lane == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (x0 + u * NWV >= total) continue;
          const float v_ = clean(v[u]);
          gt += sign * (v_ > t);
          eq += sign * (v_ == t);
        }
      }
    }
    for (; x0 < total; x0 += NWV) {
      const float* rows_[1] = {a.t + (int64_t)ev[x0 % EV_CAP] * a.ldt};
      float v[1];
      exact_dots_wave<1>(qrow, rows_, a.d, v);
      if (lane == 0) {
        const float v_ = clean(v[0]);
        gt += sign * (v_ > t);
        eq += sign * (v_ == t);
      }
    }
    __syncthreads();  // ring entries consumed before the next step overwrites them
    return total;
  };

  // The scan of the row.  step_drain: rescore the deferred entries after every step of 8 NT
  // columns (the ring holds one step's worth whatever the row looks like); otherwise they all
  // wait in the ring for ONE drain after the scan (all their row loads in flight together).
  auto scan = [&](bool step_drain) {
    unsigned done = 0;
    if (CODES) {
      // 16 codes per word; a step of NT / 2 words covers 8 NT columns (what the ring holds)
      const int64_t nwords = ((m + 63) >> 6) * 4;
      for (int64_t base = 0; base < nwords; base += NT / 2) {  // uniform trip count
        const int64_t wi = base + threadIdx.x;
        if (threadIdx.x < NT / 2 && wi < nwords) {
          const unsigned w = crow[wi];
          if (w) {
            const unsigned lo = w & 0x55555555u, hi = (w >> 1) & 0x55555555u;
            gt += __popc(lo & ~hi);
            eq += __popc(hi & ~lo);
            unsigned near = lo & hi;  // bit 2 p set: code 3 at position p of the word
            const int64_t jw = (wi >> 2) * 64 + (wi & 3) * 4;  // column of position (y = 0, r = 0)
            while (REFINE && near) {
              const int b = __ffs(near) - 1;
              near &= near - 1;
              count_code(jw + (b >> 3) * 16 + ((b >> 1) & 3), 3u, 1);
            }
          }
        }
        if (REFINE && step_drain) done = drain(done, 1);
      }
      if (threadIdx.x == 0 && tj >= 0 && tj < m) eq += 1;  // the true entry ties with itself
      return done;
    }
    if (VEC) {
      const int64_t m4 = m & ~(int64_t)3;
      for (int64_t base = 0; base < m4; base += 8 * NT) {  // uniform trip count
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int64_t j = base + 4 * (int64_t)(threadIdx.x + h * NT);
          if (j < m4) {
            const float4 v4 = *reinterpret_cast<const float4*>(row + j);
            count(j, v4.x, 1);
            count(j + 1, v4.y, 1);
            count(j + 2, v4.z, 1);
            count(j + 3, v4.w, 1);
          }
        }
        if (REFINE && step_drain) done = drain(done, 1);
      }
      if (m4 + threadIdx.x < m) count(m4 + threadIdx.x, row[m4 + threadIdx.x], 1);
      if (REFINE && step_drain) done = drain(done, 1);
    } else {
      for (int64_t base = 0; base < m; base += 8 * NT) {
#pragma unroll
        for (int h = 0; h < 8; ++h) {
          const int64_t j = base + threadIdx.x + h * NT;
          if (j < m) count(j, row[j], 1);
        }
        if (REFINE && step_drain) done = drain(done, 1);
      }
    }
    return done;
  };
  // CODES with 16-byte aligned rows.  The kernel is a chain of dependent loads (words of the row,
  // then per filter list: its bounds, its columns, their codes, then the rescored table rows), far
  // too short in bytes for bandwidth to matter: here every load that does not depend on a count is
  // requested before the first word is looked at -- the row four words per thread and round, the
  // first NT columns of each filter list and their codes -- which leaves three round trips.
  const int nfilt = P.t_ptr ? 2 : (P.f_ptr ? 1 : 0);
  const bool pre = CODES && a.codes_vec;
  int64_t fb[2] = {0, 0}, fe[2] = {0, 0}, fj[2] = {-1, -1};
  unsigned fcode[2] = {0u, 0u};
  auto scan_code_quads = [&]() {
    const int64_t nquads = (m + 63) >> 6;
    const uint4* c4 = reinterpret_cast<const uint4*>(crow);
    auto words = [&](int64_t qi, const uint4& w4) {
      const unsigned ws[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned w = ws[k];
        if (!w) continue;
        const unsigned lo = w & 0x55555555u, hi = (w >> 1) & 0x55555555u;
        gt += __popc(lo & ~hi);
        eq += __popc(hi & ~lo);
        unsigned near = lo & hi;
        const int64_t jw = qi * 64 + k * 4;
        while (REFINE && near) {
          const int b = __ffs(near) - 1;
          near &= near - 1;
          count_code(jw + (b >> 3) * 16 + ((b >> 1) & 3), 3u, 1);
        }
      }
    };
    uint4 w4 = make_uint4(0u, 0u, 0u, 0u);
    if (threadIdx.x < nquads) w4 = c4[threadIdx.x];
#pragma unroll
    for (int r = 0; r < 2; ++r) {  // (constant indexes: the arrays stay in registers)
      if (r >= nfilt) continue;
      const int64_t* ptr = r == 0 ? P.f_ptr : P.t_ptr;
      fb[r] = ptr[li];
      fe[r] = ptr[li + 1];
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (r >= nfilt) continue;
      const int64_t x = fb[r] + threadIdx.x;
      if (x < fe[r]) {
        const int64_t j = (r == 0 ? a.f_col : a.t_col)[x] - a.c0;
        if (j >= 0 && j < m && j != tj) {
          fj[r] = j;
          fcode[r] = kge_rank_code_of(crow, j);
        }
      }
    }
    words(threadIdx.x, w4);
    for (int64_t base = NT; base < nquads; base += 2 * NT) {  // uniform trip count
      const int64_t q0 = base + threadIdx.x, q1 = q0 + NT;
      uint4 u0 = make_uint4(0u, 0u, 0u, 0u), u1 = u0;
      if (q0 < nquads) u0 = c4[q0];
      if (q1 < nquads) u1 = c4[q1];
      words(q0, u0);
      words(q1, u1);
    }
    if (threadIdx.x == 0 && tj >= 0 && tj < m) eq += 1;  // the true entry ties with itself
  };
  unsigned done = 0;  // ring entries rescored so far
  if (REFINE) {
    // Rows with at most EV_CAP entries inside the band (all but degenerate ones: thousands of
    // candidates tied with the true score) are scanned without a barrier and drained once.  A
    // row with more has overwritten ring slots: its counts are discarded and the row is scanned
    // again, draining after every step.
    if (pre) scan_code_quads();
    else scan(false);
    __syncthreads();  // every push is visible; nobody pushes again before the next barrier
    const bool overflow = ev_total > (unsigned)EV_CAP;
    if (!overflow) {
      pushed = 1;
      done = drain(0, 1);
    } else {
      __syncthreads();  // ev_total has been read by every thread
      if (threadIdx.x == 0) ev_total = 0;
      gt = 0;
      eq = 0;
      pushed = 0;
      __syncthreads();
      done = scan(true);
    }
  } else if (pre) {
    scan_code_quads();
  } else {
    scan(false);
  }
  block_sum2(gt, eq, sm);
  auto emit = [&](int r, int64_t g, int64_t e) {  // thread 0 only
    const int64_t x = (int64_t)r * a.n + i;
    if (a.accumulate) {
      a.greater[x] += g;
      a.ties[x] += e;
    } else {
      a.greater[x] = g;
      a.ties[x] = e;
    }
    if (a.tie >= 0) {
      const int64_t rank = a.tie == KGE_TIE_ROUNDED_MEAN ? g + e / 2 : (a.tie == KGE_TIE_BEST ? g : g + e - 1);
      if (a.ranks) a.ranks[x] = rank;
      if (a.hist && rank >= 0 && rank < a.hist_len)
        atomicAdd(a.hist + (x / a.rows_per_hist) * a.hist_len + rank, 1.0f);
    }
  };
  int64_t g_run = 0, e_run = 0;  // thread 0: the running counts of the cumulative rankings
  if (threadIdx.x == 0) {
    g_run = gt;
    e_run = eq;
    emit(0, g_run, e_run);
  }
  __syncthreads();

  for (int r = 0; r < nfilt; ++r) {
    const int64_t* ptr = r == 0 ? P.f_ptr : P.t_ptr;
    const int64_t* col = r == 0 ? a.f_col : a.t_col;
    gt = 0;
    eq = 0;
    const int64_t pj = r == 0 ? fj[0] : fj[1];  // (selects, not indexed: registers)
    const unsigned pcode = r == 0 ? fcode[0] : fcode[1];
    const int64_t b = pre ? (r == 0 ? fb[0] : fb[1]) : ptr[li], e = pre ? (r == 0 ? fe[0] : fe[1]) : ptr[li + 1];
    for (int64_t x0 = b; x0 < e; x0 += NT) {  // uniform trip count
      const int64_t x = x0 + threadIdx.x;
      if (pre && x0 == b) {  // columns and codes are in registers already
        if (pj >= 0) {
          count_code(pj, pcode, -1);
          eq += (t == -INFINITY);
        }
      } else if (x < e) {
        const int64_t j = col[x] - a.c0;
        if (j >= 0 && j < m && j != tj) {
          if (CODES)
            count_code(j, kge_rank_code_of(crow, j), -1);
          else
            count(j, row[j], -1);
          eq += (t == -INFINITY);  // the filtered entry is now -inf
        }
      }
      if (REFINE) done = drain(done, -1);
    }
    block_sum2(gt, eq, sm);
    if (threadIdx.x == 0) {
      g_run += gt;
      e_run += eq;
      emit(1 + r, g_run, e_run);
    }
    __syncthreads();
  }
}

// out[0] = max over rows of the Euclidean row norm (out[0] must hold 0 on entry): a wave per
// row, 2 rows per wave, one atomic per workgroup (many short workgroups: a wave's loads are few
// and its reduction depends on all of them -- 43 us at 16 rows per wave for a 30-MB table).
// VEC (rows of a multiple of 4 floats, 16-B aligned): both rows of a wave are read together as
// float4s, all of their loads in flight before the first is used.
constexpr int NORM_ROWS = 8;
template <bool VEC>
__global__ void __launch_bounds__(256) row_norm_max_kernel(const float* __restrict__ t, int64_t ldt, int64_t m, int d,
                                                           float* out) {
  __shared__ float wmax[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float best = 0.f;
  auto take = [&](float ss) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
    ss = sqrtf(ss) * 1.000001f;
    best = (ss > best || ss != ss) ? ss : best;  // a NaN row poisons the maximum
  };
  if constexpr (VEC) {
    static_assert(NORM_ROWS == 8, "two rows per wave");
    const int64_t r0 = (int64_t)blockIdx.x * NORM_ROWS + wave * 2;
    if (r0 < m) {  // wave-uniform
      const int64_t r1 = r0 + 1 < m ? r0 + 1 : r0;  // a last odd row is read twice
      const float4* a = reinterpret_cast<const float4*>(t + r0 * ldt);
      const float4* b = reinterpret_cast<const float4*>(t + r1 * ldt);
      float sa = 0.f, sb = 0.f;
      const int d4 = d / 4;
      int k = lane;
      for (; k + 64 < d4; k += 128) {  // four loads in flight
        const float4 a0 = a[k], b0 = b[k], a1 = a[k + 64], b1 = b[k + 64];
        sa += a0.x * a0.x + a0.y * a0.y + a0.z * a0.z + a0.w * a0.w;
        sb += b0.x * b0.x + b0.y * b0.y + b0.z * b0.z + b0.w * b0.w;
        sa += a1.x * a1.x + a1.y * a1.y + a1.z * a1.z + a1.w * a1.w;
        sb += b1.x * b1.x + b1.y * b1.y + b1.z * b1.z + b1.w * b1.w;
      }
      if (k < d4) {
        const float4 a0 = a[k], b0 = b[k];
        sa += a0.x * a0.x + a0.y * a0.y + a0.z * a0.z + a0.w * a0.w;
        sb += b0.x * b0.x + b0.y * b0.y + b0.z * b0.z + b0.w * b0.w;
      }
      take(sa);
      take(sb);
    }
  } else {
    for (int i = 0; i < NORM_ROWS / 4; ++i) {
      const int64_t r = (int64_t)blockIdx.x * NORM_ROWS + wave * (NORM_ROWS / 4) + i;
      if (r >= m) break;  // wave-uniform
      float ss = 0.f;
      for (int k = lane; k < d; k += 64) {
        const float v = t[r * ldt + k];
        ss += v * v;
      }
      take(ss);
    }
  }
  if (lane == 0) wmax[wave] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) best = (wmax[w] > best || wmax[w] != wmax[w]) ? wmax[w] : best;
    // non-negative floats order like their bit patterns (NaN above every number).  The maximum only
    // grows, so a workgroup whose rows do not exceed the value it reads (possibly a stale, i.e.
    // lower, one) has nothing to add: all but a few skip the atomic, which the L2 would otherwise
    // serialise over a thousand workgroups on one address.
    unsigned* o = reinterpret_cast<unsigned*>(out);
    if (__float_as_uint(best) > __hip_atomic_load(o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(o, __float_as_uint(best));
  }
}

__global__ void zero1_kernel(float* out) { out[0] = 0.f; }

// row i counts into histogram i / rows_per_hist (hists of hist_len floats, back to back)
__global__ void rank_hist_kernel(const int64_t* __restrict__ greater, const int64_t* __restrict__ ties, int64_t n,
                                 int64_t rows_per_hist, int tie, int64_t* ranks, float* hist, int64_t hist_len) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t g = greater[i], t = ties[i];
  int64_t r = tie == KGE_TIE_ROUNDED_MEAN ? g + t / 2 : (tie == KGE_TIE_BEST ? g : g + t - 1);
  if (ranks) ranks[i] = r;
  if (hist && r >= 0 && r < hist_len) atomicAdd(hist + (i / rows_per_hist) * hist_len + r, 1.0f);
}

}  // namespace

extern "C" int kge_rank_counts(const float* s, int64_t lds, int64_t n, int64_t m, int64_t c0,
                               const int64_t* true_idx, const float* true_score, const int64_t* f_ptr,
                               const int64_t* f_col, const int64_t* t_ptr, const int64_t* t_col, int64_t* greater,
                               int64_t* ties, void* stream) {
  KGE_REQUIRE(n >= 0 && m >= 0 && (m == 0 || s) && true_idx && true_score && greater && ties && lds >= m);
  KGE_REQUIRE(!t_ptr || t_col);
  KGE_REQUIRE(!f_ptr || f_col);
  KGE_REQUIRE(n < (1LL << 31));
  if (n == 0) return 0;
  rank_counts_kernel<<<dim3((unsigned)n), dim3(NT), 0, as_stream(stream)>>>(
      s, lds, n, m, c0, true_idx, true_score, f_ptr, f_col, t_ptr, t_col, greater, ties);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_rank_hist(const int64_t* greater, const int64_t* ties, int64_t n, int tie_handling,
                             int64_t* ranks, float* hist, int64_t hist_len, void* stream) {
  return kge_rank_hist_multi(greater, ties, n, n > 0 ? n : 1, tie_handling, ranks, hist, hist_len, stream);
}

extern "C" int kge_rank_hist_multi(const int64_t* greater, const int64_t* ties, int64_t n, int64_t rows_per_hist,
                                   int tie_handling, int64_t* ranks, float* hist, int64_t hist_len, void* stream) {
  KGE_REQUIRE(n >= 0 && greater && ties && tie_handling >= 0 && tie_handling <= 2 && rows_per_hist > 0);
  if (n == 0) return 0;
  rank_hist_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream)>>>(
      greater, ties, n, rows_per_hist, tie_handling, ranks, hist, hist_len);
  KGE_CHECK_LAUNCH();
  return 0;
}

namespace {

// One workgroup per rank histogram: out[k] = (n, sum_j h[j] (j + 1), sum_j h[j] / (j + 1),
// hits@1 .. hits@kmax) with the operands of entity_ranking.py:553-577 -- fp32 counts, fp32 ranks,
// fp32 reciprocals, fp32 hits quotients -- and the two weighted sums accumulated in fp64 in a
// fixed order (thread-strided partial sums, then a tree over the 1,024 threads).
__global__ void __launch_bounds__(1024) rank_metrics_kernel(const float* __restrict__ hists, int64_t ld, int64_t e,
                                                            int kmax, double* __restrict__ out) {
  constexpr int NT = 1024, UNROLL = 8;
  __shared__ double red[3][NT];
  __shared__ float head[NT];  // the first NT counts, for the hits quotients
  const int tid = threadIdx.x;
  const float* h = hists + (int64_t)blockIdx.x * ld;
  double n = 0.0, s1 = 0.0, s2 = 0.0;
  head[tid] = 0.f;
  // few workgroups run (one per histogram), so nothing hides a load's latency but the loads of the
  // same thread: UNROLL of them are in flight at a time
  for (int64_t j0 = tid; j0 < e; j0 += (int64_t)NT * UNROLL) {
    float c[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t j = j0 + (int64_t)u * NT;
      c[u] = j < e ? h[j] : 0.f;
    }
    if (j0 == tid) head[tid] = c[0];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const float rank = (float)(j0 + (int64_t)u * NT + 1);
      const double cd = (double)c[u];
      n += cd;
      s1 += cd * (double)rank;
      s2 += cd * (double)(1.0f / rank);
    }
  }
  red[0][tid] = n, red[1][tid] = s1, red[2][tid] = s2;
  __syncthreads();
  for (int off = NT / 2; off > 0; off >>= 1) {
    if (tid < off) {
#pragma unroll
      for (int q = 0; q < 3; ++q) red[q][tid] += red[q][tid + off];
    }
    __syncthreads();
  }
  double* o = out + (int64_t)blockIdx.x * (3 + kmax);
  if (tid < 3) o[tid] = red[tid][0];
  // hits@(tid + 1): the cumulative counts of the first ranks in fp32, as torch.cumsum forms them
  // -- a prefix scan: the counts are integers, so below 2^24 evaluation triples every partial sum
  // is exact whatever the order of the additions
  for (int off = 1; off < NT; off <<= 1) {
    const float v = tid >= off ? head[tid - off] : 0.f;
    __syncthreads();
    head[tid] += v;
    __syncthreads();
  }
  if (tid < kmax) {
    const float nf = (float)red[0][0];
    o[3 + tid] = nf > 0.f ? (double)(head[tid] / nf) : 0.0;
  }
}

}  // namespace

extern "C" int kge_rank_metrics(const float* hists, int64_t ld, int64_t k, int64_t e, int kmax, double* out,
                                void* stream) {
  KGE_REQUIRE(k >= 0 && e > 0 && kmax >= 0 && ld >= e && (hists || k == 0) && (out || k == 0));
  if (k == 0) return 0;
  KGE_REQUIRE(k < (1LL << 31));
  KGE_REQUIRE(kmax <= 1024);
  rank_metrics_kernel<<<dim3((unsigned)k), dim3(1024), 0, as_stream(stream)>>>(hists, ld, e, kmax, out);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_row_norm_max(const float* t, int64_t ldt, int64_t m, int d, float* out, void* stream) {
  KGE_REQUIRE(m >= 0 && d > 0 && (t || m == 0) && out && ldt >= d);
  hipStream_t st = as_stream(stream);
  zero1_kernel<<<dim3(1), dim3(1), 0, st>>>(out);
  if (m > 0) {
    const dim3 grid((unsigned)((m + NORM_ROWS - 1) / NORM_ROWS));
    if (d % 4 == 0 && ldt % 4 == 0 && aligned16(t))
      row_norm_max_kernel<true><<<grid, dim3(256), 0, st>>>(t, ldt, m, d, out);
    else
      row_norm_max_kernel<false><<<grid, dim3(256), 0, st>>>(t, ldt, m, d, out);
  }
  KGE_CHECK_LAUNCH();
  return 0;
}

namespace {

// band[i] = band_rel * |q_i|_2 * t_norm_max[0]: the refinement band of row i, as rank_rows_kernel
// computes it for itself; a wave per row
__global__ void __launch_bounds__(256) rank_band_kernel(const float* __restrict__ q, int64_t ldq, int64_t n, int d,
                                                        float band_rel, const float* __restrict__ t_norm_max,
                                                        float* __restrict__ band) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;  // wave-uniform
  float ss = 0.f;
  for (int k = lane; k < d; k += 64) {
    const float v = q[i * ldq + k];
    ss += v * v;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
  // a hair wider than the kernel's own band (summation order): never narrower than the bound
  if (lane == 0) band[i] = band_rel * sqrtf(ss) * t_norm_max[0] * 1.000001f;
}

int rank_rows_launch(RankRowsArgs& a, bool codes, hipStream_t st) {
  const bool vec = !codes && a.lds % 4 == 0 && aligned16(a.s);
  const unsigned n = (unsigned)a.n;
  if (codes && a.q)
    rank_rows_kernel<false, true, true><<<dim3(n), dim3(NT), 0, st>>>(a);
  else if (codes)
    rank_rows_kernel<false, false, true><<<dim3(n), dim3(NT), 0, st>>>(a);
  else if (a.q && vec)
    rank_rows_kernel<true, true><<<dim3(n), dim3(NT), 0, st>>>(a);
  else if (a.q)
    rank_rows_kernel<false, true><<<dim3(n), dim3(NT), 0, st>>>(a);
  else if (vec)
    rank_rows_kernel<true, false><<<dim3(n), dim3(NT), 0, st>>>(a);
  else
    rank_rows_kernel<false, false><<<dim3(n), dim3(NT), 0, st>>>(a);
  KGE_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int kge_rank_band(const float* q, int64_t ldq, int64_t n, int d, float band_rel, const float* t_norm_max,
                             float* band, void* stream) {
  KGE_REQUIRE(n >= 0 && d > 0 && (q || n == 0) && ldq >= d && band_rel >= 0.f && t_norm_max && band && n < (1LL << 31));
  if (n == 0) return 0;
  rank_band_kernel<<<dim3((unsigned)((n + 3) / 4)), dim3(256), 0, as_stream(stream)>>>(q, ldq, n, d, band_rel,
                                                                                       t_norm_max, band);
  KGE_CHECK_LAUNCH();
  return 0;
}

static int rank_rows_common(const float* s, int64_t lds, const unsigned* codes, int64_t ldc, int64_t n_a, int64_t n_b,
                            int64_t m, int64_t c0, const int64_t* true_idx_a, const float* true_score_a,
                            const int64_t* f_ptr_a, const int64_t* t_ptr_a, const int64_t* true_idx_b,
                            const float* true_score_b, const int64_t* f_ptr_b, const int64_t* t_ptr_b,
                            const int64_t* f_col, const int64_t* t_col, int64_t* greater, int64_t* ties,
                            int accumulate, int tie_handling, int64_t* ranks, float* hist, int64_t hist_len,
                            int64_t rows_per_hist, const float* q, int64_t ldq, const float* t, int64_t ldt, int d,
                            float band_rel, const float* t_norm_max, void* stream) {
  const int64_t n = n_a + n_b;
  KGE_REQUIRE(n_a >= 0 && n_b >= 0 && m >= 0 && m < (1LL << 31) && greater && ties && n < (1LL << 31));
  KGE_REQUIRE(codes ? ldc >= ((m + 63) / 64) * 4 : ((m == 0 || s) && lds >= m));
  KGE_REQUIRE(n_a == 0 || (true_idx_a && true_score_a));
  KGE_REQUIRE(n_b == 0 || (true_idx_b && true_score_b));
  KGE_REQUIRE((!f_ptr_a && !f_ptr_b) || f_col);
  KGE_REQUIRE((!t_ptr_a && !t_ptr_b) || t_col);
  // the rankings of both batches share one counts layout: filter lists come for both or neither
  KGE_REQUIRE(n_a == 0 || n_b == 0 || ((!f_ptr_a == !f_ptr_b) && (!t_ptr_a == !t_ptr_b)));
  KGE_REQUIRE(!(t_ptr_a && !f_ptr_a) && !(t_ptr_b && !f_ptr_b));
  KGE_REQUIRE(tie_handling <= 2 && (tie_handling < 0 || !hist || (hist_len > 0 && rows_per_hist > 0)));
  KGE_REQUIRE(tie_handling < 0 || !accumulate);  // ranks need the counts of every chunk
  if (q) {
    KGE_REQUIRE(t && t_norm_max && d > 0 && ldq >= d && ldt >= d && band_rel >= 0.f);
    if (d % 4 != 0 || ldq % 4 != 0 || ldt % 4 != 0 || !aligned16(q) || !aligned16(t)) return KGE_ERR_ALIGN;
  }
  if (n == 0) return 0;
  RankRowsArgs a;
  a.codes_vec = codes && ldc % 4 == 0 && aligned16(codes);
  a.s = s; a.codes = codes; a.ldc = ldc; a.lds = lds; a.n_a = n_a; a.n = n; a.m = m; a.c0 = c0;
  a.part[0] = RankPart{true_idx_a, true_score_a, f_ptr_a, t_ptr_a};
  a.part[1] = RankPart{true_idx_b, true_score_b, f_ptr_b, t_ptr_b};
  a.f_col = f_col; a.t_col = t_col; a.greater = greater; a.ties = ties; a.accumulate = accumulate;
  a.tie = tie_handling; a.ranks = ranks; a.hist = hist; a.hist_len = hist_len; a.rows_per_hist = rows_per_hist;
  a.q = q; a.ldq = ldq; a.t = t; a.ldt = ldt; a.d = d; a.band_rel = band_rel; a.t_norm_max = t_norm_max;
  return rank_rows_launch(a, codes != nullptr, as_stream(stream));
}

extern "C" int kge_rank_rows(const float* s, int64_t lds, int64_t n_a, int64_t n_b, int64_t m, int64_t c0,
                             const int64_t* true_idx_a, const float* true_score_a, const int64_t* f_ptr_a,
                             const int64_t* t_ptr_a, const int64_t* true_idx_b, const float* true_score_b,
                             const int64_t* f_ptr_b, const int64_t* t_ptr_b, const int64_t* f_col,
                             const int64_t* t_col, int64_t* greater, int64_t* ties, int accumulate, int tie_handling,
                             int64_t* ranks, float* hist, int64_t hist_len, int64_t rows_per_hist, const float* q,
                             int64_t ldq, const float* t, int64_t ldt, int d, float band_rel, const float* t_norm_max,
                             void* stream) {
  return rank_rows_common(s, lds, nullptr, 0, n_a, n_b, m, c0, true_idx_a, true_score_a, f_ptr_a, t_ptr_a, true_idx_b,
                          true_score_b, f_ptr_b, t_ptr_b, f_col, t_col, greater, ties, accumulate, tie_handling, ranks,
                          hist, hist_len, rows_per_hist, q, ldq, t, ldt, d, band_rel, t_norm_max, stream);
}

extern "C" int kge_rank_rows_codes(const void* codes, int64_t ldc, int64_t n_a, int64_t n_b, int64_t m, int64_t c0,
                                   const int64_t* true_idx_a, const float* true_score_a, const int64_t* f_ptr_a,
                                   const int64_t* t_ptr_a, const int64_t* true_idx_b, const float* true_score_b,
                                   const int64_t* f_ptr_b, const int64_t* t_ptr_b, const int64_t* f_col,
                                   const int64_t* t_col, int64_t* greater, int64_t* ties, int accumulate,
                                   int tie_handling, int64_t* ranks, float* hist, int64_t hist_len,
                                   int64_t rows_per_hist, const float* q, int64_t ldq, const float* t, int64_t ldt,
                                   int d, float band_rel, const float* t_norm_max, void* stream) {
  KGE_REQUIRE(codes || m == 0);
  return rank_rows_common(nullptr, 0, (const unsigned*)codes, ldc, n_a, n_b, m, c0, true_idx_a, true_score_a, f_ptr_a,
                          t_ptr_a, true_idx_b, true_score_b, f_ptr_b, t_ptr_b, f_col, t_col, greater, ties, accumulate,
                          tie_handling, ranks, hist, hist_len, rows_per_hist, q, ldq, t, ldt, d, band_rel, t_norm_max,
                          stream);
}

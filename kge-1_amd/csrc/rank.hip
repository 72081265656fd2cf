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

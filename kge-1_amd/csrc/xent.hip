// Softmax cross entropy over all-entity score rows, fused with its gradient (the loss the
// 1vsAll job puts on score_sp / score_po: KLDivWithSoftmaxKgeLoss with index labels ==
// torch.nn.CrossEntropyLoss(reduction="sum"), reference kge/util/loss.py:192-208, divided
// by the batch size in kge/job/train.py:1042,1052).
//
//   loss[i] = logsumexp_j S[i, j] - S[i, label_i]
//   G[i, j] = scale * (softmax_j(S[i, :]) - [j == label_i])      (optional, may alias S)
//
// HBM-bound: one workgroup per row reads the row once for an online (max, sum-exp), then
// reads it again (L2 / MALL-resident: a row is 4m bytes and was just touched) to write G.
// 8 bytes per element (read + write) + one re-read that should not reach HBM.
#include <math.h>

#include "common.h"

namespace {

constexpr int NT = 256, U = 8;

__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mm = fmaxf(m, m2);
  if (mm == -INFINITY) return;  // both empty so far
  s = s * expf(m - mm) + s2 * expf(m2 - mm);
  m = mm;
}

template <bool VEC>
__global__ void __launch_bounds__(NT) xent_kernel(const float* s, int64_t lds, int m,
                                                  const int64_t* __restrict__ labels, float scale,
                                                  float* __restrict__ loss, float* g, int64_t ldg) {
  __shared__ float red_m[NT / 64], red_s[NT / 64];
  const int64_t row = blockIdx.x;
  const float* sr = s + row * lds;
  const int tid = threadIdx.x;
  const int64_t lab = labels[row];
  const bool lab_ok = lab >= 0 && lab < m;
  // S[i, label] is read before any thread can overwrite the row (g may alias s)
  const float s_lab = (tid == 0 && lab_ok) ? sr[lab] : 0.f;

  // pass 1: per-thread online (max, sum exp(x - max)); NaN propagates through the sum
  float mx = -INFINITY, sm = 0.f;
  auto take = [&](float v) {
    if (v > mx) {
      sm = sm * expf(mx - v) + 1.f;
      mx = v;
    } else if (v != -INFINITY) {  // -inf adds 0 (and would be NaN while mx is -inf)
      sm += expf(v - mx);
    }
  };
  int j0 = 0;
  if (VEC) {
    // U float4 loads in flight per thread before any of them is consumed (the running
    // (max, sum) is a dependency chain: one load per iteration would be latency-bound)
    const int m4 = m & ~3;
    for (int base = 0; base < m4; base += NT * 4 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const float4*>(sr + min(base + (u * NT + tid) * 4, m4 - 4));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (base + (u * NT + tid) * 4 >= m4) v[u] = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
        const float vm = fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w));
        const float nm = fmaxf(mx, vm);
        if (nm != -INFINITY) {
          sm = sm * expf(mx - nm) + expf(v[u].x - nm) + expf(v[u].y - nm) + expf(v[u].z - nm) + expf(v[u].w - nm);
          mx = nm;
        } else if (v[u].x != v[u].x || v[u].y != v[u].y || v[u].z != v[u].z || v[u].w != v[u].w) {
          sm = NAN;
        }
      }
    }
    j0 = m4;
  }
  for (int j = j0 + tid; j < m; j += NT) take(sr[j]);
  // NaN anywhere in the row: fmaxf drops NaN from the max but expf(NaN) poisons the sum
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(mx, off, 64), s2 = __shfl_xor(sm, off, 64);
    lse_merge(mx, sm, m2, s2);
  }
  if ((tid & 63) == 0) {
    red_m[tid >> 6] = mx;
    red_s[tid >> 6] = sm;
  }
  __syncthreads();
  mx = red_m[0];
  sm = red_s[0];
#pragma unroll
  for (int w = 1; w < NT / 64; ++w) lse_merge(mx, sm, red_m[w], red_s[w]);
  const float lse = mx + logf(sm);
  if (tid == 0) loss[row] = lab_ok ? lse - s_lab : NAN;
  if (!g) return;

  // pass 2: G = scale * (exp(x - lse) - onehot)
  float* gr = g + row * ldg;
  if (VEC) {
    const int m4 = m & ~3;
    for (int base = 0; base < m4; base += NT * 4 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const float4*>(sr + min(base + (u * NT + tid) * 4, m4 - 4));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = base + (u * NT + tid) * 4;
        if (j < m4)
          *reinterpret_cast<float4*>(gr + j) = make_float4(scale * expf(v[u].x - lse), scale * expf(v[u].y - lse),
                                                           scale * expf(v[u].z - lse), scale * expf(v[u].w - lse));
      }
    }
  }
  for (int j = j0 + tid; j < m; j += NT) gr[j] = scale * expf(sr[j] - lse);
  __syncthreads();  // every write of the row is ordered before the label fix-up
  if (tid == 0 && lab_ok) gr[lab] = scale * (expf(s_lab - lse) - 1.f);
}

}  // namespace

extern "C" int kge_softmax_xent(const float* s, int64_t lds, int64_t n, int64_t m, const int64_t* labels,
                                float scale, float* loss, float* g, int64_t ldg, void* stream) {
  KGE_REQUIRE(n >= 0 && m > 0 && m < (1LL << 31) && n < (1LL << 31));
  KGE_REQUIRE(s && labels && loss && lds >= m && (!g || ldg >= m));
  KGE_REQUIRE(!g || g != s || ldg == lds);  // in place only row-for-row
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  const bool vec = lds % 4 == 0 && aligned16(s) && (!g || (ldg % 4 == 0 && aligned16(g)));
  if (vec)
    xent_kernel<true><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)m, labels, scale, loss, g, ldg);
  else
    xent_kernel<false><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)m, labels, scale, loss, g, ldg);
  KGE_CHECK_LAUNCH();
  return 0;
}

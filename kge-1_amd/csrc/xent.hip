// Softmax losses over all-entity score rows, fused with their gradient.
//
// KL(t_i || softmax(S_i)) for a target row t_i built from a list of positive columns P_i
// (unique) and label smoothing eps, exactly as the reference builds it:
//   labels = (1 - eps) * y + 1/m      (train.py:715-721, only when eps > 0)
//   t      = labels / max(|labels|_1, 1e-12)                            (loss.py:211-213)
// so t0 = (eps > 0 ? 1/m : 0) / Z off P_i, t1 = ((1 - eps) + (eps > 0 ? 1/m : 0)) / Z on
// P_i, Z = (1 - eps)|P_i| + (eps > 0 ? 1 : 0).  With T = sum_j t_j (1, or 0 for an empty
// row without smoothing):
//   loss_i = sum_j t_j log t_j - sum_j t_j S_ij + T lse_i
//          = H(t) - t0 rowsum_i - (t1 - t0) sum_{P_i} S_ij + T lse_i
//   G_ij   = scale * (T softmax_ij - t_ij)
// Index labels (1vsAll, KLDivWithSoftmaxKgeLoss -> CrossEntropyLoss, loss.py:198-208) are
// the case |P_i| = 1, eps = 0: loss_i = lse_i - S_i,label, G = scale (softmax - onehot).
//
// Column-sharded rows (vocab-parallel 1vsAll over the row-sharded entity table):
// kge_softmax_row_stats gives each shard's (max, sum exp(x - max), target score) for the
// cross-shard reduction, kge_softmax_grad the shard's slice of G from the global lse.
//
// HBM-bound: one workgroup per row reads the row once for the online (max, sum-exp, sum)
// and writes G, which may alias S, from registers (rows up to 16,384 columns); longer rows
// are read a second time (L2 / MALL-resident: 4m bytes just touched) to write G.
// exp is v_exp_f32 (__expf): relative error ~|x| * 6e-8 for exp(x), x = score - max <= 0,
// far inside the 1e-4 contract; libm expf made the kernel VALU-bound.
#include <math.h>

#include "common.h"

namespace {

constexpr int NT = 256, U = 8;

__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mm = fmaxf(m, m2);
  if (mm == -INFINITY) return;  // both empty so far
  s = s * __expf(m - mm) + s2 * __expf(m2 - mm);
  m = mm;
}

__device__ __forceinline__ float xlogx(float x) { return x > 0.f ? x * logf(x) : 0.f; }

// Block-wide online (max, sum exp(x - max), sum x) of row sr[0, m); every thread returns
// the block totals.  red: 3 x (NT / 64) floats of LDS.
template <bool VEC>
__device__ __forceinline__ void row_stats(const float* sr, int m, float (&red)[3][NT / 64], float& mx, float& sm,
                                          float& rs) {
  const int tid = threadIdx.x;
  mx = -INFINITY;
  sm = 0.f;
  rs = 0.f;
  int j0 = 0;
  if (VEC) {
    // U float4 loads in flight per thread before any is consumed: the running (max, sum)
    // is a dependency chain, one load per iteration would be latency-bound
    const int m4 = m & ~3;
    for (int base = 0; base < m4; base += NT * 4 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const float4*>(sr + min(base + (u * NT + tid) * 4, m4 - 4));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (base + (u * NT + tid) * 4 >= m4) continue;
        rs += (v[u].x + v[u].y) + (v[u].z + v[u].w);
        const float vm = fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w));
        const float nm = fmaxf(mx, vm);
        if (nm != -INFINITY) {
          sm = sm * __expf(mx - nm) + __expf(v[u].x - nm) + __expf(v[u].y - nm) + __expf(v[u].z - nm) +
               __expf(v[u].w - nm);
          mx = nm;
        } else if (v[u].x != v[u].x || v[u].y != v[u].y || v[u].z != v[u].z || v[u].w != v[u].w) {
          sm = NAN;
        }
      }
    }
    j0 = m4;
  }
  for (int j = j0 + tid; j < m; j += NT) {
    const float v = sr[j];
    rs += v;
    if (v > mx) {
      sm = sm * __expf(mx - v) + 1.f;
      mx = v;
    } else if (v != -INFINITY) {  // -inf adds 0 (and would be NaN while mx is -inf)
      sm += __expf(v - mx);
    }
  }
  // NaN anywhere in the row: fmaxf drops NaN from the max but exp(NaN) poisons the sum
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(mx, off, 64), s2 = __shfl_xor(sm, off, 64);
    lse_merge(mx, sm, m2, s2);
    rs += __shfl_xor(rs, off, 64);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = mx;
    red[1][tid >> 6] = sm;
    red[2][tid >> 6] = rs;
  }
  __syncthreads();
  mx = red[0][0];
  sm = red[1][0];
  rs = red[2][0];
#pragma unroll
  for (int w = 1; w < NT / 64; ++w) {
    lse_merge(mx, sm, red[0][w], red[1][w]);
    rs += red[2][w];
  }
  __syncthreads();  // red is reused by the caller
}

// gr[j] = a * exp(sr[j] - lse) - b for j in [0, m); gr may alias sr (read before write per element)
template <bool VEC>
__device__ __forceinline__ void row_grad(const float* sr, float* gr, int m, float lse, float a, float b) {
  const int tid = threadIdx.x;
  int j0 = 0;
  if (VEC) {
    const int m4 = m & ~3;
    for (int base = 0; base < m4; base += NT * 4 * U) {
      float4 v[U];
#pragma unroll
      for (int q = 0; q < U; ++q) v[q] = *reinterpret_cast<const float4*>(sr + min(base + (q * NT + tid) * 4, m4 - 4));
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int j = base + (q * NT + tid) * 4;
        if (j < m4)
          *reinterpret_cast<float4*>(gr + j) =
              make_float4(a * __expf(v[q].x - lse) - b, a * __expf(v[q].y - lse) - b, a * __expf(v[q].z - lse) - b,
                          a * __expf(v[q].w - lse) - b);
      }
    }
    j0 = m4;
  }
  for (int j = j0 + tid; j < m; j += NT) gr[j] = a * __expf(sr[j] - lse) - b;
}


// Rows of at most NI * NT * 4 * U floats (16,384 for NI = 2: every FB15K-237 / WN18RR-sized
// row): the row is loaded ONCE into registers (NI * U float4 per thread, all loads in flight
// together), the statistics come from the registers and G is written from them -- one HBM
// read and one write per element instead of a second (L2 / MALL) read pass.  Same
// per-thread element order and arithmetic as row_stats / row_grad.
template <int NI>
struct RowRegs {
  float4 v[NI][U];
};

template <int NI, int NTH = NT>
__device__ __forceinline__ void row_load_regs(const float* sr, int m, RowRegs<NI>& r) {
  const int tid = threadIdx.x, m4 = m & ~3;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int u = 0; u < U; ++u)
      r.v[i][u] = *reinterpret_cast<const float4*>(sr + min(i * NTH * 4 * U + (u * NTH + tid) * 4, m4 - 4));
}

template <int NI, int NTH = NT>
__device__ __forceinline__ void row_stats_regs(const float* sr, int m, const RowRegs<NI>& r, float (&red)[3][NTH / 64],
                                               float& mx, float& sm, float& rs) {
  const int tid = threadIdx.x, m4 = m & ~3;
  mx = -INFINITY;
  sm = 0.f;
  rs = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float4 v = r.v[i][u];
      if (i * NTH * 4 * U + (u * NTH + tid) * 4 >= m4) continue;
      rs += (v.x + v.y) + (v.z + v.w);
      const float vm = fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w));
      const float nm = fmaxf(mx, vm);
      if (nm != -INFINITY) {
        sm = sm * __expf(mx - nm) + __expf(v.x - nm) + __expf(v.y - nm) + __expf(v.z - nm) + __expf(v.w - nm);
        mx = nm;
      } else if (v.x != v.x || v.y != v.y || v.z != v.z || v.w != v.w) {
        sm = NAN;
      }
    }
  for (int j = m4 + tid; j < m; j += NTH) {
    const float v = sr[j];
    rs += v;
    if (v > mx) {
      sm = sm * __expf(mx - v) + 1.f;
      mx = v;
    } else if (v != -INFINITY) {
      sm += __expf(v - mx);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(mx, off, 64), s2 = __shfl_xor(sm, off, 64);
    lse_merge(mx, sm, m2, s2);
    rs += __shfl_xor(rs, off, 64);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = mx;
    red[1][tid >> 6] = sm;
    red[2][tid >> 6] = rs;
  }
  __syncthreads();
  mx = red[0][0];
  sm = red[1][0];
  rs = red[2][0];
#pragma unroll
  for (int w = 1; w < NTH / 64; ++w) {
    lse_merge(mx, sm, red[0][w], red[1][w]);
    rs += red[2][w];
  }
  __syncthreads();
}

template <int NI, int NTH = NT>
__device__ __forceinline__ void row_grad_regs(const float* sr, float* gr, int m, const RowRegs<NI>& r, float lse,
                                              float a, float b) {
  const int tid = threadIdx.x, m4 = m & ~3;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = i * NTH * 4 * U + (u * NTH + tid) * 4;
      const float4 v = r.v[i][u];
      if (j < m4)
        *reinterpret_cast<float4*>(gr + j) = make_float4(a * __expf(v.x - lse) - b, a * __expf(v.y - lse) - b,
                                                         a * __expf(v.z - lse) - b, a * __expf(v.w - lse) - b);
    }
  for (int j = m4 + tid; j < m; j += NTH) gr[j] = a * __expf(sr[j] - lse) - b;
}

template <int NTH = NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  float t = red[0];
#pragma unroll
  for (int w = 1; w < NTH / 64; ++w) t += red[w];
  __syncthreads();
  return t;
}

// l_ptr == NULL: index labels, P_i = {l_col[i]}
template <bool VEC, int NI = 0>
__global__ void __launch_bounds__(NT) softmax_kl_kernel(const float* s, int64_t lds, int m,
                                                        const int64_t* __restrict__ l_ptr,
                                                        const int64_t* __restrict__ l_col, float eps, float scale,
                                                        float* __restrict__ loss, float* g, int64_t ldg) {
  __shared__ float red[3][NT / 64];
  const int64_t row = blockIdx.x;
  const float* sr = s + row * lds;
  const int tid = threadIdx.x;
  const int64_t p0 = l_ptr ? l_ptr[row] : row, p1 = l_ptr ? l_ptr[row + 1] : row + 1;

  // positives' scores and the row statistics are read before the first barrier inside
  // row_stats, i.e. before any thread overwrites the row (g may alias s)
  float ps = 0.f;
  for (int64_t k = p0 + tid; k < p1; k += NT) {
    const int64_t c = l_col[k];
    ps += (c >= 0 && c < m) ? sr[c] : NAN;  // a label outside the row poisons the loss
  }
  float mx, sm, rs;
  RowRegs<NI ? NI : 1> regs;
  if constexpr (NI > 0) {
    row_load_regs<NI>(sr, m, regs);
    row_stats_regs<NI>(sr, m, regs, red, mx, sm, rs);
  } else {
    row_stats<VEC>(sr, m, red, mx, sm, rs);
  }
  ps = block_sum(ps, red[0]);

  const float lse = mx + __logf(sm);
  const int64_t np = p1 - p0;
  const float u = eps > 0.f ? 1.f / (float)m : 0.f;
  const float z = (1.f - eps) * (float)np + (eps > 0.f ? 1.f : 0.f);
  const float zi = z > 1e-12f ? 1.f / z : 0.f;  // F.normalize: x / max(|x|_1, 1e-12)
  const float t0 = u * zi, t1 = ((1.f - eps) + u) * zi;
  const float T = z > 0.f ? 1.f : 0.f;
  if (tid == 0) {
    if (!l_ptr) {  // index label: exactly lse - S[label] (no 0 * inf from the general form)
      loss[row] = lse - ps;
    } else {
      const float H = (float)(m - np) * xlogx(t0) + (float)np * xlogx(t1);
      loss[row] = H - t0 * rs - (t1 - t0) * ps + (T > 0.f ? lse : 0.f);
    }
  }
  if (!g) return;

  // pass 2: G = scale * (T softmax - t0), then positives -= scale * (t1 - t0)
  float* gr = g + row * ldg;
  if constexpr (NI > 0)
    row_grad_regs<NI>(sr, gr, m, regs, lse, scale * T, scale * t0);
  else
    row_grad<VEC>(sr, gr, m, lse, scale * T, scale * t0);
  __syncthreads();  // every write of the row is ordered before the positives' fix-up
  const float d = scale * (t1 - t0);
  for (int64_t k = p0 + tid; k < p1; k += NT) {
    const int64_t c = l_col[k];
    if (c >= 0 && c < m) gr[c] -= d;
  }
}

// column slice [c0, c0 + m) of rows whose labels are global column ids
template <bool VEC>
__global__ void __launch_bounds__(NT) row_stats_kernel(const float* __restrict__ s, int64_t lds, int m, int64_t c0,
                                                       const int64_t* __restrict__ labels, float* __restrict__ mx_out,
                                                       float* __restrict__ sm_out, float* __restrict__ tg_out) {
  __shared__ float red[3][NT / 64];
  const int64_t row = blockIdx.x;
  const float* sr = s + row * lds;
  float mx, sm, rs;
  row_stats<VEC>(sr, m, red, mx, sm, rs);
  if (threadIdx.x == 0) {
    mx_out[row] = mx;
    sm_out[row] = sm;
    if (tg_out) {
      const int64_t c = labels[row] - c0;
      tg_out[row] = (c >= 0 && c < m) ? sr[c] : 0.f;  // the owner contributes, others 0
    }
  }
}

template <bool VEC>
__global__ void __launch_bounds__(NT) grad_kernel(const float* s, int64_t lds, int m, int64_t c0,
                                                  const int64_t* __restrict__ labels, const float* __restrict__ lse,
                                                  float scale, float* g, int64_t ldg) {
  const int64_t row = blockIdx.x;
  const float* sr = s + row * lds;
  float* gr = g + row * ldg;
  row_grad<VEC>(sr, gr, m, lse[row], scale, 0.f);
  __syncthreads();
  if (threadIdx.x == 0 && labels) {
    const int64_t c = labels[row] - c0;
    if (c >= 0 && c < m) gr[c] -= scale;
  }
}

bool vec_ok(const float* s, int64_t lds, const float* g, int64_t ldg) {
  return lds % 4 == 0 && aligned16(s) && (!g || (ldg % 4 == 0 && aligned16(g)));
}

int launch(const float* s, int64_t lds, int64_t n, int64_t m, const int64_t* l_ptr, const int64_t* l_col, float eps,
           float scale, float* loss, float* g, int64_t ldg, hipStream_t st) {
  const int64_t m4 = m & ~3LL, chunk = (int64_t)NT * 4 * U;
  const bool vec = vec_ok(s, lds, g, ldg);
  if (vec && m4 >= 4 && m4 <= chunk)
    softmax_kl_kernel<true, 1><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)m, l_ptr, l_col, eps, scale,
                                                                       loss, g, ldg);
  else if (vec && m4 > chunk && m4 <= 2 * chunk)
    softmax_kl_kernel<true, 2><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)m, l_ptr, l_col, eps, scale,
                                                                       loss, g, ldg);
  else if (vec)
    softmax_kl_kernel<true><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)m, l_ptr, l_col, eps, scale, loss,
                                                                    g, ldg);
  else
    softmax_kl_kernel<false><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)m, l_ptr, l_col, eps, scale, loss,
                                                                     g, ldg);
  KGE_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// The same losses with G written as bf16 hi / lo planes IN PLACE of the score row, for the
// plane-fed backward GEMMs (gemm_bwd3p.hip): row i of the buffer (lds floats = 4 lds bytes)
// ends up holding the hi plane of G[i, :] in its first lds bf16 and the lo plane in its
// second lds bf16 (G ~= hi + lo to 2^-16, the split the GEMMs would otherwise do per tile).
// Columns [m, lds) of both planes and the rows [n, n_pad) are zeroed: the GEMMs read them as
// K padding.  The row is held in registers (one read, one write per element); rows up to
// NI * NTH * 4 * U floats.  Positives are fixed up from the planes themselves: hi + lo
// reproduces the value to 2^-16 relative, far below the 2^-16 of the products it feeds.
typedef __bf16 kge_bf16_t;

//
// BCE: the binary cross entropy with logits of the reference's "bce" loss (kge/util/loss.py:137-158,
// reduction "sum") on x = s + offset against the label row y_j = (1 - eps) [j in P_i] + (eps > 0 ?
// 1 / m : 0) (train.py:715-721: smoothed labels are NOT normalised for this loss):
//   loss_i = sum_j softplus(x_j) - y_j x_j,     G_ij = scale (sigmoid(x_j) - y_j)
// in the same in-place plane form; no row statistics are needed, only the three sums.
// softplus(x) = max(x, 0) + log1p(e), sigmoid(x) = 1 / (1 + e) or e / (1 + e), e = exp(-|x|) in
// (0, 1] (no overflow for any x), on the hardware's exp / log / rcp (1 ulp each) instead of the
// correctly rounded library routines: log1p(e) as log(1 + e) while 1 + e keeps enough of e
// (e >= 2^-10: relative error below 2^-13 of a term that is itself below 1e-3 of the row's
// loss sum), as e - e^2 / 2 below (error e^3 / 3 < 2^-30 e).
__device__ __forceinline__ float softplus_f(float x) {
  const float e = __expf(-fabsf(x));
  const float big = __logf(1.f + e), small = e - 0.5f * e * e;
  return fmaxf(x, 0.f) + (e >= 9.765625e-4f ? big : small);
}
__device__ __forceinline__ float sigmoid_f(float x) {
  const float e = __expf(-fabsf(x));
  const float r = __builtin_amdgcn_rcpf(1.f + e);
  return x >= 0.f ? r : e * r;
}

template <int NI, int NTH, bool BCE = false>
__global__ void __launch_bounds__(NTH) softmax_planes_kernel(float* s, int64_t lds, int n, int m,
                                                             const int64_t* __restrict__ l_ptr,
                                                             const int64_t* __restrict__ l_col, float eps, float scale,
                                                             float* __restrict__ loss, float offset = 0.f) {
  __shared__ float red[3][NTH / 64];
  const int64_t row = blockIdx.x;
  float* sr = s + row * lds;
  const int tid = threadIdx.x;
  if (row >= n) {  // K-padding rows of both planes
    for (int64_t j = (int64_t)tid * 4; j < lds; j += (int64_t)NTH * 4)
      *reinterpret_cast<float4*>(sr + j) = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const int m4 = m & ~3;
  const int64_t p0 = l_ptr ? l_ptr[row] : row, p1 = l_ptr ? l_ptr[row + 1] : row + 1;
  // every read of the score row happens before the barriers inside row_stats_regs, i.e.
  // before any thread overwrites the row with the planes
  float ps = 0.f;
  for (int64_t k = p0 + tid; k < p1; k += NTH) {
    const int64_t c = l_col[k];
    ps += (c >= 0 && c < m) ? sr[c] : NAN;
  }
  const float tail = (m4 + tid < m) ? sr[m4 + tid] : 0.f;  // m - m4 <= 3 elements past the float4 part
  float mx, sm, rs;
  RowRegs<NI> regs;
  row_load_regs<NI, NTH>(sr, m, regs);
  if constexpr (BCE) {
    float sp = 0.f, sx = 0.f;  // sum of softplus(x), sum of x over this thread's elements
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int q = 0; q < U; ++q) {
        if (i * NTH * 4 * U + (q * NTH + tid) * 4 >= m4) continue;
        const float4 v = regs.v[i][q];
        const float x0 = v.x + offset, x1 = v.y + offset, x2 = v.z + offset, x3 = v.w + offset;
        sp += (softplus_f(x0) + softplus_f(x1)) + (softplus_f(x2) + softplus_f(x3));
        sx += (x0 + x1) + (x2 + x3);
      }
    if (m4 + tid < m) {
      sp += softplus_f(tail + offset);
      sx += tail + offset;
    }
    // every read of the score row is done once these sums have passed their barriers
    sp = block_sum<NTH>(sp, red[0]);
    sx = block_sum<NTH>(sx, red[1]);
    ps = block_sum<NTH>(ps, red[0]);
    const int64_t np = p1 - p0;
    const float u = eps > 0.f ? 1.f / (float)m : 0.f;
    if (tid == 0) loss[row] = sp - u * sx - (1.f - eps) * (ps + (float)np * offset);
    kge_bf16_t* hi = reinterpret_cast<kge_bf16_t*>(sr);
    kge_bf16_t* lo = hi + lds;
    const float b = scale * u;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int j = i * NTH * 4 * U + (q * NTH + tid) * 4;
        if (j >= m4) continue;
        const float4 v = regs.v[i][q];
        const float4 gv = make_float4(scale * sigmoid_f(v.x + offset) - b, scale * sigmoid_f(v.y + offset) - b,
                                      scale * sigmoid_f(v.z + offset) - b, scale * sigmoid_f(v.w + offset) - b);
        bf16x4 h, l;
        split_bf16x4_pk(gv, h, l);
        *reinterpret_cast<bf16x4*>(hi + j) = h;
        *reinterpret_cast<bf16x4*>(lo + j) = l;
      }
    if (m4 + tid < m) {
      kge_bf16_t h, l;
      split_bf16(scale * sigmoid_f(tail + offset) - b, h, l);
      hi[m4 + tid] = h;
      lo[m4 + tid] = l;
    }
    for (int64_t j = m + tid; j < lds; j += NTH) {  // K padding columns
      hi[j] = (kge_bf16_t)0.f;
      lo[j] = (kge_bf16_t)0.f;
    }
    __syncthreads();  // the row's planes are complete before the positives' fix-up
    const float dpos = scale * (1.f - eps);
    for (int64_t k = p0 + tid; k < p1; k += NTH) {
      const int64_t c = l_col[k];
      if (c >= 0 && c < m) {
        kge_bf16_t h, l;
        split_bf16(((float)hi[c] + (float)lo[c]) - dpos, h, l);
        hi[c] = h;
        lo[c] = l;
      }
    }
    return;
  }
  row_stats_regs<NI, NTH>(sr, m, regs, red, mx, sm, rs);
  ps = block_sum<NTH>(ps, red[0]);

  const float lse = mx + __logf(sm);
  const int64_t np = p1 - p0;
  const float u = eps > 0.f ? 1.f / (float)m : 0.f;
  const float z = (1.f - eps) * (float)np + (eps > 0.f ? 1.f : 0.f);
  const float zi = z > 1e-12f ? 1.f / z : 0.f;
  const float t0 = u * zi, t1 = ((1.f - eps) + u) * zi;
  const float T = z > 0.f ? 1.f : 0.f;
  if (tid == 0) {
    if (!l_ptr) {
      loss[row] = lse - ps;
    } else {
      const float H = (float)(m - np) * xlogx(t0) + (float)np * xlogx(t1);
      loss[row] = H - t0 * rs - (t1 - t0) * ps + (T > 0.f ? lse : 0.f);
    }
  }
  kge_bf16_t* hi = reinterpret_cast<kge_bf16_t*>(sr);
  kge_bf16_t* lo = hi + lds;
  const float a = scale * T, b = scale * t0;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int j = i * NTH * 4 * U + (q * NTH + tid) * 4;
      if (j >= m4) continue;
      const float4 v = regs.v[i][q];
      const float4 gv = make_float4(a * __expf(v.x - lse) - b, a * __expf(v.y - lse) - b, a * __expf(v.z - lse) - b,
                                    a * __expf(v.w - lse) - b);
      bf16x4 h, l;
      split_bf16x4_pk(gv, h, l);
      *reinterpret_cast<bf16x4*>(hi + j) = h;
      *reinterpret_cast<bf16x4*>(lo + j) = l;
    }
  if (m4 + tid < m) {
    kge_bf16_t h, l;
    split_bf16(a * __expf(tail - lse) - b, h, l);
    hi[m4 + tid] = h;
    lo[m4 + tid] = l;
  }
  for (int64_t j = m + tid; j < lds; j += NTH) {  // K padding columns
    hi[j] = (kge_bf16_t)0.f;
    lo[j] = (kge_bf16_t)0.f;
  }
  __syncthreads();  // the row's planes are complete before the positives' fix-up
  const float d = scale * (t1 - t0);
  for (int64_t k = p0 + tid; k < p1; k += NTH) {
    const int64_t c = l_col[k];
    if (c >= 0 && c < m) {
      kge_bf16_t h, l;
      split_bf16(((float)hi[c] + (float)lo[c]) - d, h, l);
      hi[c] = h;
      lo[c] = l;
    }
  }
}

template <bool BCE>
int launch_planes_t(float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m, const int64_t* l_ptr,
                    const int64_t* l_col, float eps, float scale, float* loss, float offset, hipStream_t st) {
  const int64_t m4 = m & ~3LL;
  const dim3 grid((unsigned)n_pad);
  if (m4 <= 256 * 4 * U)
    softmax_planes_kernel<1, 256, BCE><<<grid, dim3(256), 0, st>>>(s, lds, (int)n, (int)m, l_ptr, l_col, eps, scale,
                                                                   loss, offset);
  else if (m4 <= 2 * 256 * 4 * U)
    softmax_planes_kernel<2, 256, BCE><<<grid, dim3(256), 0, st>>>(s, lds, (int)n, (int)m, l_ptr, l_col, eps, scale,
                                                                   loss, offset);
  // wider rows: 512 threads holding 2 .. 4 register slabs each (1,024-thread workgroups cap a
  // thread at 128 VGPRs, which the two-slab row does not fit: it spilled 34 of them)
  else if (m4 <= 2 * 512 * 4 * U)
    softmax_planes_kernel<2, 512, BCE><<<grid, dim3(512), 0, st>>>(s, lds, (int)n, (int)m, l_ptr, l_col, eps, scale,
                                                                   loss, offset);
  else if (m4 <= 3 * 512 * 4 * U)
    softmax_planes_kernel<3, 512, BCE><<<grid, dim3(512), 0, st>>>(s, lds, (int)n, (int)m, l_ptr, l_col, eps, scale,
                                                                   loss, offset);
  else if (m4 <= 4 * 512 * 4 * U)
    softmax_planes_kernel<4, 512, BCE><<<grid, dim3(512), 0, st>>>(s, lds, (int)n, (int)m, l_ptr, l_col, eps, scale,
                                                                   loss, offset);
  else
    return KGE_ERR_ARG;
  KGE_CHECK_LAUNCH();
  return 0;
}

int launch_planes(float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m, const int64_t* l_ptr,
                  const int64_t* l_col, float eps, float scale, float* loss, hipStream_t st) {
  return launch_planes_t<false>(s, lds, n, n_pad, m, l_ptr, l_col, eps, scale, loss, 0.f, st);
}

// parts[0] = scale * sum of loss[0 .. n_first), parts[1] = scale * sum of loss[n_first .. n),
// total[0] = parts[0] + parts[1]: one workgroup, fixed summation order (deterministic).
__global__ void __launch_bounds__(256) loss_sums_kernel(const float* __restrict__ loss, int64_t n, int64_t n_first,
                                                        const int64_t* __restrict__ n_first_dev, float scale,
                                                        float* __restrict__ parts, float* __restrict__ total) {
  __shared__ float red[256 / 64];
  if (n_first_dev) n_first = *n_first_dev;
  float a = 0.f, b = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const float v = loss[i];
    if (i < n_first)
      a += v;
    else
      b += v;
  }
  a = block_sum<256>(a, red) * scale;
  b = block_sum<256>(b, red) * scale;
  if (threadIdx.x == 0) {
    parts[0] = a;
    parts[1] = b;
    total[0] = a + b;
  }
}

}  // namespace

extern "C" int kge_loss_sums(const float* loss, int64_t n, int64_t n_first, const int64_t* n_first_dev, float scale,
                             float* parts, float* total, void* stream) {
  KGE_REQUIRE(n >= 0 && n_first >= 0 && n_first <= n && (loss || n == 0) && parts && total);
  loss_sums_kernel<<<dim3(1), dim3(256), 0, as_stream(stream)>>>(loss, n, n_first, n_first_dev, scale, parts, total);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t kge_softmax_planes_max_columns(void) { return 4LL * 512 * 4 * U; }

extern "C" int kge_softmax_xent_planes(float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m,
                                       const int64_t* labels, float scale, float* loss, void* stream) {
  KGE_REQUIRE(n >= 0 && n_pad >= n && m >= 4 && m <= kge_softmax_planes_max_columns() && n_pad < (1LL << 31));
  KGE_REQUIRE(s && labels && loss && lds >= m);
  if (lds % 32 != 0 || !aligned16(s)) return KGE_ERR_ALIGN;
  if (n_pad == 0) return 0;
  return launch_planes(s, lds, n, n_pad, m, nullptr, labels, 0.f, scale, loss, as_stream(stream));
}

extern "C" int kge_softmax_kl_planes(float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m, const int64_t* l_ptr,
                                     const int64_t* l_col, float smoothing, float scale, float* loss, void* stream) {
  KGE_REQUIRE(n >= 0 && n_pad >= n && m >= 4 && m <= kge_softmax_planes_max_columns() && n_pad < (1LL << 31));
  KGE_REQUIRE(s && l_ptr && l_col && loss && lds >= m);
  KGE_REQUIRE(smoothing >= 0.f && smoothing < 1.f);
  if (lds % 32 != 0 || !aligned16(s)) return KGE_ERR_ALIGN;
  if (n_pad == 0) return 0;
  return launch_planes(s, lds, n, n_pad, m, l_ptr, l_col, smoothing, scale, loss, as_stream(stream));
}

// ---------------------------------------------------------------------------------------
// Negative-sampling losses on a [n, k] score block whose column 0 is the positive and whose other
// columns are its negatives (train.py:858-871, 982-993), loss and gradient in one launch:
//   KGE_NS_MARGIN  loss_i = sum_{j >= 1} max(0, arg - s_i0 + s_ij)            (loss.py:227-250:
//                  MarginRankingLoss(positives, negatives, +1), margin = arg, reduction sum)
//   KGE_NS_BCE     loss_i = softplus(x_i0) - x_i0 + sum_{j >= 1} softplus(x_ij), x = s + arg
//                  (loss.py:137-158: BCEWithLogitsLoss against the label matrix [1, 0, ..., 0])
// g = scale * dloss/ds; one workgroup per row, fixed summation order.
namespace {
template <int KIND>
__global__ void __launch_bounds__(NT) ns_loss_kernel(const float* __restrict__ s, int64_t lds, int k, float arg,
                                                     float scale, float* __restrict__ loss, float* __restrict__ g,
                                                     int64_t ldg) {
  __shared__ float red[2][NT / 64];
  const int64_t row = blockIdx.x;
  const float* sr = s + row * lds;
  float* gr = g + row * ldg;
  const int tid = threadIdx.x;
  const float pos = sr[0];
  float acc = 0.f, cnt = 0.f;
  for (int j = 1 + tid; j < k; j += NT) {
    const float v = sr[j];
    if (KIND == KGE_NS_MARGIN) {
      const float h = (v - pos) + arg;  // torch: -(x1 - x2) + margin, clamped at 0
      const bool on = h >= 0.f;         // clamp_min's backward passes the gradient where h >= 0
      acc += on ? h : 0.f;
      cnt += on ? 1.f : 0.f;
      gr[j] = on ? scale : 0.f;
    } else {
      const float x = v + arg;
      acc += softplus_f(x);
      gr[j] = scale * sigmoid_f(x);
    }
  }
  acc = block_sum<NT>(acc, red[0]);
  cnt = block_sum<NT>(cnt, red[1]);
  if (tid == 0) {
    if (KIND == KGE_NS_MARGIN) {
      loss[row] = acc;
      gr[0] = -scale * cnt;
    } else {
      const float x = pos + arg;
      loss[row] = acc + softplus_f(x) - x;
      gr[0] = -scale * sigmoid_f(-x);  // sigmoid(x) - 1 without the cancellation
    }
  }
}
}  // namespace

extern "C" int kge_ns_loss(int kind, const float* s, int64_t lds, int64_t n, int64_t k, float arg, float scale,
                           float* loss, float* g, int64_t ldg, void* stream) {
  KGE_REQUIRE(n >= 0 && k >= 1 && k < (1LL << 31) && n < (1LL << 31) && s && loss && g && lds >= k && ldg >= k);
  KGE_REQUIRE(kind == KGE_NS_MARGIN || kind == KGE_NS_BCE);
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  if (kind == KGE_NS_MARGIN)
    ns_loss_kernel<KGE_NS_MARGIN><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)k, arg, scale, loss, g, ldg);
  else
    ns_loss_kernel<KGE_NS_BCE><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)k, arg, scale, loss, g, ldg);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_bce_planes(float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m, const int64_t* l_ptr,
                              const int64_t* l_col, float smoothing, float offset, float scale, float* loss,
                              void* stream) {
  KGE_REQUIRE(n >= 0 && n_pad >= n && m >= 4 && m <= kge_softmax_planes_max_columns() && n_pad < (1LL << 31));
  KGE_REQUIRE(s && l_col && loss && lds >= m);
  KGE_REQUIRE(smoothing >= 0.f && smoothing < 1.f && (l_ptr || smoothing == 0.f));
  if (lds % 32 != 0 || !aligned16(s)) return KGE_ERR_ALIGN;
  if (n_pad == 0) return 0;
  return launch_planes_t<true>(s, lds, n, n_pad, m, l_ptr, l_col, smoothing, scale, loss, offset, as_stream(stream));
}

extern "C" int kge_softmax_xent(const float* s, int64_t lds, int64_t n, int64_t m, const int64_t* labels,
                                float scale, float* loss, float* g, int64_t ldg, void* stream) {
  KGE_REQUIRE(n >= 0 && m > 0 && m < (1LL << 31) && n < (1LL << 31));
  KGE_REQUIRE(s && labels && loss && lds >= m && (!g || ldg >= m));
  KGE_REQUIRE(!g || g != s || ldg == lds);  // in place only row-for-row
  if (n == 0) return 0;
  return launch(s, lds, n, m, nullptr, labels, 0.f, scale, loss, g, ldg, as_stream(stream));
}

extern "C" int kge_softmax_kl(const float* s, int64_t lds, int64_t n, int64_t m, const int64_t* l_ptr,
                              const int64_t* l_col, float smoothing, float scale, float* loss, float* g, int64_t ldg,
                              void* stream) {
  KGE_REQUIRE(n >= 0 && m > 0 && m < (1LL << 31) && n < (1LL << 31));
  KGE_REQUIRE(s && l_ptr && l_col && loss && lds >= m && (!g || ldg >= m));
  KGE_REQUIRE(!g || g != s || ldg == lds);
  KGE_REQUIRE(smoothing >= 0.f && smoothing < 1.f);
  if (n == 0) return 0;
  return launch(s, lds, n, m, l_ptr, l_col, smoothing, scale, loss, g, ldg, as_stream(stream));
}

extern "C" int kge_softmax_row_stats(const float* s, int64_t lds, int64_t n, int64_t m, int64_t c0,
                                     const int64_t* labels, float* row_max, float* row_sumexp, float* target,
                                     void* stream) {
  KGE_REQUIRE(n >= 0 && m > 0 && m < (1LL << 31) && n < (1LL << 31) && lds >= m);
  KGE_REQUIRE(s && row_max && row_sumexp && (!target || labels));
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  if (vec_ok(s, lds, nullptr, 0))
    row_stats_kernel<true><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)m, c0, labels, row_max, row_sumexp,
                                                                   target);
  else
    row_stats_kernel<false><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)m, c0, labels, row_max, row_sumexp,
                                                                    target);
  KGE_CHECK_LAUNCH();
  return 0;
}

// kge_softmax_grad with G left as bf16 hi / lo planes in a buffer of its own (rows of ld floats:
// ld bf16 of the hi plane, then ld bf16 of the lo plane -- the layout of the in-place kernels
// above, which the plane-fed GEMMs read).  Out of place because a row need not fit a workgroup's
// registers here (a shard of a large entity table): elementwise, any row length.  Columns
// [m, ld) and rows [n, n_pad) are zeroed (K padding of the GEMMs).
constexpr int GP_CH = 4096;  // columns per workgroup

// BCE: the same planes for binary cross entropy with logits on x = s + offset against the one-hot
// label row (loss.py:137-158, reduction "sum"): G = scale (sigmoid(x) - y), and the chunk's share of
// the row's loss, sum_j softplus(x_j) - y_j x_j, into loss_part[row][chunk] (summed by the caller
// in a fixed order).  Nothing couples the columns, so a shard needs no statistics of the others.
template <bool VEC, bool BCE = false>
__global__ void __launch_bounds__(NT) grad_planes_kernel(const float* __restrict__ s, int64_t lds, int n, int m,
                                                         int64_t c0, const int64_t* __restrict__ labels,
                                                         const float* __restrict__ lse, float scale,
                                                         float* __restrict__ planes, int64_t ld, float offset = 0.f,
                                                         float* __restrict__ loss_part = nullptr) {
  __shared__ float red[NT / 64];
  const int64_t row = blockIdx.y;
  const int tid = threadIdx.x;
  const int64_t j0 = (int64_t)blockIdx.x * GP_CH, j1 = min(j0 + GP_CH, ld);
  kge_bf16_t* hi = reinterpret_cast<kge_bf16_t*>(planes + row * ld);
  kge_bf16_t* lo = hi + ld;
  if (row >= n) {  // K-padding rows
    for (int64_t j = j0 + (int64_t)tid * 4; j < j1; j += (int64_t)NT * 4) {  // ld % 4 == 0
      *reinterpret_cast<uint2*>(hi + j) = make_uint2(0u, 0u);
      *reinterpret_cast<uint2*>(lo + j) = make_uint2(0u, 0u);
    }
    return;
  }
  const float* sr = s + row * lds;
  const float l = BCE ? 0.f : lse[row];
  const int64_t lab = labels ? labels[row] - c0 : -1;
  float part = 0.f;
  for (int64_t j = j0 + (int64_t)tid * 4; j < j1; j += (int64_t)NT * 4) {
    float v[4];
    if (VEC && j + 3 < m) {
      const float4 x = *reinterpret_cast<const float4*>(sr + j);
      v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w;
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = j + c < m ? sr[j + c] : 0.f;
    }
    float g[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bool in = j + c < m, hit = j + c == lab && in;  // a label of another shard may fall into the padding
      if constexpr (BCE) {
        const float x = v[c] + offset;
        g[c] = in ? scale * sigmoid_f(x) : 0.f;  // K padding columns: 0
        if (in) part += softplus_f(x) - (hit ? x : 0.f);
      } else {
        g[c] = in ? scale * __expf(v[c] - l) : 0.f;
      }
      if (hit) g[c] -= scale;
    }
    bf16x4 h, lw;
    split_bf16x4_pk(make_float4(g[0], g[1], g[2], g[3]), h, lw);
    *reinterpret_cast<bf16x4*>(hi + j) = h;
    *reinterpret_cast<bf16x4*>(lo + j) = lw;
  }
  if constexpr (BCE) {
    part = block_sum<NT>(part, red);
    if (tid == 0) loss_part[row * gridDim.x + blockIdx.x] = part;
  }
}

extern "C" int kge_softmax_grad_planes(const float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m, int64_t c0,
                                       const int64_t* labels, const float* lse, float scale, float* planes,
                                       int64_t ld, void* stream) {
  KGE_REQUIRE(n >= 0 && n_pad >= n && n_pad < (1LL << 31) && m > 0 && m < (1LL << 31) && lds >= m);
  KGE_REQUIRE(s && lse && planes && ld >= m && planes != s);
  if (ld % 32 != 0 || !aligned16(planes)) return KGE_ERR_ALIGN;
  if (n_pad == 0) return 0;
  hipStream_t st = as_stream(stream);
  // grid.y carries the rows (<= 65,535 per launch: larger batches go in slices)
  for (int64_t r0 = 0; r0 < n_pad; r0 += 65535) {
    const int64_t rows = std::min<int64_t>(65535, n_pad - r0);
    const int64_t n_here = std::max<int64_t>(0, std::min<int64_t>(n - r0, rows));
    const dim3 grid((unsigned)((ld + GP_CH - 1) / GP_CH), (unsigned)rows);
    const float* sp = s + r0 * lds;
    const int64_t* lp = labels ? labels + r0 : nullptr;
    if (lds % 4 == 0 && aligned16(s))
      grad_planes_kernel<true><<<grid, dim3(NT), 0, st>>>(sp, lds, (int)n_here, (int)m, c0, lp, lse + r0, scale,
                                                          planes + r0 * ld, ld);
    else
      grad_planes_kernel<false><<<grid, dim3(NT), 0, st>>>(sp, lds, (int)n_here, (int)m, c0, lp, lse + r0, scale,
                                                           planes + r0 * ld, ld);
    KGE_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int64_t kge_grad_planes_chunks(int64_t ld) { return ld <= 0 ? 0 : (ld + GP_CH - 1) / GP_CH; }

extern "C" int kge_bce_grad_planes(const float* s, int64_t lds, int64_t n, int64_t n_pad, int64_t m, int64_t c0,
                                   const int64_t* labels, float offset, float scale, float* planes, int64_t ld,
                                   float* loss_part, void* stream) {
  KGE_REQUIRE(n >= 0 && n_pad >= n && n_pad < (1LL << 31) && m > 0 && m < (1LL << 31) && lds >= m);
  KGE_REQUIRE(s && planes && ld >= m && planes != s && (loss_part || n == 0));
  if (ld % 32 != 0 || !aligned16(planes)) return KGE_ERR_ALIGN;
  if (n_pad == 0) return 0;
  hipStream_t st = as_stream(stream);
  const int64_t chunks = kge_grad_planes_chunks(ld);
  for (int64_t r0 = 0; r0 < n_pad; r0 += 65535) {  // grid.y carries the rows, as in kge_softmax_grad_planes
    const int64_t rows = std::min<int64_t>(65535, n_pad - r0);
    const int64_t n_here = std::max<int64_t>(0, std::min<int64_t>(n - r0, rows));
    const dim3 grid((unsigned)chunks, (unsigned)rows);
    const float* sp = s + r0 * lds;
    const int64_t* lp = labels ? labels + r0 : nullptr;
    if (lds % 4 == 0 && aligned16(s))
      grad_planes_kernel<true, true><<<grid, dim3(NT), 0, st>>>(sp, lds, (int)n_here, (int)m, c0, lp, nullptr, scale,
                                                                planes + r0 * ld, ld, offset, loss_part + r0 * chunks);
    else
      grad_planes_kernel<false, true><<<grid, dim3(NT), 0, st>>>(sp, lds, (int)n_here, (int)m, c0, lp, nullptr, scale,
                                                                 planes + r0 * ld, ld, offset, loss_part + r0 * chunks);
    KGE_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int kge_softmax_grad(const float* s, int64_t lds, int64_t n, int64_t m, int64_t c0, const int64_t* labels,
                                const float* lse, float scale, float* g, int64_t ldg, void* stream) {
  KGE_REQUIRE(n >= 0 && m > 0 && m < (1LL << 31) && n < (1LL << 31) && lds >= m);
  KGE_REQUIRE(s && lse && g && ldg >= m && (g != s || ldg == lds));
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  if (vec_ok(s, lds, g, ldg))
    grad_kernel<true><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)m, c0, labels, lse, scale, g, ldg);
  else
    grad_kernel<false><<<dim3((unsigned)n), dim3(NT), 0, st>>>(s, lds, (int)m, c0, labels, lse, scale, g, ldg);
  KGE_CHECK_LAUNCH();
  return 0;
}

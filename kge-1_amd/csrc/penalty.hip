// Frequency-weighted Lp penalty of a lookup embedder over the OCCURRENCES of a batch's indexes
// (lookup_embedder.py:138-158: sum over unique indexes of count * sum_k |x_k|^p -- a row that
// occurs c times contributes c equal terms, so the sum over occurrences is the same number):
//   row_sums[i]  = sum_k |w[idx[i], k]|^p                              (kge_lp_rows)
//   d_w[idx[i], k] += gscale * p * sign(x) * |x|^(p-1),  x = w[idx[i], k]   (kge_lp_rows_bwd)
// One workgroup per occurrence; the caller sums the row sums (fixed order) and scales.  The
// backward adds with float atomics: the c contributions to one row are equal, so their order
// does not change the result.  p = 1, 2, 3 or 4.
#include "common.h"

namespace {

template <int P>
__device__ __forceinline__ float lp_term(float x) {
  const float a = fabsf(x);
  if (P == 1) return a;
  if (P == 2) return x * x;
  if (P == 3) return a * a * a;
  return (x * x) * (x * x);
}

template <int P>
__device__ __forceinline__ float lp_grad(float x) {  // d/dx |x|^p
  if (P == 1) return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
  if (P == 2) return 2.f * x;
  if (P == 3) return 3.f * x * fabsf(x);
  return 4.f * x * x * x;
}

template <int P>
__global__ void __launch_bounds__(128) lp_rows_kernel(const float* __restrict__ w, int64_t ldw,
                                                      const int64_t* __restrict__ idx, int d,
                                                      float* __restrict__ row_sums) {
  __shared__ float red[2];
  const int64_t i = blockIdx.x;
  const float* x = w + idx[i] * ldw;
  float acc = 0.f;
  for (int k = threadIdx.x; k < d; k += 128) acc += lp_term<P>(x[k]);
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) row_sums[i] = red[0] + red[1];
}

template <int P>
__global__ void __launch_bounds__(128) lp_rows_bwd_kernel(const float* __restrict__ w, int64_t ldw,
                                                          const int64_t* __restrict__ idx, int d,
                                                          const float* __restrict__ gscale, float coeff,
                                                          float* __restrict__ dw, int64_t lddw) {
  const int64_t row = idx[blockIdx.x];
  const float* x = w + row * ldw;
  float* o = dw + row * lddw;
  const float s = coeff * (gscale ? *gscale : 1.f);
  for (int k = threadIdx.x; k < d; k += 128) atomicAdd(o + k, s * lp_grad<P>(x[k]));
}

}  // namespace

extern "C" int kge_lp_rows(const float* w, int64_t ldw, const int64_t* idx, int64_t n, int d, int p, float* row_sums,
                           void* stream) {
  KGE_REQUIRE(n >= 0 && n < (1LL << 31) && d > 0 && ldw >= d && p >= 1 && p <= 4);
  if (n == 0) return 0;
  KGE_REQUIRE(w && idx && row_sums);
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)n), block(128);
  switch (p) {
    case 1: lp_rows_kernel<1><<<grid, block, 0, st>>>(w, ldw, idx, d, row_sums); break;
    case 2: lp_rows_kernel<2><<<grid, block, 0, st>>>(w, ldw, idx, d, row_sums); break;
    case 3: lp_rows_kernel<3><<<grid, block, 0, st>>>(w, ldw, idx, d, row_sums); break;
    default: lp_rows_kernel<4><<<grid, block, 0, st>>>(w, ldw, idx, d, row_sums); break;
  }
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_lp_rows_bwd(const float* w, int64_t ldw, const int64_t* idx, int64_t n, int d, int p,
                               const float* gscale, float coeff, float* dw, int64_t lddw, void* stream) {
  KGE_REQUIRE(n >= 0 && n < (1LL << 31) && d > 0 && ldw >= d && lddw >= d && p >= 1 && p <= 4);
  if (n == 0) return 0;
  KGE_REQUIRE(w && idx && dw);
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)n), block(128);
  switch (p) {
    case 1: lp_rows_bwd_kernel<1><<<grid, block, 0, st>>>(w, ldw, idx, d, gscale, coeff, dw, lddw); break;
    case 2: lp_rows_bwd_kernel<2><<<grid, block, 0, st>>>(w, ldw, idx, d, gscale, coeff, dw, lddw); break;
    case 3: lp_rows_bwd_kernel<3><<<grid, block, 0, st>>>(w, ldw, idx, d, gscale, coeff, dw, lddw); break;
    default: lp_rows_bwd_kernel<4><<<grid, block, 0, st>>>(w, ldw, idx, d, gscale, coeff, dw, lddw); break;
  }
  KGE_CHECK_LAUNCH();
  return 0;
}

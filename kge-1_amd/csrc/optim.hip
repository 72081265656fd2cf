// Fused Adagrad step for the embedding tables: one pass over (param, grad, state sum)
// instead of torch's foreach sequence (addcmul, sqrt, add, mul, addcdiv: five passes,
// ~82 us per 1vsAll step at C2).  Same arithmetic per element, in the same order, as
// torch.optim.Adagrad's multi-tensor path (torch/optim/adagrad.py, _multi_tensor_adagrad):
//   g  = maximize ? -grad : grad;   g = g + wd * p      (weight_decay != 0)
//   s  = s + g * g
//   p  = p + (g * minus_clr) / (sqrt(s) + eps)
// The optimizer behind the reference's train.optimizer "Adagrad" (kge/util/optimizer.py:11-32).
#include "common.h"

namespace {

__device__ __forceinline__ void adagrad1(float& p, float g, float& s, float minus_clr, float eps, float wd,
                                         bool maximize) {
  if (maximize) g = -g;
  if (wd != 0.f) g = g + wd * p;
  s = s + g * g;
  const float stdv = __fsqrt_rn(s) + eps;
  p = p + (g * minus_clr) / stdv;
}

__global__ void __launch_bounds__(256) adagrad_vec_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                          float4* __restrict__ s, int64_t n4, float minus_clr,
                                                          float eps, float wd, int maximize) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 pv = p[i], sv = s[i];
    const float4 gv = g[i];
    adagrad1(pv.x, gv.x, sv.x, minus_clr, eps, wd, maximize);
    adagrad1(pv.y, gv.y, sv.y, minus_clr, eps, wd, maximize);
    adagrad1(pv.z, gv.z, sv.z, minus_clr, eps, wd, maximize);
    adagrad1(pv.w, gv.w, sv.w, minus_clr, eps, wd, maximize);
    p[i] = pv;
    s[i] = sv;
  }
}

__global__ void __launch_bounds__(256) adagrad_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ s, int64_t n, float minus_clr, float eps,
                                                      float wd, int maximize) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    adagrad1(p[i], g[i], s[i], minus_clr, eps, wd, maximize);
}

// Several tensors in one launch: block b works on the tensor whose block range holds it.
constexpr int ADAGRAD_MAX = 8;
struct AdagradMulti {
  float* p[ADAGRAD_MAX];
  const float* g[ADAGRAD_MAX];
  float* s[ADAGRAD_MAX];
  int64_t n[ADAGRAD_MAX];
  float minus_clr[ADAGRAD_MAX];
  int first_block[ADAGRAD_MAX + 1];
  int vec[ADAGRAD_MAX];  // n % 4 == 0 and all three pointers 16-B aligned
};

__global__ void __launch_bounds__(256) adagrad_multi_kernel(const AdagradMulti a, int count, float eps, float wd,
                                                            int maximize) {
  int t = 0;
  while (t + 1 < count && (int)blockIdx.x >= a.first_block[t + 1]) ++t;  // block-uniform
  const int64_t b = blockIdx.x - a.first_block[t], nb = a.first_block[t + 1] - a.first_block[t];
  const float clr = a.minus_clr[t];
  if (a.vec[t]) {
    float4* p = reinterpret_cast<float4*>(a.p[t]);
    const float4* g = reinterpret_cast<const float4*>(a.g[t]);
    float4* s = reinterpret_cast<float4*>(a.s[t]);
    const int64_t n4 = a.n[t] / 4;
    for (int64_t i = b * blockDim.x + threadIdx.x; i < n4; i += nb * blockDim.x) {
      float4 pv = p[i], sv = s[i];
      const float4 gv = g[i];
      adagrad1(pv.x, gv.x, sv.x, clr, eps, wd, maximize);
      adagrad1(pv.y, gv.y, sv.y, clr, eps, wd, maximize);
      adagrad1(pv.z, gv.z, sv.z, clr, eps, wd, maximize);
      adagrad1(pv.w, gv.w, sv.w, clr, eps, wd, maximize);
      p[i] = pv;
      s[i] = sv;
    }
  } else {
    for (int64_t i = b * blockDim.x + threadIdx.x; i < a.n[t]; i += nb * blockDim.x)
      adagrad1(a.p[t][i], a.g[t][i], a.s[t][i], clr, eps, wd, maximize);
  }
}

}  // namespace

extern "C" int kge_adagrad_step_multi(int count, float* const* params, const float* const* grads,
                                      float* const* state_sums, const int64_t* ns, const float* minus_clrs, float eps,
                                      float weight_decay, int maximize, void* stream) {
  KGE_REQUIRE(count >= 0 && count <= ADAGRAD_MAX && (count == 0 || (params && grads && state_sums && ns && minus_clrs)));
  AdagradMulti a;
  const int cus = kge_num_cus();
  int blocks = 0, used = 0;
  for (int t = 0; t < count; ++t) {
    KGE_REQUIRE(ns[t] >= 0 && (ns[t] == 0 || (params[t] && grads[t] && state_sums[t])));
    if (ns[t] == 0) continue;
    a.p[used] = params[t];
    a.g[used] = grads[t];
    a.s[used] = state_sums[t];
    a.n[used] = ns[t];
    a.minus_clr[used] = minus_clrs[t];
    a.vec[used] = ns[t] % 4 == 0 && aligned16(params[t]) && aligned16(grads[t]) && aligned16(state_sums[t]);
    const int64_t items = a.vec[used] ? ns[t] / 4 : ns[t];
    a.first_block[used] = blocks;
    blocks += (int)std::min<int64_t>((items + 255) / 256, (int64_t)cus * 8);
    ++used;
  }
  if (used == 0) return 0;
  a.first_block[used] = blocks;
  adagrad_multi_kernel<<<dim3(blocks), dim3(256), 0, as_stream(stream)>>>(a, used, eps, weight_decay, maximize);
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_adagrad_step(float* param, const float* grad, float* state_sum, int64_t n, float minus_clr,
                                float eps, float weight_decay, int maximize, void* stream) {
  KGE_REQUIRE(n >= 0 && param && grad && state_sum);
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  const int cus = kge_num_cus();
  if (n % 4 == 0 && aligned16(param) && aligned16(grad) && aligned16(state_sum)) {
    const int64_t n4 = n / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, (int64_t)cus * 8);
    adagrad_vec_kernel<<<dim3(blocks), dim3(256), 0, st>>>((float4*)param, (const float4*)grad, (float4*)state_sum,
                                                           n4, minus_clr, eps, weight_decay, maximize);
  } else {
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, (int64_t)cus * 8);
    adagrad_kernel<<<dim3(blocks), dim3(256), 0, st>>>(param, grad, state_sum, n, minus_clr, eps, weight_decay,
                                                       maximize);
  }
  KGE_CHECK_LAUNCH();
  return 0;
}

// Index staging for the replayed training step: n int64 from host-pinned (device-visible)
// memory into a device buffer by a kernel on the compute stream -- no DMA-engine hand-off
// between the copy and the recorded step that reads it.
namespace {
__global__ void __launch_bounds__(256) stage_i64_kernel(const int64_t* __restrict__ src, int64_t* __restrict__ dst,
                                                        int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
}  // namespace

extern "C" int kge_stage_i64(const int64_t* src, int64_t* dst, int64_t n, void* stream) {
  KGE_REQUIRE(n >= 0 && src && dst);
  if (n == 0) return 0;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 64);
  stage_i64_kernel<<<dim3(blocks), dim3(256), 0, as_stream(stream)>>>(src, dst, n);
  KGE_CHECK_LAUNCH();
  return 0;
}

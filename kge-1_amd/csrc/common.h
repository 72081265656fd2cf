// Shared device helpers for libkgescore (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>

#include "../../include/kgescore.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define KGE_WAVE 64

#define KGE_CHECK_LAUNCH()                                   \
  do {                                                       \
    hipError_t _e = hipGetLastError();                       \
    if (_e != hipSuccess) return (int)_e;                    \
  } while (0)

#define KGE_REQUIRE(cond) \
  do {                    \
    if (!(cond)) return KGE_ERR_ARG; \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline bool aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// Split an fp32 value into bf16 hi + bf16 lo with x ~= hi + lo (|x - hi - lo| <= 2^-16 |x|).
__device__ __forceinline__ void split_bf16(float x, __bf16& hi, __bf16& lo) {
  hi = (__bf16)x;
  lo = (__bf16)(x - (float)hi);
}

// Split four fp32 values into bf16x4 hi / lo planes.
__device__ __forceinline__ void split_bf16x4(const float4& v, bf16x4& hi, bf16x4& lo) {
  const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const __bf16 h = (__bf16)x[c];
    hi[c] = h;
    lo[c] = (__bf16)(x[c] - (float)h);
  }
}

// The same split (bit-identical: round-to-nearest-even hi, round-to-nearest-even lo of the
// exact residual) with each v_cvt_pk_bf16_f32 converting a PAIR of values and hi widened back
// to fp32 by a shift / mask of the packed word: 12 VALU per 4 values instead of 20 (hipcc
// emits one single-value cvt per element for the scalar form).  The residual subtractions
// are scalar v_sub_f32 (hipcc would SLP-pack them into v_pk_add_f32, which costs issue
// cycles beside MFMAs, MI355X_MICROARCH.md cycle constants 'price of one filler').
typedef __bf16 kge_bf16x2 __attribute__((ext_vector_type(2)));
typedef float kge_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((kge_f32x2){a, b}, kge_bf16x2));
}
__device__ __forceinline__ float sub_f32_scalar(float a, float b) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ void split_bf16x4_pk(const float4& v, bf16x4& hi, bf16x4& lo) {
  const unsigned h0 = pack_bf16x2(v.x, v.y), h1 = pack_bf16x2(v.z, v.w);
  const float rx = sub_f32_scalar(v.x, __uint_as_float(h0 << 16));
  const float ry = sub_f32_scalar(v.y, __uint_as_float(h0 & 0xffff0000u));
  const float rz = sub_f32_scalar(v.z, __uint_as_float(h1 << 16));
  const float rw = sub_f32_scalar(v.w, __uint_as_float(h1 & 0xffff0000u));
  const unsigned l0 = pack_bf16x2(rx, ry), l1 = pack_bf16x2(rz, rw);
  hi = __builtin_bit_cast(bf16x4, (uint2){h0, h1});
  lo = __builtin_bit_cast(bf16x4, (uint2){l0, l1});
}

// The paired split with plain C++ subtractions (dev A/B against the asm form above).
__device__ __forceinline__ void split_bf16x4_pk_c(const float4& v, bf16x4& hi, bf16x4& lo) {
  const unsigned h0 = pack_bf16x2(v.x, v.y), h1 = pack_bf16x2(v.z, v.w);
  const float rx = v.x - __uint_as_float(h0 << 16), ry = v.y - __uint_as_float(h0 & 0xffff0000u);
  const float rz = v.z - __uint_as_float(h1 << 16), rw = v.w - __uint_as_float(h1 & 0xffff0000u);
  const unsigned l0 = pack_bf16x2(rx, ry), l1 = pack_bf16x2(rz, rw);
  hi = __builtin_bit_cast(bf16x4, (uint2){h0, h1});
  lo = __builtin_bit_cast(bf16x4, (uint2){l0, l1});
}

// Per-device host-side caches are indexed by the HIP device ordinal (one process may drive
// several GPUs; function attributes and device properties belong to one device each).
constexpr int KGE_MAX_DEVICES = 64;
static inline int kge_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= KGE_MAX_DEVICES) dev = 0;
  return dev;
}

// Compute units of the current device (256 on MI355X); cached per device.
static inline int kge_num_cus() {
  static std::atomic<int> cus[KGE_MAX_DEVICES];
  const int dev = kge_device();
  int c = cus[dev].load(std::memory_order_relaxed);
  if (c <= 0) {
    int real = 0;
    if (hipGetDevice(&real) != hipSuccess ||
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, real) != hipSuccess || c <= 0)
      c = 256;
    cus[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}

// Raise a kernel's dynamic-LDS limit once per device (hipFuncSetAttribute acts on the
// current device only).  `done` is a zero-initialised array of KGE_MAX_DEVICES flags owned by
// the launch site; concurrent first calls both set the attribute, which is harmless.
static inline int kge_allow_lds(const void* fn, int bytes, std::atomic<bool>* done) {
  const int dev = kge_device();
  if (!done[dev].load(std::memory_order_acquire)) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return (int)e;
    done[dev].store(true, std::memory_order_release);
  }
  return 0;
}

// bf16x3 backward GEMMs (gemm_bwd3.hip), dispatched from kge_score_dot_bwd_q / _t.
int kge_bwd3_q_splits(int64_t n, int64_t m, int d, int cus);
int kge_bwd3_q(const float* g, int64_t ldg, const float* t, int64_t ldt, const int64_t* tidx, int64_t n,
               int64_t m, int d, float* dq, int64_t lddq, int accumulate, float* ws, int64_t ws_elems, int cus,
               hipStream_t st);
int kge_bwd3_t(const float* g, int64_t ldg, const float* q, int64_t ldq, const int64_t* tidx, int64_t n,
               int64_t m, int d, float* dt, int64_t lddt, int accumulate, hipStream_t st);

// x[i, 0 .. d) = 0 for i < n by a fill kernel (gemm_bwd3.hip): unlike hipMemset*Async it may
// be recorded into a HIP graph by a capturing caller.
int kge_zero_rows(float* x, int64_t ldx, int64_t n, int d, hipStream_t st);

// packed-VALU all-entities distance kernel (score_dist2.hip); -1 when the layout does not fit
int kge_score_dist2(int kind, float sign, const float* q, int64_t ldq, const float* t, int64_t ldt,
                    const int64_t* tidx, int64_t n, int64_t m, int d, float* s, int64_t lds, hipStream_t st);

// owner-computes distance backward from ready pair weights (score_dist_bwd2.hip); -1 when the
// layout does not fit
int kge_score_dist_bwd_own(int kind, float scale, const float* w, int64_t ldw, const float* q, int64_t ldq,
                           const float* t, int64_t ldt, const int64_t* tidx, int64_t n, int64_t m, int d, float* dq,
                           int64_t lddq, float* dt, int64_t lddt, hipStream_t st);

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T ceil_div(T a, T b) {
  return (a + b - 1) / b;
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): consecutive logical ids land on the same XCD, so tiles that share
// an operand panel share that XCD's L2.  Placement is a speed hint only.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int nx = 8;
  int q = nblocks / nx, r = nblocks % nx;
  int xcd = bid % nx, local = bid / nx;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + local;
}

// Machine-ceiling probes for the benchmark's roofline report (measurement tooling, its own
// library libkgeprobe.so; the scoring library never loads it):
//   kge_probe_copy  -- streaming float4 copy, the achievable HBM read + write rate;
//   kge_probe_mfma  -- register-resident v_mfma_f32_16x16x32_bf16 chains on every SIMD (no
//                      LDS, no memory in the loop), the achievable dense bf16 MFMA rate of the
//                      chip at the clock it sustains for the given operand data: zeros draw
//                      little power, random operands run into the power limit first.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

int num_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return cus;
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) copy_kernel(const float4* __restrict__ src, float4* __restrict__ dst, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

__device__ __forceinline__ unsigned mix(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// ACCS independent accumulator chains per wave; every iteration issues 2 * ACCS MFMAs.
constexpr int ACCS = 8;

__global__ void __launch_bounds__(512, 1) mfma_kernel(int iters, int random, float* __restrict__ out) {
  const unsigned id = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8 a[2], b[4];
  for (int i = 0; i < 2; ++i)
    for (int k = 0; k < 8; ++k) {
      // bf16 with a random sign and mantissa and an exponent in [2^-2, 2^1): products of mixed sign
      const unsigned r = mix(id * 64u + i * 8u + k);
      const unsigned short bits = (unsigned short)((r & 0x807fu) | ((125u + ((r >> 8) & 3u)) << 7));
      a[i][k] = random ? __builtin_bit_cast(__bf16, bits) : (__bf16)0.f;
    }
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 8; ++k) {
      const unsigned r = mix(id * 64u + 32u + i * 8u + k);
      const unsigned short bits = (unsigned short)((r & 0x807fu) | ((125u + ((r >> 8) & 3u)) << 7));
      b[i][k] = random ? __builtin_bit_cast(__bf16, bits) : (__bf16)0.f;
    }
  f32x4 acc[ACCS];
  for (int i = 0; i < ACCS; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACCS; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i & 1], b[i & 3], acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < ACCS; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[(i + 1) & 1], b[(i + 2) & 3], acc[i], 0, 0, 0);
  }
  f32x4 s = acc[0];
  for (int i = 1; i < ACCS; ++i) s += acc[i];
  out[id] = s[0] + s[1] + s[2] + s[3];
}

// The contraction kernel's inner loop without its staging: 8 waves, per "stage" every wave reads
// its operand fragments from a resident 64-KB LDS image (ds_read_b128, the kernel's swizzled
// [row][k] layout: 2 * 8 A reads, one band ahead of their use, and 2 * 4 B reads) and issues
// 8 x 4 x 3 MFMAs.  MODE bit 0: the A reads, bit 1: the B reads, bit 2: a barrier per stage.
__device__ __forceinline__ int sw16_off(int row, int slot) {
  return row * 64 + ((slot ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3)) << 4);
}

template <int MODE>
__global__ void __launch_bounds__(512, 1) mfma_lds_kernel(int stages, float* __restrict__ out) {
  constexpr int TM = 8, TN = 4, PLANE = 256 * 64;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3, fr = lane & 15, fs = lane >> 4;
  for (int i = tid; i < 4 * PLANE / 4; i += 512) {
    const unsigned r0 = mix(blockIdx.x * 65536u + 2u * i), r1 = mix(blockIdx.x * 65536u + 2u * i + 1u);
    const unsigned lo16 = (r0 & 0x807fu) | ((125u + ((r0 >> 8) & 3u)) << 7);
    const unsigned hi16 = (r1 & 0x807fu) | ((125u + ((r1 >> 8) & 3u)) << 7);
    reinterpret_cast<unsigned*>(smem)[i] = lo16 | (hi16 << 16);
  }
  __syncthreads();
  bf16x8 ah[2], al[2], bh[TN], bl[TN];
  auto read_a = [&](int x, int slot) {
    const int ra = wr * 128 + x * 16 + fr;
    ah[slot] = *reinterpret_cast<const bf16x8*>(smem + sw16_off(ra, fs));
    al[slot] = *reinterpret_cast<const bf16x8*>(smem + PLANE + sw16_off(ra, fs));
  };
  auto read_b = [&](int y) {
    const int rb = wc * 64 + y * 16 + fr;
    bh[y] = *reinterpret_cast<const bf16x8*>(smem + 2 * PLANE + sw16_off(rb, fs));
    bl[y] = *reinterpret_cast<const bf16x8*>(smem + 3 * PLANE + sw16_off(rb, fs));
  };
  f32x4 acc[TM][TN];
  for (int x = 0; x < TM; ++x)
    for (int y = 0; y < TN; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
  read_a(0, 0);
  read_a(1, 1);
  for (int y = 0; y < TN; ++y) read_b(y);
  for (int st = 0; st < stages; ++st) {
#pragma unroll
    for (int x = 0; x < TM; ++x) {
      if (MODE & 1) read_a((x + 1) % TM, (x + 1) & 1);
#pragma unroll
      for (int y = 0; y < TN; ++y) {
        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[x & 1], bh[y], acc[x][y], 0, 0, 0);
        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[x & 1], bl[y], acc[x][y], 0, 0, 0);
        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[x & 1], bh[y], acc[x][y], 0, 0, 0);
        if ((MODE & 2) && x == TM - 1) {
          __builtin_amdgcn_sched_barrier(0);
          read_b(y);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (MODE & 4) __builtin_amdgcn_s_barrier();
  }
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int x = 0; x < TM; ++x)
    for (int y = 0; y < TN; ++y) s += acc[x][y];
  out[blockIdx.x * 512 + tid] = s[0] + s[1] + s[2] + s[3];
}

}  // namespace

// LDS-fed MFMA loop (see mfma_lds_kernel); returns the floating-point operations issued.
extern "C" int64_t kge_probe_mfma_lds(int mode, int stages, float* out, int64_t out_elems, void* stream) {
  const int cus = num_cus();
  if (cus <= 0 || !out || stages <= 0 || out_elems < (int64_t)cus * 512) return 0;
  const size_t shmem = 4 * 256 * 64;
  void (*k)(int, float*) = nullptr;
  switch (mode) {
    case 0: k = mfma_lds_kernel<0>; break;
    case 1: k = mfma_lds_kernel<1>; break;
    case 2: k = mfma_lds_kernel<2>; break;
    case 3: k = mfma_lds_kernel<3>; break;
    case 7: k = mfma_lds_kernel<7>; break;
    default: return 0;
  }
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem) != hipSuccess) return 0;
  k<<<dim3(cus), dim3(512), shmem, (hipStream_t)stream>>>(stages, out);
  if (hipGetLastError() != hipSuccess) return 0;
  return (int64_t)cus * 8 * stages * 96 * (2LL * 16 * 16 * 32);
}

// Copies `bytes` (a multiple of 16) from src to dst; traffic = 2 * bytes.
extern "C" int kge_probe_copy(void* dst, const void* src, int64_t bytes, void* stream) {
  if (!dst || !src || bytes <= 0 || bytes % 16 != 0) return 1;
  const int cus = num_cus();
  if (cus <= 0) return 2;
  copy_kernel<<<dim3(cus * 8), dim3(256), 0, (hipStream_t)stream>>>((const float4*)src, (float4*)dst, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// One 512-thread workgroup per compute unit (two waves per SIMD), `iters` iterations of
// 2 * 8 MFMAs per wave.  out: cus * 512 floats.  Returns the floating-point operations issued
// (0 on error): cus * 8 waves * iters * 16 MFMAs * 2 * 16 * 16 * 32.
extern "C" int64_t kge_probe_mfma(int iters, int random, float* out, int64_t out_elems, void* stream) {
  const int cus = num_cus();
  if (cus <= 0 || !out || iters <= 0 || out_elems < (int64_t)cus * 512) return 0;
  mfma_kernel<<<dim3(cus), dim3(512), 0, (hipStream_t)stream>>>(iters, random, out);
  if (hipGetLastError() != hipSuccess) return 0;
  return (int64_t)cus * 8 * iters * (2 * ACCS) * (2LL * 16 * 16 * 32);
}

extern "C" int kge_probe_cus() { return num_cus(); }

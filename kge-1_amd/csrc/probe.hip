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

// Scalar-fp32 VALU probes (one 256-thread workgroup = one wave per SIMD; the grid puts
// `waves_per_simd` of them on every CU).  VARIANT 0: the L1-distance inner loop on registers
// only -- 8 x 8 accumulators, acc += |q - t| as v_sub_f32 + v_add_f32 with an |.| source
// modifier (128 instructions per iteration, + 16 that keep the operands changing);
// 1: 64 independent v_fma_f32 chains; 2: the L1 loop with its operands read from a resident LDS
// image the way the distance kernel reads them (4 ds_read_b128 per 128 VALU instructions);
// 3 / 4: the three-instruction L1 distance-backward update with the pair weight in an SGPR.
template <int VARIANT>
__global__ void __launch_bounds__(256) valu_kernel(int iters, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float img[2][16 * 132];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  for (int i = tid; i < 2 * 16 * 132; i += 256) (&img[0][0])[i] = (float)(mix(i + blockIdx.x) & 0xffff) * 1e-5f;
  __syncthreads();
  float acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = 0.f;
  if constexpr (VARIANT == 3 || VARIANT == 4) {
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 4; b < 8; ++b) {
        acc[a][b] = (float)(mix(tid * 64 + a * 8 + b) & 0xff) * 0.01f;
        asm volatile("" : "+v"(acc[a][b]));
      }
  }
  float q[8], t[8];
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    q[a] = (float)(mix(tid * 16 + a) & 0xff) * 0.01f;
    t[a] = (float)(mix(tid * 16 + 8 + a) & 0xff) * 0.01f;
  }
  const float eps = out[0] == 123.f ? 0.5f : 0.001f;  // not a compile-time constant
  for (int it = 0; it < iters; ++it) {
    if constexpr (VARIANT == 2) {
      const float* qb = &img[0][(it & 15) * 132];
      const float* tb = &img[1][(it & 15) * 132];
      const float4 q0 = *reinterpret_cast<const float4*>(qb + 4 * ty);
      const float4 q1 = *reinterpret_cast<const float4*>(qb + 64 + 4 * ty);
      const float4 t0 = *reinterpret_cast<const float4*>(tb + 4 * tx);
      const float4 t1 = *reinterpret_cast<const float4*>(tb + 64 + 4 * tx);
      q[0] = q0.x; q[1] = q0.y; q[2] = q0.z; q[3] = q0.w; q[4] = q1.x; q[5] = q1.y; q[6] = q1.z; q[7] = q1.w;
      t[0] = t0.x; t[1] = t0.y; t[2] = t0.z; t[3] = t0.w; t[4] = t1.x; t[5] = t1.y; t[6] = t1.z; t[7] = t1.w;
    }
    if constexpr (VARIANT == 3 || VARIANT == 4) {
      // the L1 distance-backward update: d = x - y, s = med3(d, -u, u), acc = fma(s, w, acc) with
      // the weight w in an SGPR; u in a VGPR (3) or an SGPR (4).  8 rows x 4 components x 2 y rows
      // per iteration = 192 instructions + 16 that keep the operands changing.  The 32 x values
      // live in acc[a][4 ..] / xv (distinct registers, opaque to the optimiser).
      float u = eps * 1e-10f;
      int wbits[8];
#pragma unroll
      for (int a = 0; a < 8; ++a) wbits[a] = __builtin_amdgcn_readfirstlane(__float_as_int(q[a]) + it);
      int ub = __builtin_amdgcn_readfirstlane(__float_as_int(u));
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            float dd;
            asm("v_sub_f32 %0, %1, %2" : "=v"(dd) : "v"(acc[a][4 + b]), "v"(t[4 * e + b]));
            float sg;
            if constexpr (VARIANT == 3) {
              asm("v_med3_f32 %0, %1, -%2, %2" : "=v"(sg) : "v"(dd), "v"(u));
            } else {
              asm("v_med3_f32 %0, %1, -%2, %2" : "=v"(sg) : "v"(dd), "s"(ub));
            }
            asm("v_fmac_f32 %0, %1, %2" : "+v"(acc[a][b]) : "s"(wbits[a]), "v"(sg));
          }
#pragma unroll
      for (int a = 0; a < 8; ++a) t[a] -= eps;
      continue;
    }
    if constexpr (VARIANT == 1) {
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = __builtin_fmaf(acc[a][b], q[a], t[b]);
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = __builtin_fmaf(acc[a][b], t[a], q[b]);
    } else {
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const float dd = q[a] - t[b];
          asm("v_add_f32 %0, %0, |%1|" : "+v"(acc[a][b]) : "v"(dd));
        }
    }
    if constexpr (VARIANT != 2) {
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        q[a] += eps;
        t[a] -= eps;
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) s += acc[a][b];
  out[1 + blockIdx.x * 256 + tid] = s;
}

// Issue cost of single VALU instruction forms: 32 independent destination registers, the same
// instruction 32 times per iteration, operands in registers (a: 32 VGPRs, b / c: VGPRs, s: SGPR).
#define KGE_OP_LOOP(STR)                                                            \
  for (int it = 0; it < iters; ++it) {                                              \
    _Pragma("unroll") for (int i = 0; i < 32; ++i)                                  \
        asm volatile(STR : "+v"(a[i]) : "v"(b[i & 7]), "v"(c[i & 3]), "s"(sv), "v"(a[(i + 5) & 31])); \
  }

template <int OP>
__global__ void __launch_bounds__(256) valu_op_kernel(int iters, float* __restrict__ out) {
  const int tid = threadIdx.x;
  float a[32], b[8], c[4];
#pragma unroll
  for (int i = 0; i < 32; ++i) a[i] = (float)(mix(tid * 64 + i) & 0xff) * 0.01f;
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = (float)(mix(tid * 8 + i) & 0xff) * 0.02f;
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = (float)(mix(tid * 4 + i) & 0xff) * 1e-3f;
  const int sv = __builtin_amdgcn_readfirstlane(__float_as_int(out[0] == 123.f ? 0.5f : 1.0001f));
  if constexpr (OP == 0) { KGE_OP_LOOP("v_sub_f32 %0, %1, %0") }
  if constexpr (OP == 1) { KGE_OP_LOOP("v_add_f32 %0, %0, |%1|") }
  if constexpr (OP == 2) { KGE_OP_LOOP("v_fma_f32 %0, %1, %2, %0") }
  if constexpr (OP == 3) { KGE_OP_LOOP("v_fmac_f32 %0, %1, %2") }
  if constexpr (OP == 4) { KGE_OP_LOOP("v_fmac_f32 %0, %3, %1") }
  if constexpr (OP == 5) { KGE_OP_LOOP("v_med3_f32 %0, %0, -%2, %2") }
  if constexpr (OP == 6) { KGE_OP_LOOP("v_med3_f32 %0, %0, -%3, %3") }
  if constexpr (OP == 7) { KGE_OP_LOOP("v_mul_f32 %0, %3, %0") }
  if constexpr (OP == 8) { KGE_OP_LOOP("v_sub_f32 %0, %3, %0") }
  if constexpr (OP == 9) { KGE_OP_LOOP("v_max_f32 %0, %1, %0") }
  if constexpr (OP == 10) { KGE_OP_LOOP("v_and_b32 %0, %1, %0") }
  if constexpr (OP == 11) { KGE_OP_LOOP("v_bfi_b32 %0, %3, %1, %0") }
  if constexpr (OP == 12) { KGE_OP_LOOP("v_sad_u32 %0, %1, %2, %0") }
  if constexpr (OP == 13) { KGE_OP_LOOP("v_cmp_lt_f32 vcc, %1, %0\n v_cndmask_b32 %0, %0, %2, vcc") }
  if constexpr (OP == 14) { KGE_OP_LOOP("v_mul_legacy_f32 %0, %1, %0") }
  if constexpr (OP == 15) { KGE_OP_LOOP("v_mul_f32 %0, %1, %0") }
  if constexpr (OP == 16) { KGE_OP_LOOP("v_add_f32 %0, %1, %0") }
  if constexpr (OP == 17) { KGE_OP_LOOP("v_sub_f32 %0, %1, %4") }
  if constexpr (OP == 18) { KGE_OP_LOOP("v_fma_f32 %0, %1, %3, %0") }
  if constexpr (OP == 19) { KGE_OP_LOOP("v_mul_f32 %0, 2.0, %0") }
  if constexpr (OP == 20) { KGE_OP_LOOP("v_med3_f32 %0, %0, -1.0, 1.0") }
  if constexpr (OP == 21) { KGE_OP_LOOP("v_xor_b32 %0, %3, %0") }
  if constexpr (OP == 22) { KGE_OP_LOOP("v_cmp_lt_f32 vcc, %1, %0") }
  if constexpr (OP == 23) { KGE_OP_LOOP("v_cndmask_b32 %0, %0, %2, vcc") }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) sum += a[i];
  out[1 + blockIdx.x * 256 + tid] = sum;
}

}  // namespace

// VALU probe (see valu_kernel); returns the vector instructions issued per lane times the lanes
// (lane-operations), 0 on error.  out: 1 + cus * waves_per_simd * 256 floats (out[0] is read).
extern "C" int64_t kge_probe_valu(int variant, int waves_per_simd, int iters, float* out, int64_t out_elems,
                                  void* stream) {
  const int cus = num_cus();
  if (cus <= 0 || !out || iters <= 0 || waves_per_simd < 1 || waves_per_simd > 8 ||
      out_elems < 1 + (int64_t)cus * waves_per_simd * 256)
    return 0;
  const dim3 grid(cus * waves_per_simd), block(256);
  switch (variant) {
    case 0: valu_kernel<0><<<grid, block, 0, (hipStream_t)stream>>>(iters, out); break;
    case 1: valu_kernel<1><<<grid, block, 0, (hipStream_t)stream>>>(iters, out); break;
    case 2: valu_kernel<2><<<grid, block, 0, (hipStream_t)stream>>>(iters, out); break;
    case 3: valu_kernel<3><<<grid, block, 0, (hipStream_t)stream>>>(iters, out); break;
    case 4: valu_kernel<4><<<grid, block, 0, (hipStream_t)stream>>>(iters, out); break;
    default: return 0;
  }
  if (hipGetLastError() != hipSuccess) return 0;
  const int64_t per_iter = variant == 0 ? 144 : variant >= 3 ? 200 : 128;
  return (int64_t)cus * waves_per_simd * 256 * iters * per_iter;
}

#include "probe_bank.inc"

// VGPR bank probe: the same instruction 32 times per iteration on explicit registers whose
// sources sit in different banks (register number mod 4) or in one bank.  The registers hold
// whatever the zero-initialising moves below leave (timing only).
template <int MODE>
__global__ void __launch_bounds__(256) valu_bank_kernel(int iters, float* __restrict__ out) {
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) asm volatile(KGE_BANK_FMA_FREE ::: KGE_BANK_CLOBBERS);
    if constexpr (MODE == 1) asm volatile(KGE_BANK_FMA_SAME ::: KGE_BANK_CLOBBERS);
    if constexpr (MODE == 2) asm volatile(KGE_BANK_SUB_FREE ::: KGE_BANK_CLOBBERS);
    if constexpr (MODE == 3) asm volatile(KGE_BANK_SUB_SAME ::: KGE_BANK_CLOBBERS);
    if constexpr (MODE == 4) asm volatile(KGE_BANK_FMA_TWO_SAME ::: KGE_BANK_CLOBBERS);
  }
  if (iters < 0) out[threadIdx.x] = 0.f;
}

extern "C" int64_t kge_probe_valu_bank(int mode, int waves_per_simd, int iters, float* out, int64_t out_elems,
                                       void* stream) {
  const int cus = num_cus();
  if (cus <= 0 || !out || iters <= 0 || waves_per_simd < 1 || waves_per_simd > 8 || out_elems < 256) return 0;
  const dim3 grid(cus * waves_per_simd), block(256);
  hipStream_t st = (hipStream_t)stream;
  switch (mode) {
    case 0: valu_bank_kernel<0><<<grid, block, 0, st>>>(iters, out); break;
    case 1: valu_bank_kernel<1><<<grid, block, 0, st>>>(iters, out); break;
    case 2: valu_bank_kernel<2><<<grid, block, 0, st>>>(iters, out); break;
    case 3: valu_bank_kernel<3><<<grid, block, 0, st>>>(iters, out); break;
    case 4: valu_bank_kernel<4><<<grid, block, 0, st>>>(iters, out); break;
    default: return 0;
  }
  if (hipGetLastError() != hipSuccess) return 0;
  return (int64_t)cus * waves_per_simd * 256 * iters * 32;
}

// Single-instruction VALU probe (see valu_op_kernel): returns the instructions issued per lane
// times the lanes (the two-instruction form 13 counts 2), 0 on error.
extern "C" int64_t kge_probe_valu_op(int op, int waves_per_simd, int iters, float* out, int64_t out_elems,
                                     void* stream) {
  const int cus = num_cus();
  if (cus <= 0 || !out || iters <= 0 || waves_per_simd < 1 || waves_per_simd > 8 ||
      out_elems < 1 + (int64_t)cus * waves_per_simd * 256)
    return 0;
  const dim3 grid(cus * waves_per_simd), block(256);
  hipStream_t st = (hipStream_t)stream;
  switch (op) {
#define KGE_OP_CASE(N) case N: valu_op_kernel<N><<<grid, block, 0, st>>>(iters, out); break;
    KGE_OP_CASE(0) KGE_OP_CASE(1) KGE_OP_CASE(2) KGE_OP_CASE(3) KGE_OP_CASE(4) KGE_OP_CASE(5) KGE_OP_CASE(6)
    KGE_OP_CASE(7) KGE_OP_CASE(8) KGE_OP_CASE(9) KGE_OP_CASE(10) KGE_OP_CASE(11) KGE_OP_CASE(12) KGE_OP_CASE(13)
    KGE_OP_CASE(14) KGE_OP_CASE(15) KGE_OP_CASE(16) KGE_OP_CASE(17) KGE_OP_CASE(18) KGE_OP_CASE(19) KGE_OP_CASE(20)
    KGE_OP_CASE(21) KGE_OP_CASE(22) KGE_OP_CASE(23)
#undef KGE_OP_CASE
    default: return 0;
  }
  if (hipGetLastError() != hipSuccess) return 0;
  return (int64_t)cus * waves_per_simd * 256 * iters * 32 * (op == 13 ? 2 : 1);
}

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

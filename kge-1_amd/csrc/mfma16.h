// Shared pieces of the bf16x3 MFMA kernels built on v_mfma_f32_16x16x32_bf16 (score_dot3.hip:
// the all-entities contraction; gemm_bwd3p.hip: its backward GEMMs on pre-split operand planes).
#pragma once
#include "common.h"

constexpr int KGE_BK = 32;  // K columns per stage: one 16x16x32 MFMA covers a whole stage

typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));  // 4-B-aligned float4
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// [row][k] bf16 image of a 32-wide K stage (64 B per row).  The 16x16x32 fragment reads
// (row = lane & 15, 16-B slot = lane >> 4) are conflict-free with the slot XOR-ed by
// g((row >> 2) & 3), g = {0, 2, 3, 1}: every ds_read_b128 lane group then covers 16 distinct
// 4-bank groups.
__device__ __forceinline__ int sw16_swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }
__device__ __forceinline__ int sw16_off(int row, int slot) { return row * 64 + ((slot ^ sw16_swz(row)) << 4); }

// VMEM issued from inline asm: hipcc neither counts nor waits for these, the kernel does
// (mixing LDS-DMA with compiler-visible register loads makes hipcc drain vmcnt to 0 at
// every use of a loaded register).  An asm register load's destination counts as written at
// the end of the statement, so every path from a load to the next use of its registers must
// pass a wait statement that names them ("+v") and retires the load: hipcc is otherwise free
// to reuse the registers (e.g. for an address) while the data is still in flight
// (checked on every build by tests/test_asm_audit.py).
__device__ __forceinline__ void glds16_asm(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
__device__ __forceinline__ u32x4 gload16_asm(const void* gsrc) {
  u32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(gsrc) : "memory");
  return r;
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

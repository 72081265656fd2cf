// Backward of the all-entities distance scores (TransE / RotatE), owner-computes form.
//
//   S[i, j] = sign * dist(Q[i], T[j])            (transe.py:19-21, rotate.py:41-60)
//   dQ[i, k] += sum_j W[i, j] * phi(Q[i, k] - T[j, k])
//   dT[j, k] += sum_i W[i, j] * phi(T[j, k] - Q[i, k])        (phi is odd for every kind)
// with W = sign * G for the L1 kinds and W = sign * G / dist for the L2 kinds, and
//   L1      phi(x) = sign(x)                      (0 at x = 0, like torch.sign)
//   L2      phi(x) = x
//   ROT_L1  phi(z) = z / |z|   per complex component (0 at z = 0)
//   ROT_L2  phi(z) = z
//
// Both gradients are the SAME kernel: "X rows own their gradient": a workgroup holds a
// 64-row x 64-component block of X in registers (4 x 4 per thread), streams the other operand's
// rows Y and the weights through LDS in chunks of 32 rows and accumulates in registers -- no
// pairwise tensor, no shared accumulators, no atomics inside the loop (the kernel this replaces
// reduced every pair into LDS with atomic adds and ran 30x slower than the forward).  dQ is
// X = Q, Y = T; dT is X = T, Y = Q with the weights read transposed.  When X has few rows the
// Y range is split over blockIdx.z; every launch ends in one atomic add per owned element (the
// interface accumulates into dq / dt, and candidate row maps may repeat a row).
#include "common.h"

namespace {

constexpr int XT = 64;   // X rows per workgroup
constexpr int KT = 64;   // components per workgroup (complex components for the RotatE kinds)
constexpr int YC = 32;   // Y rows per LDS chunk
constexpr int NT = 256;
constexpr int LD = KT + 4;  // padded LDS rows (floats)

template <int KIND>
struct Phi {
  static constexpr bool ROT = KIND >= KGE_DIST_ROT_L1;
};

// acc += w * phi(x - y) for one real component
template <int KIND>
__device__ __forceinline__ void pair_real(float& acc, float w, float x, float y) {
  const float d = x - y;
  if (KIND == KGE_DIST_L1) {
    // sign(d): +-1, and exactly 0 at d == 0 (d * 2^126 never underflows to 0 for d != 0)
    const float s = __builtin_amdgcn_fmed3f(d * 8.507059173023462e37f, -1.0f, 1.0f);
    acc = fmaf(w, s, acc);
  } else {
    acc = fmaf(w, d, acc);
  }
}

// (acc_re, acc_im) += w * phi(x - y) for one complex component
template <int KIND>
__device__ __forceinline__ void pair_cplx(float& are, float& aim, float w, float xr, float xi, float yr, float yi) {
  const float dr = xr - yr, di = xi - yi;
  if (KIND == KGE_DIST_ROT_L1) {
    const float sq = fmaf(di, di, dr * dr);
    const float f = sq > 0.f ? w * __builtin_amdgcn_rsqf(sq) : 0.f;
    are = fmaf(f, dr, are);
    aim = fmaf(f, di, aim);
  } else {
    are = fmaf(w, dr, are);
    aim = fmaf(w, di, aim);
  }
}

// WT false: weight of (x, y) = w[x * ldw + y]   (X = queries:  W rows)
// WT true : weight of (x, y) = w[y * ldw + x]   (X = entities: W columns)
template <int KIND, bool WT>
__global__ void __launch_bounds__(NT) dist_bwd_own_kernel(float scale, const float* __restrict__ w, int64_t ldw,
                                                          const float* __restrict__ x, int64_t ldx,
                                                          const int64_t* __restrict__ xmap, int nx,
                                                          const float* __restrict__ y, int64_t ldy,
                                                          const int64_t* __restrict__ ymap, int ny, int kdim, int h,
                                                          float* __restrict__ out, int64_t ldo, int ychunks_per_z) {
  constexpr bool ROT = Phi<KIND>::ROT;
  __shared__ __attribute__((aligned(16))) float ys_re[YC * LD];
  __shared__ __attribute__((aligned(16))) float ys_im[ROT ? YC * LD : 4];
  __shared__ __attribute__((aligned(16))) float ws[YC * LD];
  const int tid = threadIdx.x;
  const int tk = tid & 15, tx = tid >> 4;
  const int x0 = blockIdx.x * XT, k0 = blockIdx.y * KT;
  const int kb = k0 + 4 * tk;  // this thread's four components (all in or all out: kdim % 4 == 0)
  const bool k_in = kb < kdim;

  // this thread's 4 x 4 block of X
  float xr[4][4], xi[4][4];
  int64_t xrow[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int gx = x0 + 4 * tx + a;
    const int gxc = min(gx, nx - 1);
    xrow[a] = xmap ? xmap[gxc] : (int64_t)gxc;
    float4 vr = make_float4(0.f, 0.f, 0.f, 0.f), vi = vr;
    if (k_in) {
      vr = *reinterpret_cast<const float4*>(x + xrow[a] * ldx + kb);
      if (ROT) vi = *reinterpret_cast<const float4*>(x + xrow[a] * ldx + kb + h);
    }
    xr[a][0] = vr.x, xr[a][1] = vr.y, xr[a][2] = vr.z, xr[a][3] = vr.w;
    xi[a][0] = vi.x, xi[a][1] = vi.y, xi[a][2] = vi.z, xi[a][3] = vi.w;
  }
  float are[4][4], aim[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) are[a][c] = 0.f, aim[a][c] = 0.f;

  const int c_begin = blockIdx.z * ychunks_per_z;
  const int c_end = min(c_begin + ychunks_per_z, (ny + YC - 1) / YC);
  for (int ch = c_begin; ch < c_end; ++ch) {
    const int y0 = ch * YC;
    // Y chunk: YC rows x KT components -> ys[yy][k]; 16 float4 per row (and plane), 2 rows per pass
#pragma unroll
    for (int p = 0; p < YC * 16 / NT; ++p) {
      const int f = p * NT + tid;
      const int yy = f >> 4, kq = (f & 15) * 4;
      const int gy = y0 + yy, gk = k0 + kq;
      float4 vr = make_float4(0.f, 0.f, 0.f, 0.f), vi = vr;
      if (gy < ny && gk < kdim) {
        const int64_t row = ymap ? ymap[gy] : (int64_t)gy;
        vr = *reinterpret_cast<const float4*>(y + row * ldy + gk);
        if (ROT) vi = *reinterpret_cast<const float4*>(y + row * ldy + gk + h);
      }
      *reinterpret_cast<float4*>(ys_re + yy * LD + kq) = vr;
      if (ROT) *reinterpret_cast<float4*>(ys_im + yy * LD + kq) = vi;
    }
    // weights of (X rows x0 .. x0 + 63) x (Y rows y0 .. y0 + 31) -> ws[yy][xx], scaled; pairs
    // outside the matrix weigh 0
    if (WT) {  // rows of w are Y rows: 64 consecutive floats each
#pragma unroll
      for (int p = 0; p < YC * XT / NT; ++p) {
        const int f = p * NT + tid;
        const int yy = f >> 6, xx = f & 63;
        const int gy = y0 + yy, gx = x0 + xx;
        ws[yy * LD + xx] = (gy < ny && gx < nx) ? scale * w[(int64_t)gy * ldw + gx] : 0.f;
      }
    } else {  // rows of w are X rows: 32 consecutive floats each
#pragma unroll
      for (int p = 0; p < YC * XT / NT; ++p) {
        const int f = p * NT + tid;
        const int xx = f >> 5, yy = f & 31;
        const int gy = y0 + yy, gx = x0 + xx;
        ws[yy * LD + xx] = (gy < ny && gx < nx) ? scale * w[(int64_t)gx * ldw + gy] : 0.f;
      }
    }
    __syncthreads();
    if (k_in) {
#pragma unroll 2
      for (int yy = 0; yy < YC; ++yy) {
        const float4 wv = *reinterpret_cast<const float4*>(ws + yy * LD + 4 * tx);
        const float4 yr4 = *reinterpret_cast<const float4*>(ys_re + yy * LD + 4 * tk);
        const float wa[4] = {wv.x, wv.y, wv.z, wv.w};
        const float yr[4] = {yr4.x, yr4.y, yr4.z, yr4.w};
        if (ROT) {
          const float4 yi4 = *reinterpret_cast<const float4*>(ys_im + yy * LD + 4 * tk);
          const float yi[4] = {yi4.x, yi4.y, yi4.z, yi4.w};
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) pair_cplx<KIND>(are[a][c], aim[a][c], wa[a], xr[a][c], xi[a][c], yr[c], yi[c]);
        } else {
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) pair_real<KIND>(are[a][c], wa[a], xr[a][c], yr[c]);
        }
      }
    }
    __syncthreads();
  }
  if (!k_in) return;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    if (x0 + 4 * tx + a >= nx) continue;
    float* o = out + xrow[a] * ldo + kb;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      atomicAdd(o + c, are[a][c]);
      if (ROT) atomicAdd(o + h + c, aim[a][c]);
    }
  }
}

template <int KIND, bool WT>
int launch_own(float scale, const float* w, int64_t ldw, const float* x, int64_t ldx, const int64_t* xmap, int64_t nx,
               const float* y, int64_t ldy, const int64_t* ymap, int64_t ny, int kdim, int h, float* out, int64_t ldo,
               hipStream_t st) {
  const int64_t xt = (nx + XT - 1) / XT, kt = (kdim + KT - 1) / KT;
  const int64_t chunks = (ny + YC - 1) / YC;
  // enough workgroups for every CU several times over; at least 8 chunks per workgroup
  const int64_t want = 4LL * kge_num_cus();
  int64_t z = std::max<int64_t>(1, std::min<int64_t>((want + xt * kt - 1) / (xt * kt), chunks / 8));
  z = std::min<int64_t>(z, 65535);
  const int64_t per_z = (chunks + z - 1) / z;
  z = (chunks + per_z - 1) / per_z;
  if (xt > 0x7fffffff || kt > 65535) return -1;
  dim3 grid((unsigned)xt, (unsigned)kt, (unsigned)z);
  dist_bwd_own_kernel<KIND, WT><<<grid, NT, 0, st>>>(scale, w, ldw, x, ldx, xmap, (int)nx, y, ldy, ymap, (int)ny, kdim, h,
                                                     out, ldo, (int)per_z);
  return 0;
}

template <int KIND>
int run_kind(float scale, const float* w, int64_t ldw, const float* q, int64_t ldq, const float* t, int64_t ldt,
             const int64_t* tidx, int64_t n, int64_t m, int kdim, int h, float* dq, int64_t lddq, float* dt,
             int64_t lddt, hipStream_t st) {
  if (dq) {
    const int r = launch_own<KIND, false>(scale, w, ldw, q, ldq, nullptr, n, t, ldt, tidx, m, kdim, h, dq, lddq, st);
    if (r) return r;
  }
  if (dt) {
    const int r = launch_own<KIND, true>(scale, w, ldw, t, ldt, tidx, m, q, ldq, nullptr, n, kdim, h, dt, lddt, st);
    if (r) return r;
  }
  return 0;
}

}  // namespace

// dq += / dt += from ready pair weights w (see the header of this file); -1 when the layout
// does not fit (rows that float4 loads cannot read): the caller then uses the generic kernel.
int kge_score_dist_bwd_own(int kind, float scale, const float* w, int64_t ldw, const float* q, int64_t ldq,
                           const float* t, int64_t ldt, const int64_t* tidx, int64_t n, int64_t m, int d, float* dq,
                           int64_t lddq, float* dt, int64_t lddt, hipStream_t st) {
  const bool rot = kind >= KGE_DIST_ROT_L1;
  const int kdim = rot ? d / 2 : d, h = d / 2;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (kdim % 4 != 0 || (rot && h % 4 != 0) || ldq % 4 != 0 || ldt % 4 != 0 || !al16(q) || !al16(t)) return -1;
  if (n <= 0 || m <= 0) return 0;
  switch (kind) {
    case KGE_DIST_L1: return run_kind<KGE_DIST_L1>(scale, w, ldw, q, ldq, t, ldt, tidx, n, m, kdim, h, dq, lddq, dt, lddt, st);
    case KGE_DIST_L2: return run_kind<KGE_DIST_L2>(scale, w, ldw, q, ldq, t, ldt, tidx, n, m, kdim, h, dq, lddq, dt, lddt, st);
    case KGE_DIST_ROT_L1: return run_kind<KGE_DIST_ROT_L1>(scale, w, ldw, q, ldq, t, ldt, tidx, n, m, kdim, h, dq, lddq, dt, lddt, st);
    default: return run_kind<KGE_DIST_ROT_L2>(scale, w, ldw, q, ldq, t, ldt, tidx, n, m, kdim, h, dq, lddq, dt, lddt, st);
  }
}

extern "C" int kge_score_dist_bwd_weighted(int kind, const float* w, int64_t ldw, const float* q, int64_t ldq,
                                           const float* t, int64_t ldt, const int64_t* tidx, int64_t n, int64_t m,
                                           int d, float* dq, int64_t lddq, float* dt, int64_t lddt, void* stream) {
  KGE_REQUIRE(n >= 0 && m >= 0 && d > 0 && n < (1LL << 31) && m < (1LL << 31));
  KGE_REQUIRE(w && q && t && ldw >= m && ldq >= d && ldt >= d);
  KGE_REQUIRE(kind >= KGE_DIST_L1 && kind <= KGE_DIST_ROT_L2);
  KGE_REQUIRE(kind < KGE_DIST_ROT_L1 || d % 2 == 0);
  if (n == 0 || m == 0 || (!dq && !dt)) return 0;
  const int r = kge_score_dist_bwd_own(kind, 1.0f, w, ldw, q, ldq, t, ldt, tidx, n, m, d, dq, lddq, dt, lddt,
                                       as_stream(stream));
  if (r < 0) return KGE_ERR_ALIGN;
  if (r == 0) KGE_CHECK_LAUNCH();
  return r;
}

// Query preparation (fused LookupEmbedder gather + per-model prologue) and its backward.
//
// Every in-scope scorer reduces to "per-query prep + one contraction (dot or distance)
// against the entity table".  These kernels produce the query
// rows Q[n, d_e]; they are small (n * d work) next to the contraction.
#include "common.h"

namespace {

struct Rows {
  const float* e;
  const float* r;
};

__device__ __forceinline__ Rows fetch_rows(const float* ent, int64_t ld_ent, const int64_t* eidx,
                                           const float* rel, int64_t ld_rel, const int64_t* ridx,
                                           int64_t i) {
  const int64_t ei = eidx ? eidx[i] : i;
  const int64_t ri = ridx ? ridx[i] : i;
  return Rows{ent + ei * ld_ent, rel + ri * ld_rel};
}

// Query-row sink: fp32 rows and/or bf16 hi / lo planes (the bf16x3 contraction's input),
// planes zero-padded from the query width up to padw columns (the K padding the contraction
// reads: the width rounded up to 32, or the whole row when it is shorter than that).
struct QOut {
  float* q;
  int64_t ldq;
  __bf16* hi;
  __bf16* lo;
  int64_t ldp;
  int padw;
  // optional: band[i] = band_rel * |q_i|_2 * tmax[0] (the refinement band of an evaluation row,
  // kge_rank_band) written by the vectorised kernel, whose wave holds the whole row anyway
  float* band = nullptr;
  float band_rel = 0.f;
  const float* tmax = nullptr;
  __device__ __forceinline__ void put(int64_t i, int k, float v) const {
    if (q) q[i * ldq + k] = v;
    if (hi) {
      __bf16 h, l;
      split_bf16(v, h, l);
      hi[i * ldp + k] = h;
      lo[i * ldp + k] = l;
    }
  }
  __device__ __forceinline__ void pad(int64_t i, int d) const {
    if (!hi) return;
    for (int k = d + threadIdx.x; k < padw; k += blockDim.x) {
      hi[i * ldp + k] = (__bf16)0.f;
      lo[i * ldp + k] = (__bf16)0.f;
    }
  }
};

// Direction of query row i: rows [0, n_a) take direction a, the rest direction b (the stacked
// sp_ / _po query batches of a training step or an evaluation batch in ONE launch).  n_a may
// live in device memory (n_a_dev != null), so that a recorded launch serves batches whose
// split differs.
struct Dirs {
  int a, b;
  int64_t n_a;
  const int64_t* n_a_dev;
  __device__ __forceinline__ int of(int64_t i) const { return i < (n_a_dev ? *n_a_dev : n_a) ? a : b; }
};

// Elementwise models: complex / distmult / transe / rotate.  One block per query row.
template <int MODEL, int DIR>
__device__ __forceinline__ void prep_row(const Rows rw, int64_t i, int d_e, const QOut& out) {
  out.pad(i, MODEL == KGE_CP ? d_e / 2 : d_e);
  if (MODEL == KGE_CP) {  // s_h * r (sp) / o_t * r (po), d_e / 2 columns
    const int h = d_e / 2;
    const float* e = rw.e + (DIR == KGE_DIR_SP ? 0 : h);
    for (int k = threadIdx.x; k < h; k += blockDim.x) out.put(i, k, e[k] * rw.r[k]);
  } else if (MODEL == KGE_SIMPLE) {  // q[j] = e[j'] r[j'] / 2 (sp), e[j'] r[j] / 2 (po), j' = other half
    const int h = d_e / 2;
    for (int j = threadIdx.x; j < d_e; j += blockDim.x) {
      const int jp = j < h ? j + h : j - h;
      out.put(i, j, 0.5f * rw.e[jp] * rw.r[DIR == KGE_DIR_SP ? jp : j]);
    }
  } else if (MODEL == KGE_COMPLEX || MODEL == KGE_ROTATE) {
    const int h = d_e / 2;
    for (int k = threadIdx.x; k < h; k += blockDim.x) {
      const float a_re = rw.e[k], a_im = rw.e[k + h];
      float c, s;
      if (MODEL == KGE_COMPLEX) {
        c = rw.r[k];
        s = rw.r[k + h];
      } else {
        sincosf(rw.r[k], &s, &c);  // rotate.py:26 (radians -> unit complex)
      }
      if (DIR == KGE_DIR_SP) {  // a * (c + i s)
        out.put(i, k, a_re * c - a_im * s);
        out.put(i, k + h, a_re * s + a_im * c);
      } else {  // conj(c + i s) * a
        out.put(i, k, c * a_re + s * a_im);
        out.put(i, k + h, c * a_im - s * a_re);
      }
    }
  } else {
    for (int k = threadIdx.x; k < d_e; k += blockDim.x) {
      const float a = rw.e[k], b = rw.r[k];
      if (MODEL == KGE_DISTMULT)
        out.put(i, k, a * b);
      else  // TRANSE
        out.put(i, k, (DIR == KGE_DIR_SP) ? a + b : a - b);
    }
  }
}

template <int MODEL>
__global__ void __launch_bounds__(256) prep_elementwise(const float* __restrict__ ent, int64_t ld_ent,
                                                         const int64_t* __restrict__ eidx,
                                                         const float* __restrict__ rel, int64_t ld_rel,
                                                         const int64_t* __restrict__ ridx, int d_e, QOut out,
                                                         Dirs dirs) {
  const int64_t i = blockIdx.x;
  const Rows rw = fetch_rows(ent, ld_ent, eidx, rel, ld_rel, ridx, i);
  if (dirs.of(i) == KGE_DIR_SP)
    prep_row<MODEL, KGE_DIR_SP>(rw, i, d_e, out);
  else
    prep_row<MODEL, KGE_DIR_PO>(rw, i, d_e, out);
}

// Vectorised elementwise prep: one wave per query row, 4 consecutive elements (complex
// positions for ComplEx / RotatE) per lane per step, float4 loads, float4 / bf16x4 stores.
// Needs d_e % 8 == 0 (complex halves % 4) and 16-B aligned rows (checked by the launcher).
template <int MODEL, int DIR>
__device__ __forceinline__ void prep_row_vec(const Rows rw, int64_t i, int lane, int d_e, const QOut& out) {
  float ss = 0.f;  // this lane's share of |q_i|^2
  auto put4 = [&](int k, float4 v) {
    ss = fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, fmaf(v.w, v.w, ss))));
    if (out.q) *reinterpret_cast<float4*>(out.q + i * out.ldq + k) = v;
    if (out.hi) {
      bf16x4 h, l;
      split_bf16x4_pk(v, h, l);
      *reinterpret_cast<bf16x4*>(out.hi + i * out.ldp + k) = h;
      *reinterpret_cast<bf16x4*>(out.lo + i * out.ldp + k) = l;
    }
  };
  const int qw = MODEL == KGE_CP ? d_e / 2 : d_e;
  if (out.hi)
    for (int k = qw + lane * 4; k < out.padw; k += 256) {  // zero K padding (padw % 4 == 0)
      *reinterpret_cast<bf16x4*>(out.hi + i * out.ldp + k) = bf16x4{};
      *reinterpret_cast<bf16x4*>(out.lo + i * out.ldp + k) = bf16x4{};
    }
  auto mul4 = [](float4 a, float4 b, float c) {
    return make_float4(c * a.x * b.x, c * a.y * b.y, c * a.z * b.z, c * a.w * b.w);
  };
  if (MODEL == KGE_CP) {
    const int h = d_e / 2;
    const float* e = rw.e + (DIR == KGE_DIR_SP ? 0 : h);
    for (int k = lane * 4; k < h; k += 256)
      put4(k, mul4(*reinterpret_cast<const float4*>(e + k), *reinterpret_cast<const float4*>(rw.r + k), 1.f));
  } else if (MODEL == KGE_SIMPLE) {
    const int h = d_e / 2;
    for (int k = lane * 4; k < h; k += 256) {
      const float4 e0 = *reinterpret_cast<const float4*>(rw.e + k), e1 = *reinterpret_cast<const float4*>(rw.e + k + h);
      const float4 r0 = *reinterpret_cast<const float4*>(rw.r + k), r1 = *reinterpret_cast<const float4*>(rw.r + k + h);
      put4(k, mul4(e1, DIR == KGE_DIR_SP ? r1 : r0, 0.5f));
      put4(k + h, mul4(e0, DIR == KGE_DIR_SP ? r0 : r1, 0.5f));
    }
  } else if (MODEL == KGE_COMPLEX || MODEL == KGE_ROTATE) {
    const int h = d_e / 2;
    for (int k = lane * 4; k < h; k += 256) {
      const float4 ar = *reinterpret_cast<const float4*>(rw.e + k), ai = *reinterpret_cast<const float4*>(rw.e + k + h);
      float4 c, s;
      if (MODEL == KGE_COMPLEX) {
        c = *reinterpret_cast<const float4*>(rw.r + k);
        s = *reinterpret_cast<const float4*>(rw.r + k + h);
      } else {
        const float4 ph = *reinterpret_cast<const float4*>(rw.r + k);  // rotate.py:26
        sincosf(ph.x, &s.x, &c.x);
        sincosf(ph.y, &s.y, &c.y);
        sincosf(ph.z, &s.z, &c.z);
        sincosf(ph.w, &s.w, &c.w);
      }
      float4 re, im;
      if (DIR == KGE_DIR_SP) {  // a * (c + i s)
        re = make_float4(ar.x * c.x - ai.x * s.x, ar.y * c.y - ai.y * s.y, ar.z * c.z - ai.z * s.z, ar.w * c.w - ai.w * s.w);
        im = make_float4(ar.x * s.x + ai.x * c.x, ar.y * s.y + ai.y * c.y, ar.z * s.z + ai.z * c.z, ar.w * s.w + ai.w * c.w);
      } else {  // conj(c + i s) * a
        re = make_float4(c.x * ar.x + s.x * ai.x, c.y * ar.y + s.y * ai.y, c.z * ar.z + s.z * ai.z, c.w * ar.w + s.w * ai.w);
        im = make_float4(c.x * ai.x - s.x * ar.x, c.y * ai.y - s.y * ar.y, c.z * ai.z - s.z * ar.z, c.w * ai.w - s.w * ar.w);
      }
      put4(k, re);
      put4(k + h, im);
    }
  } else {
    for (int k = lane * 4; k < d_e; k += 256) {
      const float4 a = *reinterpret_cast<const float4*>(rw.e + k), b = *reinterpret_cast<const float4*>(rw.r + k);
      float4 v;
      if (MODEL == KGE_DISTMULT)
        v = make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
      else if (DIR == KGE_DIR_SP)  // TRANSE
        v = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
      else
        v = make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
      put4(k, v);
    }
  }
  if (out.band) {
    ss = wave_sum(ss);
    // a hair wider than a band computed in another summation order: never narrower than the bound
    if (lane == 0) out.band[i] = out.band_rel * sqrtf(ss) * out.tmax[0] * 1.000001f;
  }
}

template <int MODEL>
__global__ void __launch_bounds__(256) prep_elementwise_vec(const float* __restrict__ ent, int64_t ld_ent,
                                                             const int64_t* __restrict__ eidx,
                                                             const float* __restrict__ rel, int64_t ld_rel,
                                                             const int64_t* __restrict__ ridx, int64_t n, int d_e,
                                                             QOut out, Dirs dirs) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int lane = threadIdx.x & 63;
  const Rows rw = fetch_rows(ent, ld_ent, eidx, rel, ld_rel, ridx, i);
  if (dirs.of(i) == KGE_DIR_SP)  // wave-uniform
    prep_row_vec<MODEL, KGE_DIR_SP>(rw, i, lane, d_e, out);
  else
    prep_row_vec<MODEL, KGE_DIR_PO>(rw, i, lane, d_e, out);
}

// RESCAL: Q = s^T M (sp) or M o (po), M = rel row viewed as [d, d] row-major.
template <int DIR>
__device__ __forceinline__ void prep_rescal_row(const Rows rw, int64_t i, int d, const QOut& out, float* xs) {
  for (int k = threadIdx.x; k < d; k += blockDim.x) xs[k] = rw.e[k];
  out.pad(i, d);
  __syncthreads();
  if (DIR == KGE_DIR_SP) {  // q_j = sum_a x_a M[a][j]  (coalesced over j)
    for (int j = threadIdx.x; j < d; j += blockDim.x) {
      float acc = 0.f;
      for (int a = 0; a < d; ++a) acc = fmaf(xs[a], rw.r[(int64_t)a * d + j], acc);
      out.put(i, j, acc);
    }
  } else {  // q_a = sum_j M[a][j] x_j : one wave per output row
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int a = wave; a < d; a += nw) {
      float acc = 0.f;
      for (int j = lane; j < d; j += 64) acc = fmaf(rw.r[(int64_t)a * d + j], xs[j], acc);
      acc = wave_sum(acc);
      if (lane == 0) out.put(i, a, acc);
    }
  }
}

__global__ void __launch_bounds__(256) prep_rescal(const float* __restrict__ ent, int64_t ld_ent,
                                                    const int64_t* __restrict__ eidx,
                                                    const float* __restrict__ rel, int64_t ld_rel,
                                                    const int64_t* __restrict__ ridx, int d, QOut out, Dirs dirs) {
  extern __shared__ float xs[];
  const int64_t i = blockIdx.x;
  const Rows rw = fetch_rows(ent, ld_ent, eidx, rel, ld_rel, ridx, i);
  if (dirs.of(i) == KGE_DIR_SP)  // block-uniform: the barrier inside is reached by every thread
    prep_rescal_row<KGE_DIR_SP>(rw, i, d, out, xs);
  else
    prep_rescal_row<KGE_DIR_PO>(rw, i, d, out, xs);
}

// ---------------------------------------------------------------------- backward
__device__ __forceinline__ void atomic_add_row(float* base, int k, float v) {
  if (base) atomicAdd(base + k, v);
}

template <int MODEL, int DIR>
__device__ __forceinline__ void prep_row_bwd(const Rows rw, int d_e, const float* __restrict__ g, float* ge,
                                             float* gr) {
  if (MODEL == KGE_CP) {
    const int h = d_e / 2, off = DIR == KGE_DIR_SP ? 0 : h;
    for (int k = threadIdx.x; k < h; k += blockDim.x) {
      atomic_add_row(ge, k + off, g[k] * rw.r[k]);
      atomic_add_row(gr, k, g[k] * rw.e[k + off]);
    }
  } else if (MODEL == KGE_SIMPLE) {
    const int h = d_e / 2;
    for (int j = threadIdx.x; j < d_e; j += blockDim.x) {
      const int jp = j < h ? j + h : j - h, jr = DIR == KGE_DIR_SP ? jp : j;
      atomic_add_row(ge, jp, 0.5f * g[j] * rw.r[jr]);
      atomic_add_row(gr, jr, 0.5f * g[j] * rw.e[jp]);
    }
  } else if (MODEL == KGE_COMPLEX) {
    const int h = d_e / 2;
    for (int k = threadIdx.x; k < h; k += blockDim.x) {
      const float a_re = rw.e[k], a_im = rw.e[k + h], r_re = rw.r[k], r_im = rw.r[k + h];
      const float g_re = g[k], g_im = g[k + h];
      if (DIR == KGE_DIR_SP) {  // q = a*r: da = g*conj(r), dr = g*conj(a)
        atomic_add_row(ge, k, g_re * r_re + g_im * r_im);
        atomic_add_row(ge, k + h, g_im * r_re - g_re * r_im);
        atomic_add_row(gr, k, g_re * a_re + g_im * a_im);
        atomic_add_row(gr, k + h, g_im * a_re - g_re * a_im);
      } else {  // q = conj(r)*a: da = g*r, dr = conj(g)*a
        atomic_add_row(ge, k, g_re * r_re - g_im * r_im);
        atomic_add_row(ge, k + h, g_re * r_im + g_im * r_re);
        atomic_add_row(gr, k, g_re * a_re + g_im * a_im);
        atomic_add_row(gr, k + h, g_re * a_im - g_im * a_re);
      }
    }
  } else if (MODEL == KGE_ROTATE) {
    const int h = d_e / 2;
    for (int k = threadIdx.x; k < h; k += blockDim.x) {
      const float a_re = rw.e[k], a_im = rw.e[k + h];
      float c, s;
      sincosf(rw.r[k], &s, &c);
      const float g_re = g[k], g_im = g[k + h];
      if (DIR == KGE_DIR_SP) {  // q = a*rot: da = g*conj(rot), dtheta = g_re(-q_im) + g_im q_re
        const float q_re = a_re * c - a_im * s, q_im = a_re * s + a_im * c;
        atomic_add_row(ge, k, g_re * c + g_im * s);
        atomic_add_row(ge, k + h, g_im * c - g_re * s);
        atomic_add_row(gr, k, g_im * q_re - g_re * q_im);
      } else {  // q = a*conj(rot): da = g*rot, dtheta = g_re q_im - g_im q_re
        const float q_re = c * a_re + s * a_im, q_im = c * a_im - s * a_re;
        atomic_add_row(ge, k, g_re * c - g_im * s);
        atomic_add_row(ge, k + h, g_re * s + g_im * c);
        atomic_add_row(gr, k, g_re * q_im - g_im * q_re);
      }
    }
  } else {
    for (int k = threadIdx.x; k < d_e; k += blockDim.x) {
      const float a = rw.e[k], b = rw.r[k], gk = g[k];
      if (MODEL == KGE_DISTMULT) {
        atomic_add_row(ge, k, gk * b);
        atomic_add_row(gr, k, gk * a);
      } else {  // TRANSE: q = a + b (sp) / a - b (po)
        atomic_add_row(ge, k, gk);
        atomic_add_row(gr, k, DIR == KGE_DIR_SP ? gk : -gk);
      }
    }
  }
}

template <int MODEL>
__global__ void __launch_bounds__(256) prep_elementwise_bwd(
    const float* __restrict__ ent, int64_t ld_ent, const int64_t* __restrict__ eidx,
    const float* __restrict__ rel, int64_t ld_rel, const int64_t* __restrict__ ridx, int d_e,
    const float* __restrict__ dq, int64_t lddq, float* d_ent, int64_t ld_dent, float* d_rel,
    int64_t ld_drel, Dirs dirs) {
  const int64_t i = blockIdx.x;
  const Rows rw = fetch_rows(ent, ld_ent, eidx, rel, ld_rel, ridx, i);
  const float* g = dq + i * lddq;
  float* ge = d_ent ? d_ent + (eidx ? eidx[i] : i) * ld_dent : nullptr;
  float* gr = d_rel ? d_rel + (ridx ? ridx[i] : i) * ld_drel : nullptr;
  if (dirs.of(i) == KGE_DIR_SP)
    prep_row_bwd<MODEL, KGE_DIR_SP>(rw, d_e, g, ge, gr);
  else
    prep_row_bwd<MODEL, KGE_DIR_PO>(rw, d_e, g, ge, gr);
}

template <int DIR>
__device__ __forceinline__ void prep_rescal_row_bwd(const Rows rw, int d, const float* xs, const float* gs, float* ge,
                                                    float* gr) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // dM[a][b] = x_a g_b (sp) or g_a x_b (po)
  if (gr) {
    for (int64_t t = threadIdx.x; t < (int64_t)d * d; t += blockDim.x) {
      const int a = (int)(t / d), b = (int)(t % d);
      atomicAdd(gr + t, DIR == KGE_DIR_SP ? xs[a] * gs[b] : gs[a] * xs[b]);
    }
  }
  if (ge) {
    if (DIR == KGE_DIR_SP) {  // dx_a = sum_b M[a][b] g_b
      for (int a = wave; a < d; a += nw) {
        float acc = 0.f;
        for (int b = lane; b < d; b += 64) acc = fmaf(rw.r[(int64_t)a * d + b], gs[b], acc);
        acc = wave_sum(acc);
        if (lane == 0) atomicAdd(ge + a, acc);
      }
    } else {  // dx_b = sum_a M[a][b] g_a
      for (int b = threadIdx.x; b < d; b += blockDim.x) {
        float acc = 0.f;
        for (int a = 0; a < d; ++a) acc = fmaf(rw.r[(int64_t)a * d + b], gs[a], acc);
        atomicAdd(ge + b, acc);
      }
    }
  }
}

__global__ void __launch_bounds__(256) prep_rescal_bwd(
    const float* __restrict__ ent, int64_t ld_ent, const int64_t* __restrict__ eidx,
    const float* __restrict__ rel, int64_t ld_rel, const int64_t* __restrict__ ridx, int d,
    const float* __restrict__ dq, int64_t lddq, float* d_ent, int64_t ld_dent, float* d_rel,
    int64_t ld_drel, Dirs dirs) {
  extern __shared__ float sm[];
  float* xs = sm;      // entity row
  float* gs = sm + d;  // dq row
  const int64_t i = blockIdx.x;
  const Rows rw = fetch_rows(ent, ld_ent, eidx, rel, ld_rel, ridx, i);
  for (int k = threadIdx.x; k < d; k += blockDim.x) {
    xs[k] = rw.e[k];
    gs[k] = dq[i * lddq + k];
  }
  __syncthreads();
  float* ge = d_ent ? d_ent + (eidx ? eidx[i] : i) * ld_dent : nullptr;
  float* gr = d_rel ? d_rel + (ridx ? ridx[i] : i) * ld_drel : nullptr;
  if (dirs.of(i) == KGE_DIR_SP)
    prep_rescal_row_bwd<KGE_DIR_SP>(rw, d, xs, gs, ge, gr);
  else
    prep_rescal_row_bwd<KGE_DIR_PO>(rw, d, xs, gs, ge, gr);
}

int launch_prep(int model, const float* ent, int64_t ld_ent, const int64_t* eidx, const float* rel,
                int64_t ld_rel, const int64_t* ridx, int64_t n, int d_e, QOut q, Dirs dirs, hipStream_t st,
                bool* band_written = nullptr) {
  dim3 grid((unsigned)n), block(256);
  const bool halves = model == KGE_COMPLEX || model == KGE_ROTATE || model == KGE_CP || model == KGE_SIMPLE;
  const int unit = halves ? d_e / 2 : d_e;
  const bool vec = model != KGE_RESCAL && (!halves || d_e % 2 == 0) &&
                   unit % 4 == 0 && ld_ent % 4 == 0 && ld_rel % 4 == 0 && aligned16(ent) && aligned16(rel) &&
                   (!q.q || (q.ldq % 4 == 0 && aligned16(q.q))) &&
                   (!q.hi || (q.ldp % 8 == 0 && aligned16(q.hi) && aligned16(q.lo)));
  if (band_written) *band_written = vec && q.band;
  if (!vec) q.band = nullptr;  // only the vectorised kernel writes it
  if (vec) {
    const dim3 g4((unsigned)((n + 3) / 4));
    switch (model) {
      case KGE_COMPLEX:
        prep_elementwise_vec<KGE_COMPLEX><<<g4, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, q, dirs);
        break;
      case KGE_DISTMULT:
        prep_elementwise_vec<KGE_DISTMULT><<<g4, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, q, dirs);
        break;
      case KGE_TRANSE:
        prep_elementwise_vec<KGE_TRANSE><<<g4, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, q, dirs);
        break;
      case KGE_CP:
        prep_elementwise_vec<KGE_CP><<<g4, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, q, dirs);
        break;
      case KGE_SIMPLE:
        prep_elementwise_vec<KGE_SIMPLE><<<g4, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, q, dirs);
        break;
      default:
        prep_elementwise_vec<KGE_ROTATE><<<g4, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, q, dirs);
        break;
    }
    KGE_CHECK_LAUNCH();
    return 0;
  }
  switch (model) {
    case KGE_COMPLEX:
      prep_elementwise<KGE_COMPLEX><<<grid, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, d_e, q, dirs);
      break;
    case KGE_DISTMULT:
      prep_elementwise<KGE_DISTMULT><<<grid, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, d_e, q, dirs);
      break;
    case KGE_TRANSE:
      prep_elementwise<KGE_TRANSE><<<grid, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, d_e, q, dirs);
      break;
    case KGE_ROTATE:
      prep_elementwise<KGE_ROTATE><<<grid, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, d_e, q, dirs);
      break;
    case KGE_CP:
      prep_elementwise<KGE_CP><<<grid, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, d_e, q, dirs);
      break;
    case KGE_SIMPLE:
      prep_elementwise<KGE_SIMPLE><<<grid, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, d_e, q, dirs);
      break;
    case KGE_RESCAL:
      prep_rescal<<<grid, block, d_e * sizeof(float), st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, d_e, q, dirs);
      break;
    default:
      return KGE_ERR_ARG;
  }
  KGE_CHECK_LAUNCH();
  return 0;
}

int launch_prep_bwd(int model, const float* ent, int64_t ld_ent, const int64_t* eidx, const float* rel,
                    int64_t ld_rel, const int64_t* ridx, int64_t n, int d_e, const float* dq,
                    int64_t lddq, float* d_ent, int64_t ld_dent, float* d_rel, int64_t ld_drel, Dirs dirs,
                    hipStream_t st) {
  dim3 grid((unsigned)n), block(256);
#define KGE_PB(M)                                                                          \
  prep_elementwise_bwd<M><<<grid, block, 0, st>>>(ent, ld_ent, eidx, rel, ld_rel, ridx, d_e, dq, lddq, d_ent, \
                                                  ld_dent, d_rel, ld_drel, dirs)
  switch (model) {
    case KGE_COMPLEX: KGE_PB(KGE_COMPLEX); break;
    case KGE_DISTMULT: KGE_PB(KGE_DISTMULT); break;
    case KGE_TRANSE: KGE_PB(KGE_TRANSE); break;
    case KGE_ROTATE: KGE_PB(KGE_ROTATE); break;
    case KGE_CP: KGE_PB(KGE_CP); break;
    case KGE_SIMPLE: KGE_PB(KGE_SIMPLE); break;
    case KGE_RESCAL:
      prep_rescal_bwd<<<grid, block, 2 * d_e * sizeof(float), st>>>(
          ent, ld_ent, eidx, rel, ld_rel, ridx, d_e, dq, lddq, d_ent, ld_dent, d_rel, ld_drel, dirs);
      break;
    default:
      return KGE_ERR_ARG;
  }
#undef KGE_PB
  KGE_CHECK_LAUNCH();
  return 0;
}

int check_dims(int model, int d_e, int d_r) {
  if (d_e <= 0) return KGE_ERR_ARG;
  switch (model) {
    case KGE_COMPLEX: return (d_e % 2 == 0 && d_r == d_e) ? 0 : KGE_ERR_ARG;
    case KGE_DISTMULT:
    case KGE_TRANSE: return d_r == d_e ? 0 : KGE_ERR_ARG;
    case KGE_ROTATE: return (d_e % 2 == 0 && d_r == d_e / 2) ? 0 : KGE_ERR_ARG;
    case KGE_RESCAL: return (d_r == d_e * d_e && d_e <= 8192) ? 0 : KGE_ERR_ARG;
    case KGE_CP: return (d_e % 2 == 0 && d_r == d_e / 2) ? 0 : KGE_ERR_ARG;
    case KGE_SIMPLE: return (d_e % 2 == 0 && d_r == d_e) ? 0 : KGE_ERR_ARG;
    default: return KGE_ERR_ARG;
  }
}

int query_width(int model, int d_e) { return model == KGE_CP ? d_e / 2 : d_e; }

}  // namespace

extern "C" int kge_prep_query(int model, int dir, const float* ent, int64_t ld_ent, const int64_t* eidx,
                              const float* rel, int64_t ld_rel, const int64_t* ridx, int64_t n, int d_e,
                              int d_r, float* q, int64_t ldq, void* stream) {
  return kge_prep_query_split(model, dir, ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, d_r, q, ldq, nullptr,
                              nullptr, 0, stream);
}

extern "C" int kge_prep_query_split(int model, int dir, const float* ent, int64_t ld_ent, const int64_t* eidx,
                                    const float* rel, int64_t ld_rel, const int64_t* ridx, int64_t n, int d_e,
                                    int d_r, float* q, int64_t ldq, void* q_hi, void* q_lo, int64_t ldp,
                                    void* stream) {
  return kge_prep_query_split2(model, dir, dir, 0, nullptr, ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, d_r, q, ldq,
                               q_hi, q_lo, ldp, stream);
}

extern "C" int kge_prep_query_split2(int model, int dir_a, int dir_b, int64_t n_a, const int64_t* n_a_dev,
                                     const float* ent, int64_t ld_ent, const int64_t* eidx, const float* rel,
                                     int64_t ld_rel, const int64_t* ridx, int64_t n, int d_e, int d_r, float* q,
                                     int64_t ldq, void* q_hi, void* q_lo, int64_t ldp, void* stream) {
  if (int e = check_dims(model, d_e, d_r)) return e;
  KGE_REQUIRE(n >= 0 && ent && rel && (q || q_hi));
  KGE_REQUIRE(!q || ldq >= query_width(model, d_e));
  KGE_REQUIRE(!q_hi || (q_lo && ldp >= query_width(model, d_e) && ldp % 8 == 0));
  KGE_REQUIRE((dir_a == KGE_DIR_SP || dir_a == KGE_DIR_PO) && (dir_b == KGE_DIR_SP || dir_b == KGE_DIR_PO));
  KGE_REQUIRE(n_a >= 0);
  if (n == 0) return 0;
  const int qw = query_width(model, d_e);
  QOut out{q, ldq, (__bf16*)q_hi, (__bf16*)q_lo, ldp, (int)std::min<int64_t>(ldp, (qw + 31) / 32 * 32)};
  return launch_prep(model, ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, out, Dirs{dir_a, dir_b, n_a, n_a_dev},
                     as_stream(stream));
}

extern "C" int kge_rank_band(const float* q, int64_t ldq, int64_t n, int d, float band_rel, const float* t_norm_max,
                             float* band, void* stream);

extern "C" int kge_prep_query_split2_band(int model, int dir_a, int dir_b, int64_t n_a, const float* ent,
                                          int64_t ld_ent, const int64_t* eidx, const float* rel, int64_t ld_rel,
                                          const int64_t* ridx, int64_t n, int d_e, int d_r, float* q, int64_t ldq,
                                          void* q_hi, void* q_lo, int64_t ldp, float band_rel,
                                          const float* t_norm_max, float* band, void* stream) {
  if (int e = check_dims(model, d_e, d_r)) return e;
  KGE_REQUIRE(n >= 0 && ent && rel && q && q_hi && q_lo && band && t_norm_max && band_rel >= 0.f);
  KGE_REQUIRE(ldq >= query_width(model, d_e) && ldp >= query_width(model, d_e) && ldp % 8 == 0);
  KGE_REQUIRE((dir_a == KGE_DIR_SP || dir_a == KGE_DIR_PO) && (dir_b == KGE_DIR_SP || dir_b == KGE_DIR_PO));
  KGE_REQUIRE(n_a >= 0);
  if (n == 0) return 0;
  const int qw = query_width(model, d_e);
  QOut out{q, ldq, (__bf16*)q_hi, (__bf16*)q_lo, ldp, (int)std::min<int64_t>(ldp, (qw + 31) / 32 * 32)};
  out.band = band;
  out.band_rel = band_rel;
  out.tmax = t_norm_max;
  bool written = false;
  const int r = launch_prep(model, ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, out, Dirs{dir_a, dir_b, n_a, nullptr},
                            as_stream(stream), &written);
  if (r != 0 || written) return r;
  return kge_rank_band(q, ldq, n, qw, band_rel, t_norm_max, band, stream);  // layouts the vector kernel does not take
}

extern "C" int kge_prep_query_bwd(int model, int dir, const float* ent, int64_t ld_ent, const int64_t* eidx,
                                  const float* rel, int64_t ld_rel, const int64_t* ridx, int64_t n, int d_e,
                                  int d_r, const float* dq, int64_t lddq, float* d_ent, int64_t ld_dent,
                                  float* d_rel, int64_t ld_drel, void* stream) {
  return kge_prep_query_bwd2(model, dir, dir, 0, nullptr, ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, d_r, dq, lddq,
                             d_ent, ld_dent, d_rel, ld_drel, stream);
}

extern "C" int kge_prep_query_bwd2(int model, int dir_a, int dir_b, int64_t n_a, const int64_t* n_a_dev,
                                   const float* ent, int64_t ld_ent, const int64_t* eidx, const float* rel,
                                   int64_t ld_rel, const int64_t* ridx, int64_t n, int d_e, int d_r, const float* dq,
                                   int64_t lddq, float* d_ent, int64_t ld_dent, float* d_rel, int64_t ld_drel,
                                   void* stream) {
  if (int e = check_dims(model, d_e, d_r)) return e;
  KGE_REQUIRE(n >= 0 && ent && rel && dq && n_a >= 0);
  KGE_REQUIRE((dir_a == KGE_DIR_SP || dir_a == KGE_DIR_PO) && (dir_b == KGE_DIR_SP || dir_b == KGE_DIR_PO));
  if (n == 0 || (!d_ent && !d_rel)) return 0;
  return launch_prep_bwd(model, ent, ld_ent, eidx, rel, ld_rel, ridx, n, d_e, dq, lddq, d_ent, ld_dent, d_rel, ld_drel,
                         Dirs{dir_a, dir_b, n_a, n_a_dev}, as_stream(stream));
}

// Row-wise triple scores, combine="spo" (KgeModel.score_spo, kge_model.py:620-637), and
// their backward.  Used for the eval true scores (entity_ranking.py:139-140) and the
// negative-sampling "triple" implementation (train.py:887-892).  One wave per triple:
// the three rows are gathered coalesced and reduced across the wave.
#include "common.h"

namespace {

constexpr int NT = 256;  // 4 triples per block

struct Trip {
  const float* s;
  const float* p;
  const float* o;
};

__device__ __forceinline__ Trip rows_of(const float* ent, int64_t ld_ent, const int64_t* sidx, const float* rel,
                                        int64_t ld_rel, const int64_t* pidx, const int64_t* oidx, int64_t i) {
  return Trip{ent + sidx[i] * ld_ent, rel + pidx[i] * ld_rel, ent + oidx[i] * ld_ent};
}

// value of the per-element "difference" of the distance models
__device__ __forceinline__ float transe_diff(float s, float p, float o) {
  return ((s + p) - o) + 1e-6f;  // F.pairwise_distance: ||x1 - x2 + eps|| (transe.py:17)
}

template <int MODEL>
__global__ void __launch_bounds__(NT) spo_kernel(float l_norm, const float* __restrict__ ent, int64_t ld_ent,
                                                 const int64_t* __restrict__ sidx, const float* __restrict__ rel,
                                                 int64_t ld_rel, const int64_t* __restrict__ pidx,
                                                 const int64_t* __restrict__ oidx, int64_t n, int d_e,
                                                 float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (i >= n) return;
  Trip t = rows_of(ent, ld_ent, sidx, rel, ld_rel, pidx, oidx, i);
  float acc = 0.f;
  if (MODEL == KGE_COMPLEX) {
    const int h = d_e / 2;
    for (int k = lane; k < h; k += 64) {
      const float s_re = t.s[k], s_im = t.s[k + h], r_re = t.p[k], r_im = t.p[k + h];
      const float q_re = s_re * r_re - s_im * r_im, q_im = s_re * r_im + s_im * r_re;
      acc = fmaf(q_re, t.o[k], acc);
      acc = fmaf(q_im, t.o[k + h], acc);
    }
  } else if (MODEL == KGE_DISTMULT) {
    for (int k = lane; k < d_e; k += 64) acc = fmaf(t.s[k] * t.p[k], t.o[k], acc);
  } else if (MODEL == KGE_CP) {  // sum s_h p o_t (cp.py:21)
    const int h = d_e / 2;
    for (int k = lane; k < h; k += 64) acc = fmaf(t.s[k] * t.p[k], t.o[k + h], acc);
  } else if (MODEL == KGE_SIMPLE) {  // (sum s_h p_f o_t + sum s_t p_b o_h) / 2 (simple.py:21-23,34)
    const int h = d_e / 2;
    for (int k = lane; k < h; k += 64) {
      acc = fmaf(t.s[k] * t.p[k], t.o[k + h], acc);
      acc = fmaf(t.s[k + h] * t.p[k + h], t.o[k], acc);
    }
  } else if (MODEL == KGE_RESCAL) {  // s^T M o, M = p.view(d, d)
    for (int a = 0; a < d_e; ++a) {
      float row = 0.f;
      for (int b = lane; b < d_e; b += 64) row = fmaf(t.p[(int64_t)a * d_e + b], t.o[b], row);
      acc = fmaf(t.s[a], row, acc);
    }
  } else if (MODEL == KGE_TRANSE) {
    for (int k = lane; k < d_e; k += 64) {
      const float df = transe_diff(t.s[k], t.p[k], t.o[k]);
      acc = (l_norm == 1.f) ? acc + fabsf(df) : fmaf(df, df, acc);
    }
  } else {  // ROTATE
    const int h = d_e / 2;
    for (int k = lane; k < h; k += 64) {
      float c, sn;
      sincosf(t.p[k], &sn, &c);
      const float s_re = t.s[k], s_im = t.s[k + h];
      const float dr = (s_re * c - s_im * sn) - t.o[k];
      const float di = (s_re * sn + s_im * c) - t.o[k + h];
      const float sq = fmaf(di, di, dr * dr);
      acc += (l_norm == 1.f) ? sqrtf(sq) : sq;
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    if (MODEL == KGE_TRANSE) acc = -((l_norm == 1.f) ? acc : sqrtf(acc));
    if (MODEL == KGE_ROTATE && l_norm != 1.f) acc = sqrtf(acc);
    if (MODEL == KGE_SIMPLE) acc *= 0.5f;
    out[i] = acc;
  }
}

template <int MODEL>
__global__ void __launch_bounds__(NT) spo_bwd_kernel(float l_norm, const float* __restrict__ ent, int64_t ld_ent,
                                                     const int64_t* __restrict__ sidx, const float* __restrict__ rel,
                                                     int64_t ld_rel, const int64_t* __restrict__ pidx,
                                                     const int64_t* __restrict__ oidx, int64_t n, int d_e,
                                                     const float* __restrict__ g, float* d_ent, int64_t ld_dent,
                                                     float* d_rel, int64_t ld_drel) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (i >= n) return;
  Trip t = rows_of(ent, ld_ent, sidx, rel, ld_rel, pidx, oidx, i);
  const float gi = g[i];
  float* gs = d_ent ? d_ent + sidx[i] * ld_dent : nullptr;
  float* go = d_ent ? d_ent + oidx[i] * ld_dent : nullptr;
  float* gp = d_rel ? d_rel + pidx[i] * ld_drel : nullptr;
  auto add = [](float* base, int64_t k, float v) {
    if (base) atomicAdd(base + k, v);
  };
  if (MODEL == KGE_COMPLEX) {
    const int h = d_e / 2;
    for (int k = lane; k < h; k += 64) {
      const float s_re = t.s[k], s_im = t.s[k + h], r_re = t.p[k], r_im = t.p[k + h];
      const float o_re = t.o[k], o_im = t.o[k + h];
      const float q_re = s_re * r_re - s_im * r_im, q_im = s_re * r_im + s_im * r_re;
      add(go, k, gi * q_re);
      add(go, k + h, gi * q_im);
      const float gq_re = gi * o_re, gq_im = gi * o_im;  // dq = g*o; ds = dq*conj(r); dr = dq*conj(s)
      add(gs, k, gq_re * r_re + gq_im * r_im);
      add(gs, k + h, gq_im * r_re - gq_re * r_im);
      add(gp, k, gq_re * s_re + gq_im * s_im);
      add(gp, k + h, gq_im * s_re - gq_re * s_im);
    }
  } else if (MODEL == KGE_DISTMULT) {
    for (int k = lane; k < d_e; k += 64) {
      const float s = t.s[k], p = t.p[k], o = t.o[k];
      add(gs, k, gi * p * o);
      add(gp, k, gi * s * o);
      add(go, k, gi * s * p);
    }
  } else if (MODEL == KGE_CP) {
    const int h = d_e / 2;
    for (int k = lane; k < h; k += 64) {
      const float s = t.s[k], p = t.p[k], o = t.o[k + h];
      add(gs, k, gi * p * o);
      add(gp, k, gi * s * o);
      add(go, k + h, gi * s * p);
    }
  } else if (MODEL == KGE_SIMPLE) {
    const int h = d_e / 2;
    const float g2 = 0.5f * gi;
    for (int k = lane; k < h; k += 64) {
      const float sh = t.s[k], st = t.s[k + h], pf = t.p[k], pb = t.p[k + h], oh = t.o[k], ot = t.o[k + h];
      add(gs, k, g2 * pf * ot);
      add(gs, k + h, g2 * pb * oh);
      add(gp, k, g2 * sh * ot);
      add(gp, k + h, g2 * st * oh);
      add(go, k, g2 * st * pb);
      add(go, k + h, g2 * sh * pf);
    }
  } else if (MODEL == KGE_RESCAL) {
    for (int a = 0; a < d_e; ++a) {
      float row = 0.f;  // (M o)_a
      for (int b = lane; b < d_e; b += 64) {
        const float m = t.p[(int64_t)a * d_e + b];
        row = fmaf(m, t.o[b], row);
        add(gp, (int64_t)a * d_e + b, gi * t.s[a] * t.o[b]);
        add(go, b, gi * t.s[a] * m);
      }
      row = wave_sum(row);
      if (lane == 0) add(gs, a, gi * row);
    }
  } else if (MODEL == KGE_TRANSE) {
    float nrm = 0.f;
    if (l_norm != 1.f) {
      for (int k = lane; k < d_e; k += 64) {
        const float df = transe_diff(t.s[k], t.p[k], t.o[k]);
        nrm = fmaf(df, df, nrm);
      }
      nrm = sqrtf(wave_sum(nrm));
    }
    for (int k = lane; k < d_e; k += 64) {
      const float df = transe_diff(t.s[k], t.p[k], t.o[k]);
      float gd;  // d(-||df||)/d df
      if (l_norm == 1.f)
        gd = df > 0.f ? -gi : (df < 0.f ? gi : 0.f);
      else
        gd = nrm > 0.f ? -gi * df / nrm : 0.f;
      add(gs, k, gd);
      add(gp, k, gd);
      add(go, k, -gd);
    }
  } else {  // ROTATE
    const int h = d_e / 2;
    float tot = 0.f;
    if (l_norm != 1.f) {
      for (int k = lane; k < h; k += 64) {
        float c, sn;
        sincosf(t.p[k], &sn, &c);
        const float dr = (t.s[k] * c - t.s[k + h] * sn) - t.o[k];
        const float di = (t.s[k] * sn + t.s[k + h] * c) - t.o[k + h];
        tot = fmaf(di, di, fmaf(dr, dr, tot));
      }
      tot = sqrtf(wave_sum(tot));
    }
    for (int k = lane; k < h; k += 64) {
      float c, sn;
      sincosf(t.p[k], &sn, &c);
      const float s_re = t.s[k], s_im = t.s[k + h];
      const float q_re = s_re * c - s_im * sn, q_im = s_re * sn + s_im * c;
      const float dr = q_re - t.o[k], di = q_im - t.o[k + h];
      float f;
      if (l_norm == 1.f) {
        const float a = sqrtf(fmaf(di, di, dr * dr));
        f = a > 0.f ? gi / a : 0.f;
      } else {
        f = tot > 0.f ? gi / tot : 0.f;
      }
      const float g_re = f * dr, g_im = f * di;  // d/dq
      add(go, k, -g_re);
      add(go, k + h, -g_im);
      add(gs, k, g_re * c + g_im * sn);
      add(gs, k + h, g_im * c - g_re * sn);
      add(gp, k, g_im * q_re - g_re * q_im);
    }
  }
}

int check(int model, int d_e, int d_r) {
  switch (model) {
    case KGE_COMPLEX: return (d_e % 2 == 0 && d_r == d_e) ? 0 : KGE_ERR_ARG;
    case KGE_DISTMULT:
    case KGE_TRANSE: return d_r == d_e ? 0 : KGE_ERR_ARG;
    case KGE_ROTATE: return (d_e % 2 == 0 && d_r == d_e / 2) ? 0 : KGE_ERR_ARG;
    case KGE_RESCAL: return d_r == d_e * d_e ? 0 : KGE_ERR_ARG;
    case KGE_CP: return (d_e % 2 == 0 && d_r == d_e / 2) ? 0 : KGE_ERR_ARG;
    case KGE_SIMPLE: return (d_e % 2 == 0 && d_r == d_e) ? 0 : KGE_ERR_ARG;
    default: return KGE_ERR_ARG;
  }
}

}  // namespace

extern "C" int kge_score_spo(int model, float l_norm, const float* ent, int64_t ld_ent, const int64_t* sidx,
                             const float* rel, int64_t ld_rel, const int64_t* pidx, const int64_t* oidx, int64_t n,
                             int d_e, int d_r, float* out, void* stream) {
  if (int e = check(model, d_e, d_r)) return e;
  KGE_REQUIRE(n >= 0 && ent && rel && sidx && pidx && oidx && out);
  KGE_REQUIRE(l_norm == 1.f || l_norm == 2.f || (model != KGE_TRANSE && model != KGE_ROTATE));
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)((n + 3) / 4)), block(NT);
#define KGE_S(M) spo_kernel<M><<<grid, block, 0, st>>>(l_norm, ent, ld_ent, sidx, rel, ld_rel, pidx, oidx, n, d_e, out)
  switch (model) {
    case KGE_COMPLEX: KGE_S(KGE_COMPLEX); break;
    case KGE_DISTMULT: KGE_S(KGE_DISTMULT); break;
    case KGE_RESCAL: KGE_S(KGE_RESCAL); break;
    case KGE_TRANSE: KGE_S(KGE_TRANSE); break;
    case KGE_CP: KGE_S(KGE_CP); break;
    case KGE_SIMPLE: KGE_S(KGE_SIMPLE); break;
    default: KGE_S(KGE_ROTATE); break;
  }
#undef KGE_S
  KGE_CHECK_LAUNCH();
  return 0;
}

extern "C" int kge_score_spo_bwd(int model, float l_norm, const float* ent, int64_t ld_ent, const int64_t* sidx,
                                 const float* rel, int64_t ld_rel, const int64_t* pidx, const int64_t* oidx,
                                 int64_t n, int d_e, int d_r, const float* g, float* d_ent, int64_t ld_dent,
                                 float* d_rel, int64_t ld_drel, void* stream) {
  if (int e = check(model, d_e, d_r)) return e;
  KGE_REQUIRE(n >= 0 && ent && rel && sidx && pidx && oidx && g);
  KGE_REQUIRE(l_norm == 1.f || l_norm == 2.f || (model != KGE_TRANSE && model != KGE_ROTATE));
  if (n == 0 || (!d_ent && !d_rel)) return 0;
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)((n + 3) / 4)), block(NT);
#define KGE_S(M)                                                                                            \
  spo_bwd_kernel<M><<<grid, block, 0, st>>>(l_norm, ent, ld_ent, sidx, rel, ld_rel, pidx, oidx, n, d_e, g, \
                                            d_ent, ld_dent, d_rel, ld_drel)
  switch (model) {
    case KGE_COMPLEX: KGE_S(KGE_COMPLEX); break;
    case KGE_DISTMULT: KGE_S(KGE_DISTMULT); break;
    case KGE_RESCAL: KGE_S(KGE_RESCAL); break;
    case KGE_TRANSE: KGE_S(KGE_TRANSE); break;
    case KGE_CP: KGE_S(KGE_CP); break;
    case KGE_SIMPLE: KGE_S(KGE_SIMPLE); break;
    default: KGE_S(KGE_ROTATE); break;
  }
#undef KGE_S
  KGE_CHECK_LAUNCH();
  return 0;
}

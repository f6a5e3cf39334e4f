// qsc_common.cuh — device helpers shared by the gfx950 kernels of libqsc_hip.so.
//
// Numerics follow the reference's torch CPU expressions op for op where that is cheap:
//   F_probit(y, std) = (1/2)*(1 + erf(y/(std*1.414213)))      qmc/quantization_model.py:57-61
//   the tensor / python-float division is a true fp32 division by fp32(std*1.414213)
//   (measured on torch 2.10: 100 % match with correctly rounded x/a), reproduced here by a
//   Markstein-corrected reciprocal multiply.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/qsc.h"

#define QSC_WAVE 64

#define QSC_CHECK_LAUNCH()                          \
  do {                                              \
    hipError_t e__ = hipGetLastError();             \
    if (e__ != hipSuccess) return (int)e__;         \
  } while (0)

#define QSC_TRY(x)                                  \
  do {                                              \
    hipError_t e__ = (x);                           \
    if (e__ != hipSuccess) return (int)e__;         \
  } while (0)

namespace qsc {

// Derived per-call constants of the probit model, passed by value to kernels.
struct Probit {
  float a;        // fp32(sigma * 1.414213)
  float inv_a;    // RN(1 / a)
  float kgrad;    // 1 / (a * sqrt(pi))      d/dy F(y) = exp(-(y/a)^2) * kgrad
  float offset;   // fp32(offset)
  int log_model;
  int nbins;
  int lo_sat;     // linear model: erf((-1e5 - x)/a) == -1 exactly for every finite x of interest
  int hi_sat;     // linear model: erf(( 1e5 - x)/a) ==  1
};

// host-side helper: build Probit from the C-ABI model
inline Probit make_probit(const qsc_model* m) {
  Probit p;
  p.a = (float)(m->sigma * 1.414213);
  p.inv_a = 1.0f / p.a;
  p.kgrad = (float)(1.0 / ((double)p.a * 1.7724538509055160273));
  p.offset = (float)m->offset;
  p.log_model = m->log_model;
  p.nbins = m->nbounds - 1;
  // erf saturates to exactly +-1 in fp32 for |z| >= 3.92; the clamp edges are +-1e5.  The
  // "saturated edge" shortcut is exact whenever 1e5/a stays far beyond that (a < 2.5e4).
  int sat = (m->log_model == 0) && (p.a < 2.5e4f);
  p.lo_sat = sat;
  p.hi_sat = sat;
  return p;
}

// Bin edge table: lo/hi boundary of code c (linear model clamps b[0], b[-1] to -/+1e5 as in
// qmc/quantization_model.py:31-33; the log model uses the raw edges, _log.py:32-36).
struct Edges {
  float2 e[QSC_MAX_BOUNDS - 1];
};

inline void make_edges(const qsc_model* m, Edges* E) {
  const int nb = m->nbounds;
  for (int c = 0; c < nb - 1; ++c) {
    float lo = m->bounds[c], hi = m->bounds[c + 1];
    if (m->log_model == 0) {
      if (c == 0) lo = -100000.0f;
      if (c == nb - 2) hi = 100000.0f;
    }
    E->e[c] = make_float2(lo, hi);
  }
}

// Squared-loss targets: e[c].x = fp32(b[c] + b[c+1]) / 2 on the raw edges, the operation
// order of get_quantized_obs_from_ordinal (qmc/quantization_model_log.py:48-51).
inline void make_sq_targets(const qsc_model* m, Edges* E) {
  for (int c = 0; c < m->nbounds - 1; ++c) {
    const float lo = m->bounds[c], hi = m->bounds[c + 1];
    E->e[c] = make_float2((lo + hi) / 2.0f, 0.0f);
  }
}

// Correctly rounded x / a for a > 0 (one reciprocal multiply + one FMA residual correction).
__device__ __forceinline__ float div_a(float x, const Probit& pr) {
  float q = x * pr.inv_a;
  float r = __builtin_fmaf(-q, pr.a, x);
  return __builtin_fmaf(r, pr.inv_a, q);
}

// F_probit of an already-scaled argument z = y/a:  0.5f * (1.0f + erff(z))
__device__ __forceinline__ float phi_scaled(float z) { return 0.5f * (1.0f + erff(z)); }

// Likelihood of one observed entry with value x (already in the model domain) and code bin
// edges (lo, hi):  P = F(hi - x) - F(lo - x),  gx = d(-log P)/dx.
// `sat` selects the single-erf form for edges that saturate exactly (see make_probit).
__device__ __forceinline__ void probit_lik(float x, float lo, float hi, bool lo_is_sat,
                                           bool hi_is_sat, const Probit& pr, float& P,
                                           float& gx) {
  if (lo_is_sat) {
    // F(lo - x) == 0.5f*(1 + (-1)) == 0 exactly
    const float u = div_a(hi - x, pr);
    P = phi_scaled(u);
    gx = __expf(-u * u) * pr.kgrad / P;
  } else if (hi_is_sat) {
    // F(hi - x) == 0.5f*(1 + 1) == 1 exactly
    const float w = div_a(lo - x, pr);
    P = 1.0f - phi_scaled(w);
    gx = -__expf(-w * w) * pr.kgrad / P;
  } else {
    const float u = div_a(hi - x, pr);
    const float w = div_a(lo - x, pr);
    P = phi_scaled(u) - phi_scaled(w);
    gx = (__expf(-u * u) - __expf(-w * w)) * pr.kgrad / P;
  }
}

// ------------------------------------------------------------------------------------
// Branch-free erf with the exact operation sequence of ROCm's ocml erff (ROCm 7.2,
// read back from its gfx950 ISA): |x| < 1 -> x + x*poly(x^2); |x| >= 1 -> 1 - exp(-p(|x|))
// with ocml's two-part exp; sign copied from x.  Bitwise identical to erff, but both halves
// are evaluated and selected so that a wavefront never diverges on |x| and the compiler can
// interleave independent entries.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ float bits(uint32_t u) { return __uint_as_float(u); }

__device__ __forceinline__ float erf_bf(float x) {
  const float ax = fabsf(x);
  // |x| >= 1 branch
  float p = __builtin_fmaf(ax, bits(0x378e98abu), bits(0xb9c68948u));
  p = __builtin_fmaf(ax, p, bits(0x3b7cd369u));
  p = __builtin_fmaf(ax, p, bits(0xbcc618b2u));
  p = __builtin_fmaf(ax, p, bits(0x3dda74e4u));
  p = __builtin_fmaf(ax, p, bits(0x3f228afdu));
  p = __builtin_fmaf(ax, p, bits(0x3e03c728u));
  p = __builtin_fmaf(ax, p, ax);
  // exp(-p), ocml expf: hi/lo split of -log2(e), round, exp2, ldexp, range selects
  const float nl2e = bits(0xbfb8aa3bu);
  const float h = p * nl2e;
  float l = __builtin_fmaf(p, nl2e, -h);
  const float n = __builtin_rintf(h);
  l = __builtin_fmaf(p, bits(0xb2a5705fu), l);
  float r = __builtin_amdgcn_exp2f((h - n) + l);
  r = __builtin_amdgcn_ldexpf(r, (int)n);
  r = !(p > bits(0x42ce8ed0u)) ? r : 0.0f;             // NaN keeps r (v_cmp_nlt)
  r = !(p < bits(0xc2b17218u)) ? r : __builtin_inff();  // (v_cmp_ngt)
  const float big = 1.0f - r;
  // |x| < 1 branch
  const float t = x * x;
  float q = __builtin_fmaf(bits(0xba1345e1u), t, bits(0x3ba10414u));
  q = __builtin_fmaf(t, q, bits(0xbcdac9b8u));
  q = __builtin_fmaf(t, q, bits(0x3de703beu));
  q = __builtin_fmaf(t, q, bits(0xbec09330u));
  q = __builtin_fmaf(t, q, bits(0x3e0375d0u));
  const float small = __builtin_fmaf(ax, q, ax);
  const float m = (ax < 1.0f) ? small : big;  // NaN takes the |x| >= 1 path, as in ocml
  return __builtin_copysignf(m, x);
}

// erf of the fused passes: ocml erff's two polynomials (the coefficients above), with the
// |x| >= 1 tail exp(-p) taken straight from the hardware exp2 (v_exp_f32) instead of ocml's
// range-reduced expf.  p >= 1.8 there, so exp(-p) <= 0.16 and its few-ulp relative error moves
// erf by < 1 ulp (checked against erff by qsc_selftest_erf).  Both halves are evaluated so a
// wavefront never diverges on |x|.  ~24 VALU instead of erf_bf's ~35.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  float p = __builtin_fmaf(ax, bits(0x378e98abu), bits(0xb9c68948u));
  p = __builtin_fmaf(ax, p, bits(0x3b7cd369u));
  p = __builtin_fmaf(ax, p, bits(0xbcc618b2u));
  p = __builtin_fmaf(ax, p, bits(0x3dda74e4u));
  p = __builtin_fmaf(ax, p, bits(0x3f228afdu));
  p = __builtin_fmaf(ax, p, bits(0x3e03c728u));
  p = __builtin_fmaf(ax, p, ax);
  const float big = 1.0f - __builtin_amdgcn_exp2f(p * bits(0xbfb8aa3bu));  // 1 - exp(-p)
  const float t = x * x;
  float q = __builtin_fmaf(bits(0xba1345e1u), t, bits(0x3ba10414u));
  q = __builtin_fmaf(t, q, bits(0xbcdac9b8u));
  q = __builtin_fmaf(t, q, bits(0x3de703beu));
  q = __builtin_fmaf(t, q, bits(0xbec09330u));
  q = __builtin_fmaf(t, q, bits(0x3e0375d0u));
  const float small = __builtin_fmaf(ax, q, ax);
  return __builtin_copysignf((ax < 1.0f) ? small : big, x);
}

// Per-call constants of the fused passes.
struct Lik {
  float a, inv_a, kgrad, offset;
  float thr;      // b[1]: the single active edge of the saturated one-bit model
  float thr_a;    // fp32(thr / a): the one-bit model's z offset in the scaled form
};

inline Lik make_lik(const qsc_model* m) {
  const Probit p = make_probit(m);
  Lik l;
  l.a = p.a;
  l.inv_a = p.inv_a;
  l.kgrad = p.kgrad;
  l.offset = p.offset;
  l.thr = m->nbounds >= 2 ? m->bounds[1] : 0.0f;
  l.thr_a = (float)((double)l.thr / (double)l.a);
  return l;
}

// Fused-pass likelihood kinds: one active edge (linear one-bit with saturated +-1e5 outer
// edges: P = F(thr - x) for code 0, 1 - F(thr - x) for code 1, exactly the reference's values),
// or the general two-edge form (multi-bin and/or log model).
enum { LIK_ONEBIT = 0, LIK_GENERAL = 1, LIK_SQUARED = 2 };

inline int lik_kind(const qsc_model* m) {
  if (m->loss == QSC_LOSS_SQUARED) return LIK_SQUARED;
  const Probit p = make_probit(m);
  return (m->log_model == 0 && m->nbounds == 3 && p.lo_sat && p.hi_sat) ? LIK_ONEBIT : LIK_GENERAL;
}

__device__ __forceinline__ float div_lik(float x, const Lik& c) {
  const float q = x * c.inv_a;
  const float r = __builtin_fmaf(-q, c.a, x);
  return __builtin_fmaf(r, c.inv_a, q);
}

constexpr float kNegLog2e = -1.44269504088896340736f;
constexpr float kLn2 = 0.69314718055994530942f;
constexpr float kInvLn2 = 1.44269504088896340736f;

// One observed entry: t = reconstruction value; returns log2 P (the caller scales the summed
// NLL by ln 2 once) and g = d(-log P)/dt.  Branch-free; `edges` is only read by the general kind.
template <int KIND, bool LOG>
__device__ __forceinline__ void lik_grad(float t, int code, const float2* __restrict__ edges,
                                         const Lik& c, float& log2P, float& g) {
  if (KIND == LIK_SQUARED) {
    float x = t, tinv = 1.0f;
    if (LOG) {
      const float tp = t + c.offset;
      x = logf(tp);
      tinv = __builtin_amdgcn_rcpf(tp);
    }
    const float r = x - edges[code].x;
    g = 2.0f * r * tinv;
    log2P = -(r * r) * kInvLn2;
  } else if (KIND == LIK_ONEBIT) {
    const float z = div_lik(c.thr - t, c);
    const float F = 0.5f * (1.0f + erf_fast(z));
    const bool c0 = (code == 0);
    const float P = c0 ? F : 1.0f - F;
    const float e = __builtin_amdgcn_exp2f(z * z * kNegLog2e) * c.kgrad;  // exp(-z^2) / (a sqrt(pi))
    g = (c0 ? e : -e) * __builtin_amdgcn_rcpf(P);
    log2P = __builtin_amdgcn_logf(P);
  } else {
    float x = t, tinv = 1.0f;
    if (LOG) {
      const float tp = t + c.offset;
      x = logf(tp);
      tinv = __builtin_amdgcn_rcpf(tp);
    }
    const float2 e2 = edges[code];
    const float u = div_lik(e2.y - x, c);
    const float w = div_lik(e2.x - x, c);
    const float P = 0.5f * (1.0f + erf_fast(u)) - 0.5f * (1.0f + erf_fast(w));
    const float d = (__builtin_amdgcn_exp2f(u * u * kNegLog2e) -
                     __builtin_amdgcn_exp2f(w * w * kNegLog2e)) * c.kgrad;
    g = d * __builtin_amdgcn_rcpf(P) * tinv;
    log2P = __builtin_amdgcn_logf(P);
  }
}

// ------------------------------------------------------------------------------------
// Two-entry (packed) forms.  gfx950 issues a wave64 f32 VALU op every ~4 cycles whether it is
// v_fma_f32 or v_pk_fma_f32 (measured, tools/micro/valu_rate.hip), so the polynomial / FMA
// parts of the per-entry math are evaluated for two entries per instruction.
// ------------------------------------------------------------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v fma2(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2v splat2(float x) { return f2v{x, x}; }

__device__ __forceinline__ f2v erf_fast2(f2v x) {
  const f2v ax = __builtin_elementwise_abs(x);
  f2v p = fma2(ax, splat2(bits(0x378e98abu)), splat2(bits(0xb9c68948u)));
  p = fma2(ax, p, splat2(bits(0x3b7cd369u)));
  p = fma2(ax, p, splat2(bits(0xbcc618b2u)));
  p = fma2(ax, p, splat2(bits(0x3dda74e4u)));
  p = fma2(ax, p, splat2(bits(0x3f228afdu)));
  p = fma2(ax, p, splat2(bits(0x3e03c728u)));
  p = fma2(ax, p, ax);
  const f2v pe = p * splat2(bits(0xbfb8aa3bu));
  const f2v big = splat2(1.0f) - f2v{__builtin_amdgcn_exp2f(pe.x), __builtin_amdgcn_exp2f(pe.y)};
  const f2v t = x * x;
  f2v q = fma2(splat2(bits(0xba1345e1u)), t, splat2(bits(0x3ba10414u)));
  q = fma2(t, q, splat2(bits(0xbcdac9b8u)));
  q = fma2(t, q, splat2(bits(0x3de703beu)));
  q = fma2(t, q, splat2(bits(0xbec09330u)));
  q = fma2(t, q, splat2(bits(0x3e0375d0u)));
  const f2v small = fma2(ax, q, ax);
  return f2v{__builtin_copysignf(ax.x < 1.0f ? small.x : big.x, x.x),
             __builtin_copysignf(ax.y < 1.0f ? small.y : big.y, x.y)};
}

__device__ __forceinline__ f2v div_lik2(f2v x, const Lik& c) {
  const f2v ia = splat2(c.inv_a);
  const f2v q = x * ia;
  const f2v r = fma2(-q, splat2(c.a), x);
  return fma2(r, ia, q);
}

__device__ __forceinline__ f2v exp2_2(f2v x) {
  return f2v{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
}
__device__ __forceinline__ f2v rcp2(f2v x) {
  return f2v{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)};
}
__device__ __forceinline__ f2v log2_2(f2v x) {
  return f2v{__builtin_amdgcn_logf(x.x), __builtin_amdgcn_logf(x.y)};
}

// lik_grad for two entries (t.x with code c0, t.y with code c1).
// Linear model (one-bit and multi-bin): the caller passes t in the SCALED form t' = -t / a
// (its register factor vector pre-multiplied by -1/a, so the dot product yields t' directly)
// and, for the general kind, edges pre-divided by a: z = thr/a + t', u = hi/a + t',
// w = lo/a + t' (one add instead of a subtract and a division per entry).  The log model takes
// t itself (x = log(t + offset) needs it).
template <int KIND, bool LOG>
__device__ __forceinline__ void lik_grad2(f2v t, int c0, int c1, const float2* __restrict__ edges,
                                          const Lik& c, f2v& log2P, f2v& g) {
  if (KIND == LIK_SQUARED) {
    // r = x - Obs; loss r^2 (returned as -r^2/ln2: the passes scale the summed log2 P by
    // ln 2); g = d(r^2)/dt = 2 r dx/dt.  t is unscaled for this kind.
    const float2 e0 = edges[c0], e1 = edges[c1];
    f2v x = t, tinv = splat2(1.0f);
    if (LOG) {
      const f2v tp = t + splat2(c.offset);
      x = f2v{logf(tp.x), logf(tp.y)};
      tinv = rcp2(tp);
    }
    const f2v r = x - f2v{e0.x, e1.x};
    g = splat2(2.0f) * r * tinv;
    log2P = -(r * r) * splat2(kInvLn2);
  } else if (KIND == LIK_ONEBIT) {
    const f2v z = splat2(c.thr_a) + t;
    const f2v F = splat2(0.5f) * (splat2(1.0f) + erf_fast2(z));
    const f2v Fc = splat2(1.0f) - F;
    const bool z0 = (c0 == 0), z1 = (c1 == 0);
    const f2v P = f2v{z0 ? F.x : Fc.x, z1 ? F.y : Fc.y};
    const f2v e = exp2_2(z * z * splat2(kNegLog2e)) * splat2(c.kgrad);
    const f2v rp = rcp2(P);
    g = f2v{z0 ? e.x : -e.x, z1 ? e.y : -e.y} * rp;
    log2P = log2_2(P);
  } else {
    const float2 e0 = edges[c0], e1 = edges[c1];
    f2v u, w, tinv = splat2(1.0f);
    if (LOG) {
      const f2v tp = t + splat2(c.offset);
      const f2v x = f2v{logf(tp.x), logf(tp.y)};
      tinv = rcp2(tp);
      u = div_lik2(f2v{e0.y, e1.y} - x, c);
      w = div_lik2(f2v{e0.x, e1.x} - x, c);
    } else {
      u = f2v{e0.y, e1.y} + t;
      w = f2v{e0.x, e1.x} + t;
    }
    const f2v P = splat2(0.5f) * (splat2(1.0f) + erf_fast2(u)) -
                  splat2(0.5f) * (splat2(1.0f) + erf_fast2(w));
    const f2v d = (exp2_2(u * u * splat2(kNegLog2e)) - exp2_2(w * w * splat2(kNegLog2e))) *
                  splat2(c.kgrad);
    g = d * rcp2(P) * tinv;
    log2P = log2_2(P);
  }
}

// ------------------------------------------------------------------------------------
// Four-entry forms: the same per-element operation sequence as lik_grad2 (bitwise the same
// results) on 4-wide vectors, which the backend splits into two independent v_pk_* chains.
// Interleaving the two chains fills the issue slot that a dependent packed op would otherwise
// spend on an s_nop (packed-VALU read-after-write hazard) and doubles the ILP per wave.
// ------------------------------------------------------------------------------------
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v fma4(f4v a, f4v b, f4v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f4v splat4(float x) { return f4v{x, x, x, x}; }
__device__ __forceinline__ f4v exp2_4(f4v x) {
  return f4v{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y), __builtin_amdgcn_exp2f(x.z),
             __builtin_amdgcn_exp2f(x.w)};
}
__device__ __forceinline__ f4v rcp4(f4v x) {
  return f4v{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y), __builtin_amdgcn_rcpf(x.z),
             __builtin_amdgcn_rcpf(x.w)};
}
__device__ __forceinline__ f4v log2_4(f4v x) {
  return f4v{__builtin_amdgcn_logf(x.x), __builtin_amdgcn_logf(x.y), __builtin_amdgcn_logf(x.z),
             __builtin_amdgcn_logf(x.w)};
}
__device__ __forceinline__ f4v sel4(bool c0, bool c1, bool c2, bool c3, f4v a, f4v b) {
  return f4v{c0 ? a.x : b.x, c1 ? a.y : b.y, c2 ? a.z : b.z, c3 ? a.w : b.w};
}

__device__ __forceinline__ f4v erf_fast4(f4v x) {
  const f4v ax = __builtin_elementwise_abs(x);
  f4v p = fma4(ax, splat4(bits(0x378e98abu)), splat4(bits(0xb9c68948u)));
  p = fma4(ax, p, splat4(bits(0x3b7cd369u)));
  p = fma4(ax, p, splat4(bits(0xbcc618b2u)));
  p = fma4(ax, p, splat4(bits(0x3dda74e4u)));
  p = fma4(ax, p, splat4(bits(0x3f228afdu)));
  p = fma4(ax, p, splat4(bits(0x3e03c728u)));
  p = fma4(ax, p, ax);
  const f4v pe = p * splat4(bits(0xbfb8aa3bu));
  const f4v big = splat4(1.0f) - exp2_4(pe);
  const f4v t = x * x;
  f4v q = fma4(splat4(bits(0xba1345e1u)), t, splat4(bits(0x3ba10414u)));
  q = fma4(t, q, splat4(bits(0xbcdac9b8u)));
  q = fma4(t, q, splat4(bits(0x3de703beu)));
  q = fma4(t, q, splat4(bits(0xbec09330u)));
  q = fma4(t, q, splat4(bits(0x3e0375d0u)));
  const f4v small = fma4(ax, q, ax);
  return f4v{__builtin_copysignf(ax.x < 1.0f ? small.x : big.x, x.x),
             __builtin_copysignf(ax.y < 1.0f ? small.y : big.y, x.y),
             __builtin_copysignf(ax.z < 1.0f ? small.z : big.z, x.z),
             __builtin_copysignf(ax.w < 1.0f ? small.w : big.w, x.w)};
}

__device__ __forceinline__ f4v div_lik4(f4v x, const Lik& c) {
  const f4v ia = splat4(c.inv_a);
  const f4v q = x * ia;
  const f4v r = fma4(-q, splat4(c.a), x);
  return fma4(r, ia, q);
}

// lik_grad2 on four entries (codes c[0..3]); same scaled-form convention
template <int KIND, bool LOG>
__device__ __forceinline__ void lik_grad4(f4v t, const int (&cd)[4],
                                          const float2* __restrict__ edges, const Lik& c,
                                          f4v& log2P, f4v& g) {
  if (KIND == LIK_SQUARED) {
    const float2 e0 = edges[cd[0]], e1 = edges[cd[1]], e2 = edges[cd[2]], e3 = edges[cd[3]];
    f4v x = t, tinv = splat4(1.0f);
    if (LOG) {
      const f4v tp = t + splat4(c.offset);
      x = f4v{logf(tp.x), logf(tp.y), logf(tp.z), logf(tp.w)};
      tinv = rcp4(tp);
    }
    const f4v r = x - f4v{e0.x, e1.x, e2.x, e3.x};
    g = splat4(2.0f) * r * tinv;
    log2P = -(r * r) * splat4(kInvLn2);
  } else if (KIND == LIK_ONEBIT) {
    const f4v z = splat4(c.thr_a) + t;
    const f4v F = splat4(0.5f) * (splat4(1.0f) + erf_fast4(z));
    const f4v Fc = splat4(1.0f) - F;
    const bool z0 = (cd[0] == 0), z1 = (cd[1] == 0), z2 = (cd[2] == 0), z3 = (cd[3] == 0);
    const f4v P = sel4(z0, z1, z2, z3, F, Fc);
    const f4v e = exp2_4(z * z * splat4(kNegLog2e)) * splat4(c.kgrad);
    const f4v rp = rcp4(P);
    g = sel4(z0, z1, z2, z3, e, -e) * rp;
    log2P = log2_4(P);
  } else {
    const float2 e0 = edges[cd[0]], e1 = edges[cd[1]], e2 = edges[cd[2]], e3 = edges[cd[3]];
    f4v u, w, tinv = splat4(1.0f);
    if (LOG) {
      const f4v tp = t + splat4(c.offset);
      const f4v x = f4v{logf(tp.x), logf(tp.y), logf(tp.z), logf(tp.w)};
      tinv = rcp4(tp);
      u = div_lik4(f4v{e0.y, e1.y, e2.y, e3.y} - x, c);
      w = div_lik4(f4v{e0.x, e1.x, e2.x, e3.x} - x, c);
    } else {
      u = f4v{e0.y, e1.y, e2.y, e3.y} + t;
      w = f4v{e0.x, e1.x, e2.x, e3.x} + t;
    }
    const f4v P = splat4(0.5f) * (splat4(1.0f) + erf_fast4(u)) -
                  splat4(0.5f) * (splat4(1.0f) + erf_fast4(w));
    const f4v d = (exp2_4(u * u * splat4(kNegLog2e)) - exp2_4(w * w * splat4(kNegLog2e))) *
                  splat4(c.kgrad);
    g = d * rcp4(P) * tinv;
    log2P = log2_4(P);
  }
}

// One observed entry end to end: t is the linear reconstruction value; returns P and the
// gradient of -log P w.r.t. t (chain rule through log(t + offset) in the log model).
__device__ __forceinline__ void entry_grad(float t, int code, const float2* edges,
                                           const Probit& pr, float& P, float& g) {
  float x = t, tinv = 1.0f;
  if (pr.log_model) {
    const float tp = t + pr.offset;
    x = logf(tp);
    tinv = 1.0f / tp;
  }
  const float2 e = edges[code];
  const bool lo_sat = pr.lo_sat && code == 0;
  const bool hi_sat = pr.hi_sat && code == pr.nbins - 1 && !lo_sat;
  float gx;
  probit_lik(x, e.x, e.y, lo_sat, hi_sat, pr, P, gx);
  g = gx * tinv;
}

// ------------------------------------------------------------------------------------
// reductions
// ------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block sum in a fixed order (deterministic).  `sh` must hold blockDim.x/64 elements.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  T r = 0;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int i = 0; i < nw; ++i) r += sh[i];
  }
  return r;  // valid in thread 0
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
__host__ __device__ inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

// Position of row ql of C-format pixel tile t (include/qsc.h): whole slices dealt to the nt
// tiles in snake order, so that every tile carries the same mix of the count-sorted positions.
__host__ __device__ inline int64_t tile_pos(int t, int ql, int nt) {
  const int i = ql / QSC_SLICE;
  const int g = i * nt + ((i & 1) ? (nt - 1 - t) : t);
  return (int64_t)g * QSC_SLICE + (ql % QSC_SLICE);
}

// Adam bias corrections exactly as torch.optim.Adam (_single_tensor_adam) forms them in
// Python double precision, then hands them to fp32 tensor-scalar ops.
struct AdamScalars {
  float step_size;  // fp32(lr / (1 - beta1^step))
  float bc2_sqrt;   // fp32(sqrt(1 - beta2^step))
  float w1;         // fp32(1 - beta1)  (lerp weight)
  float w2;         // fp32(1 - beta2)  (addcmul value)
  float beta2;      // fp32(beta2)      (mul_ scalar)
  float eps;        // fp32(eps)        (add_ scalar)
};

// beta^step for an integer step by binary powering in double (within an ulp of libm pow; the
// fp32 values derived from it match torch's).  Small register footprint, unlike ocml pow().
__device__ __noinline__ double ipow(double b, int n) {
  double r = 1.0;
  while (n > 0) {
    if (n & 1) r *= b;
    b *= b;
    n >>= 1;
  }
  return r;
}

__device__ __forceinline__ AdamScalars adam_scalars(const qsc_adam& ad, int step) {
  AdamScalars s;
  const double b1 = ad.beta1, b2 = ad.beta2;
  const double bc1 = 1.0 - ipow(b1, step);
  const double bc2 = 1.0 - ipow(b2, step);
  s.step_size = (float)(ad.lr / bc1);
  s.beta2 = (float)b2;
  s.eps = (float)ad.eps;
  s.bc2_sqrt = (float)sqrt(bc2);
  s.w1 = (float)(1.0 - b1);
  s.w2 = (float)(1.0 - b2);
  return s;
}

// One Adam element update (torch 2.x single-tensor path):
//   m.lerp_(g, 1-b1)                        -> fma(w1, g - m, m)        (ATen's vectorised lerp)
//   v.mul_(b2).addcmul_(g, g, value=1-b2)   -> fma(w2*g, g, v*b2)
//   denom = v.sqrt() / bc2_sqrt + eps ;  p.addcdiv_(m, denom, value=-step_size) -> p + (-s*m)/denom
// (each form checked bit-for-bit against torch 2.10 CPU on 2^20 random elements)
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g,
                                          const qsc_adam& ad, const AdamScalars& s) {
  m = __builtin_fmaf(s.w1, g - m, m);
  const float vb = __fmul_rn(v, s.beta2);
  v = __builtin_fmaf(__fmul_rn(s.w2, g), g, vb);
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), s.bc2_sqrt), s.eps);
  p = __fadd_rn(p, __fdiv_rn(__fmul_rn(-s.step_size, m), denom));
  if (ad.project_nonneg && p < 0.0f) p = 0.0f;
}

// The same update with the S-side's 2M-element cost in mind: sqrt and the two divisions as a
// hardware estimate plus one residual correction each (correctly rounded but for rare
// near-halfway cases, i.e. within 1 ulp of the torch values), ~20 VALU instead of ~50.
__device__ __forceinline__ float sqrt_fix(float v) {
  const float s = __builtin_amdgcn_sqrtf(v);
  const float e = __builtin_fmaf(-s, s, v);
  const float h = 0.5f * __builtin_amdgcn_rcpf(s);
  return v > 0.0f ? __builtin_fmaf(e, h, s) : s;
}
__device__ __forceinline__ float div_fix(float x, float y) {
  const float ry = __builtin_amdgcn_rcpf(y);
  const float q = x * ry;
  const float r = __builtin_fmaf(-q, y, x);
  return __builtin_fmaf(r, ry, q);
}
__device__ __forceinline__ void adam_elem_fast(float& p, float& m, float& v, float g,
                                               const AdamScalars& s) {
  m = __builtin_fmaf(s.w1, g - m, m);
  const float vb = __fmul_rn(v, s.beta2);
  v = __builtin_fmaf(__fmul_rn(s.w2, g), g, vb);
  const float denom = __fadd_rn(div_fix(sqrt_fix(v), s.bc2_sqrt), s.eps);
  p = __fadd_rn(p, div_fix(__fmul_rn(-s.step_size, m), denom));
}

}  // namespace qsc

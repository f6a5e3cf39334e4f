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
  float thr_a;    // fp32(thr / a): the general linear kind's z offset in the scaled form
  // one-bit kind (Mills-ratio form, lik_grad2): z is carried as z*sqrt(log2 e)
  float ob_scale; // fp32(sqrt(log2 e) / a): the factor rows are pre-scaled by -ob_scale
  float ob_thr;   // fp32(thr * sqrt(log2 e) / a)
  float ob_kg;    // fp32(kgrad / kMillsK)
  // bounds the QSC_DEBUG build checks (set by the launchers; unused otherwise): rows of the
  // C^T gather table [0] and of the S-tile table [1], entries of the S / C formats
  int dbg_rows[2];
  int64_t dbg_ent[2];
};

// QSC_DEBUG=1 builds (_build.py --debug): bounds checks in the pass kernels.  A failed check
// never traps (a GPU exception can take the whole node down): it records the line in a device
// flag, the offending index is clamped into range so the kernel finishes, and the host reads
// the flag with qsc_debug_status after the call.
#ifndef QSC_DEBUG
#define QSC_DEBUG 0
#endif
#if QSC_DEBUG
extern __device__ int g_qsc_dbg_line;
#define QSC_DCHECK(c)                                      \
  do {                                                     \
    if (!(c)) atomicMax(&::qsc::g_qsc_dbg_line, __LINE__); \
  } while (0)
#else
#define QSC_DCHECK(c) \
  do {                \
  } while (0)
#endif

// one-bit Mills-ratio form.  With c = sqrt(log2 e) and u = c |z|, the probit tail
// 0.5 erfc(|z|) = exp(-z^2) * 0.5 erfcx(|z|) is evaluated as
//     T = exp2(log2(kMillsK) - (c z)^2) * N(u) / D(u)
// where kMillsK N/D is a (3,4) rational fit of 0.5 erfcx(u / c) on u in [0, 3.95 c] (relative
// error 2.9e-7 in fp32, i.e. ~2 ulp; D has no roots on u >= 0, N/D -> 1/u for large u), N, D
// monic.  Fitted by a Lawson-weighted linear least-squares in float64 (tools/fit_mills.py).
constexpr float kMillsLogK = -1.5623618665631935f;
constexpr float kMillsN2 = 6.567472368922525f, kMillsN1 = 17.9604287105516f,
                kMillsN0 = 22.97849985876764f;
constexpr float kMillsD3 = 6.547683092308922f, kMillsD2 = 18.821234758060108f,
                kMillsD1 = 26.78107767395228f, kMillsD0 = 15.560871041019581f;
constexpr double kMillsK = 0.3385963046956732;
// Tail probabilities below 2^-25 are returned as exactly 0: where the reference's fp32
// 0.5 * (1 + erf(z)) (qmc/quantization_model.py:61) has saturated (it does for tails below
// 1.5e-8 .. 4.5e-8 depending on the side), so an observed entry that far out gets the
// reference's P == 0, log P = -inf and a non-finite gradient (tests/test_gpu_fused.py).
constexpr float kMillsTsat = 2.98023223876953125e-8f;  // 2^-25
// z of pad entries: deep on the P == 1 side (E == 0), so they add exactly 0 to NLL and gradient
constexpr float kPadZ = 1.0e4f;

inline Lik make_lik(const qsc_model* m) {
  const Probit p = make_probit(m);
  Lik l;
  l.a = p.a;
  l.inv_a = p.inv_a;
  l.kgrad = p.kgrad;
  l.offset = p.offset;
  l.thr = m->nbounds >= 2 ? m->bounds[1] : 0.0f;
  l.thr_a = (float)((double)l.thr / (double)l.a);
  const double c = 1.2011224087864498;  // sqrt(log2 e)
  l.ob_scale = (float)(c / (double)l.a);
  l.ob_thr = (float)((double)l.thr * c / (double)l.a);
  l.ob_kg = (float)((double)p.kgrad / kMillsK);
  l.dbg_rows[0] = l.dbg_rows[1] = 0;
  l.dbg_ent[0] = l.dbg_ent[1] = 0;
#if QSC_FTZ_SAT
  l.ob_kg = (float)((double)p.kgrad / kMillsK * 0x1p101);  // E is carried 2^-101 low
#endif
  return l;
}

// Fused-pass likelihood kinds: one active edge (linear one-bit with saturated +-1e5 outer
// edges: P = F(thr - x) for code 0, 1 - F(thr - x) for code 1, exactly the reference's values),
// or the general two-edge form (multi-bin and/or log model).
// LIK_ONEBIT_SR: the one-bit kind on signed-row layouts (qsc_obs_desc::rowfmt 1): the gathered
// row carries the entry's sign and threshold, [s*row, s*thr'] (s = +1 for code 0, -1 for code 1,
// pad rows [0, kPadZ]), so the walk evaluates z~ = s*z' with no code, pad or sign handling.
enum { LIK_ONEBIT = 0, LIK_GENERAL = 1, LIK_SQUARED = 2, LIK_ONEBIT_SR = 3 };

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

// Signed-row one-bit kind: z~ = s z' (the sign folded into the gathered row), so the tail side
// is z~ < 0 for both codes (code 0: z' < 0; code 1: z' > 0) and g needs no sign flip, the row
// being s*row.  Same arithmetic as the one-bit kind of lik_grad2, so the same P and g (but for
// z' == 0 exactly, where T and 1 - T are both 1/2 to within the fit's 3e-7).  P itself is
// returned: the walks take log2 of the product of two pairs' P (one v_log per 4 entries).
__device__ __forceinline__ void onebit_sr_pg(f2v z, const Lik& c, f2v& P, f2v& g) {
  const f2v u = f2v{__builtin_fabsf(z.x), __builtin_fabsf(z.y)};
#if QSC_FTZ_SAT
  const f2v E = exp2_2(fma2(-z, z, splat2(kMillsLogK - 101.0f)));
#else
  const f2v E = exp2_2(fma2(-z, z, splat2(kMillsLogK)));
#endif
  f2v N = u + splat2(kMillsN2);
  N = fma2(N, u, splat2(kMillsN1));
  N = fma2(N, u, splat2(kMillsN0));
  f2v D = u + splat2(kMillsD3);
  D = fma2(D, u, splat2(kMillsD2));
  D = fma2(D, u, splat2(kMillsD1));
  D = fma2(D, u, splat2(kMillsD0));
#if QSC_FTZ_SAT
  const f2v Ts = ((E * N) * rcp2(D)) * splat2(0x1p101f);
#else
  const f2v T = (E * N) * rcp2(D);
  const f2v Ts = f2v{T.x < kMillsTsat ? 0.0f : T.x, T.y < kMillsTsat ? 0.0f : T.y};
#endif
  const f2v Q = splat2(1.0f) - Ts;
  P = f2v{z.x < 0.0f ? Ts.x : Q.x, z.y < 0.0f ? Ts.y : Q.y};
  g = (E * splat2(c.ob_kg)) * rcp2(P);
}

// lik_grad for two entries (t.x with code c0, t.y with code c1); log2P and g of -log P.
// Linear general kind: the caller passes t in the SCALED form t' = -t / a (its register factor
// vector pre-multiplied by -1/a, so the dot product yields t' directly) and edges pre-divided by
// a: u = hi/a + t', w = lo/a + t' (one add instead of a subtract and a division per entry).  The
// log model takes t itself (x = log(t + offset) needs it).
// One-bit kind (Mills-ratio form): the caller passes z' = c (thr - t) / a (c = sqrt(log2 e):
// own factors pre-scaled by -Lik::ob_scale, the dot seeded with Lik::ob_thr), and pad flags:
// pad entries are moved to z' = kPadZ (P == 1, g == 0, log2 P == 0) instead of being masked.
//     T = 0.5 erfc(|z|) (0 below 2^-25),  P = T on the tail side (code 0: z < 0; code 1:
//     z > 0) else 1 - T,  g = +-exp(-z^2) / (a sqrt(pi) P)  (+ for code 0, - for code 1)
// The reference forms P = F(hi - x) - F(lo - x) with F = 0.5 (1 + erf) and the +-1e5 clamp
// (qmc/quantization_model.py:32-38, :61): with one edge saturated that is F(z) for code 0 and
// 1 - F(z) for code 1, the same probability; this form evaluates it without the cancellation
// of 1 - F in the tail (the values agree to a few ulp where the reference is accurate, P well
// away from 0) and without erf's two polynomial branches: one exp2, two rcp, one log2 and a
// (3,4) rational per entry.  Codes: the one-bit kind reads code != 1 as code 0 (pads are 15).
template <int KIND, bool LOG>
__device__ __forceinline__ void lik_grad2(f2v t, int c0, int c1, bool pa, bool pb,
                                          const float2* __restrict__ edges, const Lik& c,
                                          f2v& log2P, f2v& g) {
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
  } else if (KIND == LIK_ONEBIT_SR) {
    f2v P;
    onebit_sr_pg(t, c, P, g);
    log2P = log2_2(P);
    (void)c0;
    (void)c1;
    (void)pa;
    (void)pb;
    (void)edges;
  } else if (KIND == LIK_ONEBIT) {
    f2v z = t;
    if (pa) z.x = kPadZ;
    if (pb) z.y = kPadZ;
    const f2v u = f2v{__builtin_fabsf(z.x), __builtin_fabsf(z.y)};
#if QSC_FTZ_SAT
    // T and E carried 2^-101 low: with f32 denormals flushed (the library's qsc_pass build
    // flag) a tail below 2^-25 underflows to exactly 0 in the products, no compare needed
    const f2v E = exp2_2(fma2(-z, z, splat2(kMillsLogK - 101.0f)));
#else
    const f2v E = exp2_2(fma2(-z, z, splat2(kMillsLogK)));  // kMillsK exp(-z^2)
#endif
    f2v N = u + splat2(kMillsN2);
    N = fma2(N, u, splat2(kMillsN1));
    N = fma2(N, u, splat2(kMillsN0));
    f2v D = u + splat2(kMillsD3);
    D = fma2(D, u, splat2(kMillsD2));
    D = fma2(D, u, splat2(kMillsD1));
    D = fma2(D, u, splat2(kMillsD0));
#if QSC_FTZ_SAT
    const f2v Ts = ((E * N) * rcp2(D)) * splat2(0x1p101f);
#else
    const f2v T = (E * N) * rcp2(D);
    const f2v Ts = f2v{T.x < kMillsTsat ? 0.0f : T.x, T.y < kMillsTsat ? 0.0f : T.y};
#endif
    const f2v Q = splat2(1.0f) - Ts;
    const bool z0 = (c0 != 1), z1 = (c1 != 1);
    const bool ta = (z.x < 0.0f) == z0, tb = (z.y < 0.0f) == z1;
    const f2v P = f2v{ta ? Ts.x : Q.x, tb ? Ts.y : Q.y};
    const f2v gm = (E * splat2(c.ob_kg)) * rcp2(P);
    g = f2v{z0 ? gm.x : -gm.x, z1 ? gm.y : -gm.y};
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

// Signed-row gather tables (include/qsc.h rowfmt 1) of `rows` factor rows: rows [0, rows) hold
// [+row, +thr'], the negated copies start at row sr_off(rows), a multiple of 16 so that a row
// and its negation share a bank residue (qsc_sched.cuh), then kSrPadRows neutral pad rows
// 2 sr_off(rows) + r, one per residue r.
constexpr int kSrPadRows = 16;
__host__ __device__ inline int sr_off(int rows) { return (rows + 15) & ~15; }
__host__ __device__ inline int sr_rows(int rows) { return 2 * sr_off(rows) + kSrPadRows; }

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
  float rbc2;       // hardware rcp(bc2_sqrt): the reciprocal div_fix forms for that divisor
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
  s.rbc2 = __builtin_amdgcn_rcpf(s.bc2_sqrt);
  return s;
}

// The AdamScalars of one step, cached in the pass workspace: a launch whose step was prepared
// by the previous one reads 32 bytes instead of recomputing the double-precision bias
// corrections (a ~1 us dependent chain on one thread) at its start.  Two slots per side, chosen
// by step parity, so a record being written for step n+1 never overlaps the one read for step
// n.  A record is used only when its tag (step) and hyper-parameters match; anything else
// (zeroed workspace, another optimiser) falls back to adam_scalars.
struct AdamCache {
  int tag;  // kAdamTag ^ step
  float lr, b1, b2, eps;
  float step_size, bc2_sqrt, rbc2;
};
constexpr int kAdamTag = 0x51534341;

__device__ __forceinline__ AdamCache adam_cache_make(const qsc_adam& ad, int step,
                                                     const AdamScalars& s) {
  AdamCache c;
  c.tag = kAdamTag ^ step;
  c.lr = (float)ad.lr;
  c.b1 = (float)ad.beta1;
  c.b2 = (float)ad.beta2;
  c.eps = (float)ad.eps;
  c.step_size = s.step_size;
  c.bc2_sqrt = s.bc2_sqrt;
  c.rbc2 = s.rbc2;
  return c;
}

// the scalars of `step` from a record read earlier (either slot), or computed
__device__ __forceinline__ AdamScalars adam_scalars_cached(const AdamCache& c, const qsc_adam& ad,
                                                           int step) {
  if (c.tag == (kAdamTag ^ step) && c.lr == (float)ad.lr && c.b1 == (float)ad.beta1 &&
      c.b2 == (float)ad.beta2 && c.eps == (float)ad.eps) {
    AdamScalars s;
    s.step_size = c.step_size;
    s.bc2_sqrt = c.bc2_sqrt;
    s.rbc2 = c.rbc2;
    s.w1 = (float)(1.0 - ad.beta1);
    s.w2 = (float)(1.0 - ad.beta2);
    s.beta2 = (float)ad.beta2;
    s.eps = (float)ad.eps;
    return s;
  }
  return adam_scalars(ad, step);
}

__device__ __forceinline__ void adam_cache_store(AdamCache* slots, const qsc_adam& ad, int step) {
  slots[step & 1] = adam_cache_make(ad, step, adam_scalars(ad, step));
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

// adam_elem_fast on RH (even) consecutive row elements, two per packed instruction (the S-side
// Adam of the fused S-pass epilogue and of qsc_supdate), with the S regulariser folded in:
// g = a + p * coef.  Per element the same operations in the same order as adam_elem_fast (the
// bc2_sqrt reciprocal is the one div_fix forms), so the results are bitwise those of the scalar
// form.  proj: the projection onto S >= 0 after the step (qsc_adam::project_nonneg, the
// reference's C[C<0] = 0 form: -0 stays -0), before the norm.  Returns sum_j p_new[j]^2
// accumulated in j order.
template <int RH>
__device__ __forceinline__ float adam_row_fast(float (&p)[RH], float (&m)[RH], float (&v)[RH],
                                               const float (&a)[RH], float coef,
                                               const AdamScalars& s, bool proj) {
  float nsq = 0.0f;
#pragma unroll
  for (int j = 0; j < RH; j += 2) {
    const f2v pp = f2v{p[j], p[j + 1]}, aa = f2v{a[j], a[j + 1]};
    const f2v g = aa + pp * splat2(coef);
    f2v mm = f2v{m[j], m[j + 1]}, vv = f2v{v[j], v[j + 1]};
    mm = fma2(splat2(s.w1), g - mm, mm);
    vv = fma2(splat2(s.w2) * g, g, vv * splat2(s.beta2));
#if QSC_ADAM_S_EST
    // hardware sqrt / reciprocal estimates without the residual corrections (a few ulp from
    // torch's correctly rounded sqrt and divisions; experimental, QSC_ADAM_S_EST=1 builds)
    {
      const f2v sq = f2v{__builtin_amdgcn_sqrtf(vv.x), __builtin_amdgcn_sqrtf(vv.y)};
      const f2v den = fma2(sq, splat2(s.rbc2), splat2(s.eps));
      const f2v pn = fma2(splat2(-s.step_size) * mm, rcp2(den), pp);
      p[j] = (proj && pn.x < 0.0f) ? 0.0f : pn.x;
      p[j + 1] = (proj && pn.y < 0.0f) ? 0.0f : pn.y;
      m[j] = mm.x;
      m[j + 1] = mm.y;
      v[j] = vv.x;
      v[j + 1] = vv.y;
      continue;
    }
#endif
    // sqrt_fix
    const f2v sq = f2v{__builtin_amdgcn_sqrtf(vv.x), __builtin_amdgcn_sqrtf(vv.y)};
    const f2v er = fma2(-sq, sq, vv);
    const f2v hh = splat2(0.5f) * rcp2(sq);
    const f2v sf = fma2(er, hh, sq);
    const f2v sx = f2v{vv.x > 0.0f ? sf.x : sq.x, vv.y > 0.0f ? sf.y : sq.y};
    // div_fix(sx, bc2_sqrt) + eps
    const f2v q1 = sx * splat2(s.rbc2);
    const f2v r1 = fma2(-q1, splat2(s.bc2_sqrt), sx);
    const f2v den = fma2(r1, splat2(s.rbc2), q1) + splat2(s.eps);
    // div_fix(-step * m, den)
    const f2v x = splat2(-s.step_size) * mm;
    const f2v ry = rcp2(den);
    const f2v q2 = x * ry;
    const f2v r2 = fma2(-q2, den, x);
    const f2v pn = pp + fma2(r2, ry, q2);
    p[j] = (proj && pn.x < 0.0f) ? 0.0f : pn.x;
    p[j + 1] = (proj && pn.y < 0.0f) ? 0.0f : pn.y;
    m[j] = mm.x;
    m[j + 1] = mm.y;
    v[j] = vv.x;
    v[j + 1] = vv.y;
  }
#pragma unroll
  for (int j = 0; j < RH; ++j) nsq = __builtin_fmaf(p[j], p[j], nsq);
  return nsq;
}

}  // namespace qsc

// qsc_pass.hip — the fused one-bit / quantized probit likelihood + gradient passes (gfx950).
//
// Replaces, per alternating-solver iteration (qmc/qmc.ipynb cell 1, :559-634):
//   T_hat = get_tensor(S, C); T_hat = log(T_hat + offset);               (:568-571, :626-629)
//   nll = -sum(Wx * log(prob_probit(Y, T_hat, b, std)))                   (:572, :631)
//   cost = nll + lambda_c*||C|| + lambda_s*||S or Z||; cost.backward()     (:573-575, :632-633)
//   optimizer.step(); C[C<0] = 0                                          (:576, :579, :634)
// with explicit gradients (include/qsc.h) over observed entries only.
//
// Work mapping (wave64):
//   S-pass: one lane per pixel position; the lane walks its pixel's observed (k, code) list
//           (S-format); S[:,p] and dS[:,p] stay in registers, C[:,k] is gathered from LDS.
//           The Adam update of S is fused into the epilogue (no dS round trip through HBM).
//   C-pass: one lane per frequency bin k of a pixel tile; the lane walks the tile's observed
//           (pixel, code) list for its k (C-format); C[:,k] and dC[:,k] stay in registers,
//           S[:,p] is gathered from an LDS copy of the tile.  Per-tile dC partials go to a
//           slab that qsc_cfinish reduces in a fixed order (bitwise deterministic; no atomics).
#include "qsc_common.cuh"

using namespace qsc;

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

template <typename E>
struct Ent;
template <>
struct Ent<uint16_t> {
  static constexpr int kBits = 12;
  static constexpr uint32_t kMask = 0xFFF;
  static constexpr int kPad = 15;
  using V4 = uint2;  // 4 entries = 8 bytes
  __device__ static __forceinline__ void unpack(const V4& v, uint32_t (&e)[4]) {
    e[0] = v.x & 0xFFFF;
    e[1] = v.x >> 16;
    e[2] = v.y & 0xFFFF;
    e[3] = v.y >> 16;
  }
};
template <>
struct Ent<uint32_t> {
  static constexpr int kBits = 24;
  static constexpr uint32_t kMask = 0xFFFFFF;
  static constexpr int kPad = 255;
  using V4 = uint4;  // 4 entries = 16 bytes
  __device__ static __forceinline__ void unpack(const V4& v, uint32_t (&e)[4]) {
    e[0] = v.x;
    e[1] = v.y;
    e[2] = v.z;
    e[3] = v.w;
  }
};

// t = sum_r s[r]*c[r] in r order with separate roundings (get_tensor order, bit-identical)
template <int RP>
__device__ __forceinline__ float dot_ref(const float* s, const float* c) {
  float t = __fmul_rn(s[0], c[0]);
#pragma unroll
  for (int r = 1; r < RP; ++r) t = __fadd_rn(t, __fmul_rn(s[r], c[r]));
  return t;
}

struct Scalars {
  float coef;       // lambda / ||x||  (0 when ||x|| == 0, as torch's norm backward)
  AdamScalars as;
};

// ---------------------------------------------------------------------------------------
// S-pass
// ---------------------------------------------------------------------------------------
template <int RP, typename E, bool ADAM>
__global__ void __launch_bounds__(kBlock) spass_kernel(
    const E* __restrict__ ent, const int* __restrict__ width, const int64_t* __restrict__ off,
    int nslices, Probit pr, Edges E_, int R, int K, int Pp, float* __restrict__ S,
    const float* __restrict__ C, float* __restrict__ dS, float* __restrict__ mS,
    float* __restrict__ vS, qsc_adam ad, float lambda_s, qsc_state* __restrict__ st,
    float* __restrict__ part_nll, float* __restrict__ part_nsq) {
  using T = Ent<E>;
  // all LDS carved from the 16-B aligned dynamic region (no statics ahead of it)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  Scalars& sc = *reinterpret_cast<Scalars*>(smem);          // 32 B reserved
  float* Cl = smem + 8;                                      // [K][RP]
  float2* El = reinterpret_cast<float2*>(Cl + (size_t)K * RP);  // [nbins]

  for (int i = threadIdx.x; i < K * RP; i += blockDim.x) {
    const int k = i / RP, r = i - k * RP;
    Cl[i] = (r < R) ? C[(int64_t)r * K + k] : 0.0f;
  }
  for (int i = threadIdx.x; i < pr.nbins; i += blockDim.x) El[i] = E_.e[i];
  if (ADAM && threadIdx.x == 0) {
    const float nsq = st->normsq_s;
    const float nrm = sqrtf(nsq);
    sc.coef = nrm > 0.0f ? lambda_s / nrm : 0.0f;
    sc.as = adam_scalars(ad, st->step_s + 1);
  }
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s = blockIdx.x * kWaves + wave;
  if (s >= nslices) return;
  const int q = s * 64 + lane;

  float sv[RP], acc[RP];
#pragma unroll
  for (int r = 0; r < RP; ++r) {
    sv[r] = (r < R) ? S[(int64_t)r * Pp + q] : 0.0f;
    acc[r] = 0.0f;
  }
  float nll = 0.0f;

  const int W4 = width[s] >> 2;
  const typename T::V4* src = reinterpret_cast<const typename T::V4*>(ent + off[s]) + lane;
  typename T::V4 cur = W4 > 0 ? src[0] : typename T::V4{};
  for (int j4 = 0; j4 < W4; ++j4) {
    typename T::V4 nxt = cur;
    if (j4 + 1 < W4) nxt = src[(j4 + 1) * 64];
    uint32_t e[4];
    T::unpack(cur, e);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int code = (int)(e[u] >> T::kBits);
      if (code != T::kPad) {
        const int k = (int)(e[u] & T::kMask);
        float c[RP];
#pragma unroll
        for (int r = 0; r < RP; r += 4) {
          const float4 cv = *reinterpret_cast<const float4*>(Cl + k * RP + r);
          c[r] = cv.x;
          c[r + 1] = cv.y;
          c[r + 2] = cv.z;
          c[r + 3] = cv.w;
        }
        const float t = dot_ref<RP>(sv, c);
        float P, g;
        entry_grad(t, code, El, pr, P, g);
        nll -= __logf(P);
#pragma unroll
        for (int r = 0; r < RP; ++r) acc[r] = __builtin_fmaf(g, c[r], acc[r]);
      }
    }
    cur = nxt;
  }

  nll = wave_sum(nll);
  if (ADAM) {
    float nsq = 0.0f;
#pragma unroll
    for (int r = 0; r < RP; ++r) {
      if (r < R) {
        const int64_t i = (int64_t)r * Pp + q;
        float p = sv[r], m = mS[i], v = vS[i];
        const float g = __fadd_rn(acc[r], __fmul_rn(p, sc.coef));
        adam_elem(p, m, v, g, ad, sc.as);
        S[i] = p;
        mS[i] = m;
        vS[i] = v;
        nsq = __builtin_fmaf(p, p, nsq);
      }
    }
    nsq = wave_sum(nsq);
    if (lane == 0) part_nsq[s] = nsq;
  } else {
#pragma unroll
    for (int r = 0; r < RP; ++r)
      if (r < R) dS[(int64_t)r * Pp + q] = acc[r];
  }
  if (lane == 0) part_nll[s] = nll;
}

// ---------------------------------------------------------------------------------------
// C-pass
// ---------------------------------------------------------------------------------------
template <int RP, typename E>
__global__ void __launch_bounds__(kBlock) cpass_kernel(
    const E* __restrict__ ent, const int* __restrict__ width, const int64_t* __restrict__ off,
    int nks, int PT, Probit pr, Edges E_, int R, int K, int Pp, const float* __restrict__ S,
    const float* __restrict__ C, float* __restrict__ slab, float* __restrict__ part_nll) {
  using T = Ent<E>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Sl = smem;                                          // [PT][RP]
  float2* El = reinterpret_cast<float2*>(smem + (size_t)PT * RP);  // [nbins]
  const int t = blockIdx.x;
  const int64_t q0 = (int64_t)t * PT;
  for (int i = threadIdx.x; i < PT * RP; i += blockDim.x) {
    const int r = i / PT, ql = i - r * PT;
    Sl[ql * RP + r] = (r < R) ? S[(int64_t)r * Pp + q0 + ql] : 0.0f;
  }
  for (int i = threadIdx.x; i < pr.nbins; i += blockDim.x) El[i] = E_.e[i];
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int Kp = nks * 64;
  for (int ks = wave; ks < nks; ks += kWaves) {
    const int k = ks * 64 + lane;
    float cv[RP], acc[RP];
#pragma unroll
    for (int r = 0; r < RP; ++r) {
      cv[r] = (r < R && k < K) ? C[(int64_t)r * K + k] : 0.0f;
      acc[r] = 0.0f;
    }
    float nll = 0.0f;
    const int64_t wi = (int64_t)t * nks + ks;
    const int W4 = width[wi] >> 2;
    const typename T::V4* src = reinterpret_cast<const typename T::V4*>(ent + off[wi]) + lane;
    typename T::V4 cur = W4 > 0 ? src[0] : typename T::V4{};
    for (int j4 = 0; j4 < W4; ++j4) {
      typename T::V4 nxt = cur;
      if (j4 + 1 < W4) nxt = src[(j4 + 1) * 64];
      uint32_t e[4];
      T::unpack(cur, e);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int code = (int)(e[u] >> T::kBits);
        if (code != T::kPad) {
          const int ql = (int)(e[u] & T::kMask);
          float s[RP];
#pragma unroll
          for (int r = 0; r < RP; r += 4) {
            const float4 v = *reinterpret_cast<const float4*>(Sl + ql * RP + r);
            s[r] = v.x;
            s[r + 1] = v.y;
            s[r + 2] = v.z;
            s[r + 3] = v.w;
          }
          const float tt = dot_ref<RP>(s, cv);
          float P, g;
          entry_grad(tt, code, El, pr, P, g);
          nll -= __logf(P);
#pragma unroll
          for (int r = 0; r < RP; ++r) acc[r] = __builtin_fmaf(g, s[r], acc[r]);
        }
      }
      cur = nxt;
    }
#pragma unroll
    for (int r = 0; r < RP; ++r)
      if (r < R) slab[((int64_t)t * R + r) * Kp + k] = acc[r];
    nll = wave_sum(nll);
    if (lane == 0) part_nll[wi] = nll;
  }
}

// ---------------------------------------------------------------------------------------
// C finish: fixed-order slab reduction (+ fused regulariser / Adam / projection)
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) cfinish_kernel(
    const float* __restrict__ slab, int ntiles, int nks, int R, int K, float* __restrict__ C,
    int mode, float* __restrict__ dC, float* __restrict__ mC, float* __restrict__ vC,
    qsc_adam ad, float lambda_c, const float* __restrict__ normsq_ext,
    qsc_state* __restrict__ st, const float* __restrict__ part_nll_c, int npart) {
  __shared__ float red[kWaves][64];
  __shared__ float shn[kWaves];
  __shared__ Scalars sc;
  const int Kp = nks * 64;
  const int r = blockIdx.x / nks, ks = blockIdx.x - r * nks;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int k = ks * 64 + lane;

  float a = 0.0f;
  for (int t = wave; t < ntiles; t += kWaves) a += slab[((int64_t)t * R + r) * Kp + k];
  red[wave][lane] = a;

  float nsq;
  if (mode == 1 && normsq_ext == nullptr) {
    // ||C||^2 of the current C, same fixed order in every block
    float s2 = 0.0f;
    for (int i = threadIdx.x; i < R * K; i += blockDim.x) s2 = __builtin_fmaf(C[i], C[i], s2);
    nsq = block_sum(s2, shn);
  } else {
    __syncthreads();
    nsq = normsq_ext ? *normsq_ext : 0.0f;
  }
  if (threadIdx.x == 0) {
    const float nrm = sqrtf(nsq);
    sc.coef = nrm > 0.0f ? lambda_c / nrm : 0.0f;
    sc.as = adam_scalars(ad, st->step_c + 1);
  }
  __syncthreads();
  if (wave == 0 && k < K) {
    float g = red[0][lane];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) g += red[w][lane];
    const int64_t i = (int64_t)r * K + k;
    if (mode == 1) {
      float p = C[i], m = mC[i], v = vC[i];
      g = __fadd_rn(g, __fmul_rn(p, sc.coef));
      adam_elem(p, m, v, g, ad, sc.as);
      C[i] = p;
      mC[i] = m;
      vC[i] = v;
    } else {
      dC[i] = g;
    }
  }
  if (blockIdx.x == 0) {
    float s = 0.0f;
    for (int i = threadIdx.x; i < npart; i += blockDim.x) s += part_nll_c[i];
    const float tot = block_sum(s, shn);
    if (threadIdx.x == 0) {
      st->nll_c = tot;
      if (mode == 1) st->normsq_c = nsq;
    }
  }
}

// ---------------------------------------------------------------------------------------
// S finish: scalars of the S-pass, counters, history
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) sfinish_kernel(const float* __restrict__ part_nll,
                                                      const float* __restrict__ part_nsq,
                                                      int nparts, int update_nsq,
                                                      int c_stepped, int s_stepped,
                                                      qsc_state* __restrict__ st,
                                                      float* __restrict__ hist, int hist_cap) {
  __shared__ float sh[16];
  float a = 0.0f, b = 0.0f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    a += part_nll[i];
    if (update_nsq) b += part_nsq[i];
  }
  const float nll = block_sum(a, sh);
  const float nsq = block_sum(b, sh);
  if (threadIdx.x == 0) {
    const int it = st->iter;
    if (hist && it < hist_cap) {
      hist[4 * it + 0] = st->nll_c;
      hist[4 * it + 1] = nll;
      hist[4 * it + 2] = st->normsq_c;
      hist[4 * it + 3] = st->normsq_s;
    }
    st->nll_s = nll;
    if (update_nsq) st->normsq_s = nsq;
    if (c_stepped) st->step_c += 1;
    if (s_stepped) st->step_s += 1;
    st->iter = it + 1;
  }
}

__global__ void __launch_bounds__(kBlock) adam_kernel(float* __restrict__ x,
                                                      float* __restrict__ mx,
                                                      float* __restrict__ vx,
                                                      const float* __restrict__ g, int64_t n,
                                                      qsc_adam ad, const int* __restrict__ step,
                                                      float lambda,
                                                      const float* __restrict__ normsq) {
  __shared__ Scalars sc;
  if (threadIdx.x == 0) {
    const float nrm = normsq ? sqrtf(*normsq) : 0.0f;
    sc.coef = (normsq && nrm > 0.0f) ? lambda / nrm : 0.0f;
    sc.as = adam_scalars(ad, *step + 1);
  }
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float p = x[i], m = mx[i], v = vx[i];
    const float gg = __fadd_rn(g[i], __fmul_rn(p, sc.coef));
    adam_elem(p, m, v, gg, ad, sc.as);
    x[i] = p;
    mx[i] = m;
    vx[i] = v;
  }
}

__global__ void state_init_kernel(qsc_state* st, const double* nsq_part, int nparts) {
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < nparts; ++i) s += nsq_part[i];
    qsc_state z{};
    z.normsq_s = (float)s;
    *st = z;
  }
}

__global__ void __launch_bounds__(kBlock) nsq_part_kernel(const float* __restrict__ x, int64_t n,
                                                          double* __restrict__ part) {
  __shared__ double sh[kWaves];
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double v = x[i];
    s += v * v;
  }
  const double r = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = r;
}

// ---- workspace layout ----
struct PassWs {
  float* slab;      // ntiles * R * Kp
  float* cnll;      // ntiles * nks
  float* snll;      // nslices
  float* snsq;      // nslices
  double* init;     // 256
};

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

PassWs carve(const qsc_obs_desc* d, int R, void* ws) {
  char* w = (char*)ws;
  PassWs p;
  const int64_t Kp = (int64_t)d->nks * 64;
  p.slab = (float*)w;
  w += al((size_t)d->ntiles * R * Kp * 4);
  p.cnll = (float*)w;
  w += al((size_t)d->ntiles * d->nks * 4);
  p.snll = (float*)w;
  w += al((size_t)(d->Pp / 64) * 4);
  p.snsq = (float*)w;
  w += al((size_t)(d->Pp / 64) * 4);
  p.init = (double*)w;
  return p;
}

size_t ws_bytes_for(const qsc_obs_desc* d, int R) {
  const int64_t Kp = (int64_t)d->nks * 64;
  return al((size_t)d->ntiles * R * Kp * 4) + al((size_t)d->ntiles * d->nks * 4) +
         2 * al((size_t)(d->Pp / 64) * 4) + al(256 * 8);
}

bool desc_ok(const qsc_obs_desc* d) {
  return d && d->K >= 1 && d->P >= 1 && d->Pp >= d->P && (d->Pp % 64) == 0 && d->PT >= 64 &&
         (d->PT % 64) == 0 && d->ntiles * d->PT == d->Pp && d->nks * 64 >= d->K &&
         d->nbins >= 1;
}

int rp_of(int R) { return R <= 4 ? 4 : (R <= 8 ? 8 : 16); }

}  // namespace

#define STREAM(s) reinterpret_cast<hipStream_t>(s)

extern "C" {

QSC_API size_t qsc_pass_workspace_bytes(const qsc_obs_desc* d, int32_t R) {
  if (!desc_ok(d) || R < 1 || R > QSC_MAX_R) return 0;
  return ws_bytes_for(d, R);
}

QSC_API int qsc_state_init(qsc_state* st, const float* S, int32_t R, int32_t Pp, void* ws,
                           size_t ws_bytes, void* stream) {
  if (!st || R < 1 || Pp < 1 || !ws || ws_bytes < 256 * sizeof(double)) return QSC_EINVAL;
  double* part = (double*)ws;
  const int nb = 256;
  if (S) {
    hipLaunchKernelGGL(nsq_part_kernel, dim3(nb), dim3(kBlock), 0, STREAM(stream), S,
                       (int64_t)R * Pp, part);
    QSC_CHECK_LAUNCH();
  } else {
    QSC_TRY(hipMemsetAsync(part, 0, nb * sizeof(double), STREAM(stream)));
  }
  hipLaunchKernelGGL(state_init_kernel, dim3(1), dim3(64), 0, STREAM(stream), st, part, nb);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

#define SPASS_LAUNCH(RPV, ET, AD)                                                            \
  hipLaunchKernelGGL((spass_kernel<RPV, ET, AD>), grid, dim3(kBlock), shm, s,                \
                     (const ET*)s_entries, s_width, s_off, nslices, pr, E, R, d->K, d->Pp, S, C, \
                     dS, mS, vS, ad, lambda_s, st, w.snll, w.snsq)

QSC_API int qsc_spass(const qsc_obs_desc* d, const void* s_entries, const int32_t* s_width,
                      const int64_t* s_off, const qsc_model* m, int32_t R, float* S,
                      const float* C, int32_t mode, float* dS, float* mS, float* vS,
                      const qsc_adam* adam, float lambda_s, qsc_state* st, void* ws,
                      size_t ws_bytes, void* stream) {
  if (!desc_ok(d) || !m || m->nbounds - 1 != d->nbins || R < 1 || R > QSC_MAX_R || !S || !C ||
      !s_width || !s_off || (d->s_entries > 0 && !s_entries) || !ws ||
      ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  if (mode == 0 && !dS) return QSC_EINVAL;
  if (mode == 1 && (!mS || !vS || !adam || !st)) return QSC_EINVAL;
  if (mode != 0 && mode != 1) return QSC_EINVAL;
  const int RP = rp_of(R);
  const size_t shm = 32 + (size_t)d->K * RP * 4 + (size_t)d->nbins * 8;
  if (shm > 160 * 1024) return QSC_EINVAL;
  PassWs w = carve(d, R, ws);
  Edges E;
  make_edges(m, &E);
  const Probit pr = make_probit(m);
  const int nslices = d->Pp / 64;
  const dim3 grid((unsigned)ceil_div(nslices, kWaves));
  qsc_adam ad{};
  if (adam) ad = *adam;
  hipStream_t s = STREAM(stream);
  const bool A = (mode == 1);
  if (d->wide) {
    if (RP == 4) { if (A) SPASS_LAUNCH(4, uint32_t, true); else SPASS_LAUNCH(4, uint32_t, false); }
    else if (RP == 8) { if (A) SPASS_LAUNCH(8, uint32_t, true); else SPASS_LAUNCH(8, uint32_t, false); }
    else { if (A) SPASS_LAUNCH(16, uint32_t, true); else SPASS_LAUNCH(16, uint32_t, false); }
  } else {
    if (RP == 4) { if (A) SPASS_LAUNCH(4, uint16_t, true); else SPASS_LAUNCH(4, uint16_t, false); }
    else if (RP == 8) { if (A) SPASS_LAUNCH(8, uint16_t, true); else SPASS_LAUNCH(8, uint16_t, false); }
    else { if (A) SPASS_LAUNCH(16, uint16_t, true); else SPASS_LAUNCH(16, uint16_t, false); }
  }
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

#define CPASS_LAUNCH(RPV, ET)                                                                \
  hipLaunchKernelGGL((cpass_kernel<RPV, ET>), dim3((unsigned)d->ntiles), dim3(kBlock), shm, s, \
                     (const ET*)c_entries, c_width, c_off, d->nks, d->PT, pr, E, R, d->K, d->Pp, \
                     S, C, w.slab, w.cnll)

QSC_API int qsc_cpass(const qsc_obs_desc* d, const void* c_entries, const int32_t* c_width,
                      const int64_t* c_off, const qsc_model* m, int32_t R, const float* S,
                      const float* C, void* ws, size_t ws_bytes, void* stream) {
  if (!desc_ok(d) || !m || m->nbounds - 1 != d->nbins || R < 1 || R > QSC_MAX_R || !S || !C ||
      !c_width || !c_off || (d->c_entries > 0 && !c_entries) || !ws ||
      ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  const int RP = rp_of(R);
  const size_t shm = (size_t)d->PT * RP * 4 + (size_t)d->nbins * 8;
  if (shm > 160 * 1024) return QSC_EINVAL;
  PassWs w = carve(d, R, ws);
  Edges E;
  make_edges(m, &E);
  const Probit pr = make_probit(m);
  hipStream_t s = STREAM(stream);
  if (d->wide) {
    if (RP == 4) CPASS_LAUNCH(4, uint32_t);
    else if (RP == 8) CPASS_LAUNCH(8, uint32_t);
    else CPASS_LAUNCH(16, uint32_t);
  } else {
    if (RP == 4) CPASS_LAUNCH(4, uint16_t);
    else if (RP == 8) CPASS_LAUNCH(8, uint16_t);
    else CPASS_LAUNCH(16, uint16_t);
  }
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_cfinish(const qsc_obs_desc* d, int32_t R, float* C, int32_t mode, float* dC,
                        float* mC, float* vC, const qsc_adam* adam, float lambda_c,
                        const float* normsq_c_ext, qsc_state* st, void* ws, size_t ws_bytes,
                        void* stream) {
  if (!desc_ok(d) || R < 1 || R > QSC_MAX_R || !C || !st || !ws || ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  if (mode == 0 && !dC) return QSC_EINVAL;
  if (mode == 1 && (!mC || !vC || !adam)) return QSC_EINVAL;
  if (mode != 0 && mode != 1) return QSC_EINVAL;
  PassWs w = carve(d, R, ws);
  qsc_adam ad{};
  if (adam) ad = *adam;
  hipLaunchKernelGGL(cfinish_kernel, dim3((unsigned)(R * d->nks)), dim3(kBlock), 0,
                     STREAM(stream), w.slab, d->ntiles, d->nks, R, d->K, C, mode, dC, mC, vC, ad,
                     lambda_c, normsq_c_ext, st, w.cnll, d->ntiles * d->nks);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_sfinish_ex(const qsc_obs_desc* d, int32_t R, qsc_state* st, float* hist,
                           int32_t hist_cap, int32_t update_normsq, int32_t c_stepped,
                           int32_t s_stepped, void* ws, size_t ws_bytes, void* stream) {
  if (!desc_ok(d) || R < 1 || R > QSC_MAX_R || !st || !ws || ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  PassWs w = carve(d, R, ws);
  hipLaunchKernelGGL(sfinish_kernel, dim3(1), dim3(1024), 0, STREAM(stream), w.snll, w.snsq,
                     d->Pp / 64, update_normsq, c_stepped, s_stepped, st, hist, hist_cap);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_sfinish(const qsc_obs_desc* d, int32_t R, qsc_state* st, float* hist,
                        int32_t hist_cap, void* ws, size_t ws_bytes, void* stream) {
  return qsc_sfinish_ex(d, R, st, hist, hist_cap, 1, 1, 1, ws, ws_bytes, stream);
}

QSC_API int qsc_adam_step(float* x, float* mx, float* vx, const float* g, int64_t n,
                          const qsc_adam* adam, const int32_t* step, float lambda,
                          const float* normsq, void* stream) {
  if (n < 0 || (n > 0 && (!x || !mx || !vx || !g)) || !adam || !step) return QSC_EINVAL;
  if (n == 0) return QSC_OK;
  const int64_t g0 = ceil_div(n, kBlock);
  const unsigned grid = (unsigned)(g0 > 8192 ? 8192 : g0);
  hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(kBlock), 0, STREAM(stream), x, mx, vx, g, n,
                     *adam, step, lambda, normsq);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

}  // extern "C"

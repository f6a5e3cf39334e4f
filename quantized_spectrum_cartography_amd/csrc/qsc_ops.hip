// qsc_ops.hip — elementwise model ops, reconstruction and reductions (gfx950).
//
// These back the reference's module-level functions one to one (see include/qsc.h for the
// file:line of each); the fused solver passes live in qsc_pass.hip.
#include <string.h>

#include "qsc_common.cuh"

using namespace qsc;

namespace {

constexpr int kBlock = 256;
constexpr int kReduceBlocks = 1024;  // fixed grid => fixed summation order

inline int grid_for(int64_t n, int per_thread = 1, int cap = 1 << 20) {
  int64_t g = ceil_div(n, (int64_t)kBlock * per_thread);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

struct Bounds {
  float b[QSC_MAX_BOUNDS];
};

// ---------------------------------------------------------------------------------------
// quantize: qmc/quantization_model.py:8-20 and qmc/quantization_model_log.py:9-21
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) quantize_kernel(const float* __restrict__ X,
                                                          const float* __restrict__ noise,
                                                          int64_t n, Bounds B, int nb,
                                                          float sigma, float offset,
                                                          int log_model,
                                                          int64_t* __restrict__ Y) {
  __shared__ float sb[QSC_MAX_BOUNDS];
  for (int i = threadIdx.x; i < nb; i += blockDim.x) sb[i] = B.b[i];
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float base = X[i];
    if (log_model) base = logf(__fadd_rn(base, offset));
    // X + randn*std: two separately rounded fp32 ops, exactly as the torch expression; no
    // noise (qsc_bin_codes): X already is the noisy observation
    const float x = noise ? __fadd_rn(base, __fmul_rn(noise[i], sigma)) : base;
    int64_t y = 0;
    // later bins overwrite earlier ones, as the reference's loop of masked assignments does
    for (int c = 1; c <= nb - 2; ++c) {
      const float lo = sb[c];
      const float hi = (c + 1 == nb - 1) ? __builtin_inff() : sb[c + 1];
      if (lo < x && x <= hi) y = c;
    }
    Y[i] = y;
  }
}

// ---------------------------------------------------------------------------------------
// prob_probit forward / backward, F_probit, ordinal -> mid-bin value
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) prob_probit_kernel(const int64_t* __restrict__ Y,
                                                             const float* __restrict__ Xh,
                                                             int64_t n, Edges E, Probit pr,
                                                             const float* __restrict__ gP,
                                                             float* __restrict__ out) {
  __shared__ float2 se[QSC_MAX_BOUNDS - 1];
  for (int i = threadIdx.x; i < pr.nbins; i += blockDim.x) se[i] = E.e[i];
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t y = Y[i];
    y = y < 0 ? 0 : (y >= pr.nbins ? pr.nbins - 1 : y);
    const int c = (int)y;
    const float2 e = se[c];
    const float x = Xh[i];
    const bool lo_sat = pr.lo_sat && c == 0;
    const bool hi_sat = pr.hi_sat && c == pr.nbins - 1 && !lo_sat;
    if (gP == nullptr) {
      float P, gx;
      probit_lik(x, e.x, e.y, lo_sat, hi_sat, pr, P, gx);
      out[i] = P;
    } else {
      // dP/dx = (exp(-w^2) - exp(-u^2)) * kgrad
      const float u = div_a(e.y - x, pr), w = div_a(e.x - x, pr);
      const float eu = hi_sat ? 0.0f : __expf(-u * u);
      const float ew = lo_sat ? 0.0f : __expf(-w * w);
      out[i] = gP[i] * ((ew - eu) * pr.kgrad);
    }
  }
}

__global__ void __launch_bounds__(kBlock) f_probit_kernel(const float* __restrict__ y, int64_t n,
                                                          Probit pr, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = phi_scaled(div_a(y[i], pr));
}

__global__ void __launch_bounds__(kBlock) ordinal_kernel(const int64_t* __restrict__ Y, int64_t n,
                                                         Bounds B, int nb,
                                                         float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t y = Y[i];
    y = y < 0 ? 0 : (y > nb - 2 ? nb - 2 : y);
    out[i] = __fdiv_rn(__fadd_rn(B.b[y], B.b[y + 1]), 2.0f);
  }
}

__global__ void __launch_bounds__(kBlock) pack_codes_kernel(const int64_t* __restrict__ Y,
                                                            const float* __restrict__ Wx,
                                                            int64_t n, int nbins,
                                                            uint8_t* __restrict__ codes,
                                                            int* __restrict__ bad) {
  int nbad = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float w = Wx ? Wx[i] : 1.0f;
    const int64_t y = Y[i];
    uint8_t c = QSC_UNOBSERVED;
    if (w != 0.0f) {
      if (w != 1.0f || y < 0 || y >= nbins) ++nbad;
      else c = (uint8_t)y;
    }
    codes[i] = c;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// ---------------------------------------------------------------------------------------
// reconstruction: T[k][p] = sum_r S[r][p] * C[r][k], accumulated in the reference's order
//   prod = 0; for r: prod += outer(S[r], C[r])      (qmc/quantization_model.py:79-86)
// thread = 4 consecutive pixels (16-B loads/stores), loop over a chunk of k; C[r][k] is
// wave-uniform and comes through the scalar cache.
// ---------------------------------------------------------------------------------------
constexpr int kRecK = 16;

template <int RM>
__global__ void __launch_bounds__(kBlock) reconstruct_kernel(const float* __restrict__ S,
                                                             const float* __restrict__ C, int R,
                                                             int P, int K,
                                                             float* __restrict__ T) {
  const int64_t p4 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 4;
  const int k0 = blockIdx.y * kRecK;
  if (p4 >= P) return;
  const bool full = (p4 + 4 <= P) && ((P & 3) == 0);
  float4 s[RM];
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    if (r < R) {
      if (full) s[r] = *reinterpret_cast<const float4*>(S + (int64_t)r * P + p4);
      else {
        float t[4];
        for (int q = 0; q < 4; ++q) t[q] = (p4 + q < P) ? S[(int64_t)r * P + p4 + q] : 0.0f;
        s[r] = make_float4(t[0], t[1], t[2], t[3]);
      }
    }
  }
  const int kend = min(K, k0 + kRecK);
  for (int k = k0; k < kend; ++k) {
    float4 acc;
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      if (r < R) {
        const float c = C[(int64_t)r * K + k];
        const float4 pr = make_float4(__fmul_rn(s[r].x, c), __fmul_rn(s[r].y, c),
                                      __fmul_rn(s[r].z, c), __fmul_rn(s[r].w, c));
        if (r == 0) acc = pr;
        else
          acc = make_float4(__fadd_rn(acc.x, pr.x), __fadd_rn(acc.y, pr.y),
                            __fadd_rn(acc.z, pr.z), __fadd_rn(acc.w, pr.w));
      }
    }
    float* dst = T + (int64_t)k * P + p4;
    if (full) *reinterpret_cast<float4*>(dst) = acc;
    else {
      const float a[4] = {acc.x, acc.y, acc.z, acc.w};
      for (int q = 0; q < 4; ++q)
        if (p4 + q < P) dst[q] = a[q];
    }
  }
}

// dS[r][p] = sum_k gT[k][p] * C[r][k]  (k ascending)
template <int RM>
__global__ void __launch_bounds__(kBlock) reconstruct_bwd_s_kernel(const float* __restrict__ gT,
                                                                   const float* __restrict__ C,
                                                                   int R, int P, int K,
                                                                   float* __restrict__ dS) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= P) return;
  float acc[RM];
#pragma unroll
  for (int r = 0; r < RM; ++r) acc[r] = 0.0f;
  for (int k = 0; k < K; ++k) {
    const float g = gT[(int64_t)k * P + p];
#pragma unroll
    for (int r = 0; r < RM; ++r)
      if (r < R) acc[r] = __builtin_fmaf(g, C[(int64_t)r * K + k], acc[r]);
  }
#pragma unroll
  for (int r = 0; r < RM; ++r)
    if (r < R) dS[(int64_t)r * P + p] = acc[r];
}

// dC partials: block (pixel chunk, k) sums gT[k][p]*S[r][p] over its pixels
constexpr int kBwdChunk = 8192;

template <int RM>
__global__ void __launch_bounds__(kBlock) reconstruct_bwd_c_kernel(const float* __restrict__ gT,
                                                                   const float* __restrict__ S,
                                                                   int R, int P, int K,
                                                                   float* __restrict__ part) {
  __shared__ float sh[kBlock / 64];
  const int k = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * kBwdChunk;
  const int64_t p1 = min((int64_t)P, p0 + kBwdChunk);
  float acc[RM];
#pragma unroll
  for (int r = 0; r < RM; ++r) acc[r] = 0.0f;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const float g = gT[(int64_t)k * P + p];
#pragma unroll
    for (int r = 0; r < RM; ++r)
      if (r < R) acc[r] = __builtin_fmaf(g, S[(int64_t)r * P + p], acc[r]);
  }
  for (int r = 0; r < R && r < RM; ++r) {
    const float v = block_sum(acc[r], sh);
    if (threadIdx.x == 0) part[((int64_t)blockIdx.x * R + r) * K + k] = v;
  }
}

__global__ void __launch_bounds__(kBlock) sum_partials_kernel(const float* __restrict__ part,
                                                              int nchunks, int64_t n,
                                                              float* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a = 0.0f;
  for (int c = 0; c < nchunks; ++c) a += part[(int64_t)c * n + i];
  out[i] = a;
}

// ---------------------------------------------------------------------------------------
// reductions (fixed grid, fixed order): NMSE / NMSE_LOG helpers and ||x||^2
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) diff_sumsq_kernel(const float* __restrict__ a,
                                                            const float* __restrict__ b,
                                                            int64_t n, int use_log, float off,
                                                            double* __restrict__ part) {
  __shared__ double sh[kBlock / 64];
  double s0 = 0.0, s1 = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float x = a[i], y = b[i];
    if (use_log) {
      x = logf(x + off);
      y = logf(y + off);
    }
    const double d = (double)x - (double)y;
    s0 += d * d;
    s1 += (double)y * (double)y;
  }
  const double r0 = block_sum(s0, sh);
  const double r1 = block_sum(s1, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = r0;
    part[2 * blockIdx.x + 1] = r1;
  }
}

// fused: t = reconstruct(S, C) on the fly, compared with Ttrue (never materialised)
template <int RM>
__global__ void __launch_bounds__(kBlock) map_diff_sumsq_kernel(
    const float* __restrict__ S, const float* __restrict__ C, const float* __restrict__ Tt,
    int R, int P, int K, int use_log, float off, double* __restrict__ part) {
  __shared__ double sh[kBlock / 64];
  double s0 = 0.0, s1 = 0.0;
  const int64_t n = (int64_t)P * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = i / P, p = i - k * P;
    float t = 0.0f;
#pragma unroll
    for (int r = 0; r < RM; ++r)
      if (r < R) {
        const float pr = __fmul_rn(S[(int64_t)r * P + p], C[(int64_t)r * K + k]);
        t = (r == 0) ? pr : __fadd_rn(t, pr);
      }
    float y = Tt[i];
    if (use_log) {
      t = logf(t + off);
      y = logf(y + off);
    }
    const double d = (double)t - (double)y;
    s0 += d * d;
    s1 += (double)y * (double)y;
  }
  const double r0 = block_sum(s0, sh);
  const double r1 = block_sum(s1, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = r0;
    part[2 * blockIdx.x + 1] = r1;
  }
}

// the solver's map NMSE history (qmc/qmc.ipynb :582, :637: NMSE(get_tensor(S, C), T_true) every
// iteration) inside the captured iteration sequence: S in the passes' position order (pixel p's
// row at position iperm[p]), run only when the device iteration counter is a multiple of
// `every` (all blocks exit otherwise, so the launch can sit in every iteration of a hipGraph)
template <int RM>
__global__ void __launch_bounds__(kBlock) map_track_kernel(
    const float* __restrict__ Sp, const int* __restrict__ iperm, int RP,
    const float* __restrict__ C, const float* __restrict__ Tt, int R, int P, int K, int use_log,
    float off, const qsc_state* __restrict__ st, int every, double* __restrict__ part) {
  __shared__ double sh[kBlock / 64];
  const int it = st->iter;
  if (every <= 0 || it <= 0 || it % every != 0) return;
  double s0 = 0.0, s1 = 0.0;
  const int64_t n = (int64_t)P * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = i / P, p = i - k * P;
    const float* row = Sp + (int64_t)iperm[p] * RP;
    float t = 0.0f;
#pragma unroll
    for (int r = 0; r < RM; ++r)
      if (r < R) {
        const float pr = __fmul_rn(row[r], C[(int64_t)r * K + k]);
        t = (r == 0) ? pr : __fadd_rn(t, pr);
      }
    float y = Tt[i];
    if (use_log) {
      t = logf(t + off);
      y = logf(y + off);
    }
    const double d = (double)t - (double)y;
    s0 += d * d;
    s1 += (double)y * (double)y;
  }
  const double r0 = block_sum(s0, sh);
  const double r1 = block_sum(s1, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = r0;
    part[2 * blockIdx.x + 1] = r1;
  }
}

__global__ void __launch_bounds__(kBlock) track_finish_kernel(const double* __restrict__ part,
                                                              int nparts,
                                                              const qsc_state* __restrict__ st,
                                                              int every, double* __restrict__ hist,
                                                              int cap) {
  __shared__ double sh[kBlock / 64];
  const int it = st->iter;
  if (every <= 0 || it <= 0 || it % every != 0) return;
  double s0 = 0.0, s1 = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    s0 += part[2 * i];
    s1 += part[2 * i + 1];
  }
  const double r0 = block_sum(s0, sh);
  const double r1 = block_sum(s1, sh);
  const int slot = it / every - 1;
  if (threadIdx.x == 0 && slot < cap) {
    hist[2 * slot] = r0;
    hist[2 * slot + 1] = r1;
  }
}

__global__ void __launch_bounds__(kBlock) finish_pairs_kernel(const double* __restrict__ part,
                                                              int nparts,
                                                              double* __restrict__ out2) {
  __shared__ double sh[kBlock / 64];
  double s0 = 0.0, s1 = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    s0 += part[2 * i];
    s1 += part[2 * i + 1];
  }
  const double r0 = block_sum(s0, sh);
  const double r1 = block_sum(s1, sh);
  if (threadIdx.x == 0) {
    out2[0] = r0;
    out2[1] = r1;
  }
}

__global__ void __launch_bounds__(kBlock) sumsq_kernel(const float* __restrict__ x, int64_t n,
                                                       double* __restrict__ part) {
  __shared__ double sh[kBlock / 64];
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double v = x[i];
    s += v * v;
  }
  const double r = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = r;
}

__global__ void __launch_bounds__(kBlock) sumsq_finish_kernel(const double* __restrict__ part,
                                                              int nparts, float* __restrict__ out) {
  __shared__ double sh[kBlock / 64];
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += part[i];
  const double r = block_sum(s, sh);
  if (threadIdx.x == 0) out[0] = (float)r;
}

// ---------------------------------------------------------------------------------------
// pixel permutation between natural and position order
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) perm_gather_kernel(const float* __restrict__ nat,
                                                             const int* __restrict__ perm, int R,
                                                             int RP, int P, int Pp,
                                                             float* __restrict__ pos) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)RP * Pp) return;
  const int64_t q = i / RP;
  const int r = (int)(i - q * RP);
  const int p = perm[q];
  pos[i] = (r < R && p >= 0 && p < P) ? nat[(int64_t)r * P + p] : 0.0f;
}

__global__ void __launch_bounds__(kBlock) perm_scatter_kernel(const float* __restrict__ pos,
                                                              const int* __restrict__ perm, int R,
                                                              int RP, int P, int Pp,
                                                              float* __restrict__ nat) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)RP * Pp) return;
  const int64_t q = i / RP;
  const int r = (int)(i - q * RP);
  const int p = perm[q];
  if (r < R && p >= 0 && p < P) nat[(int64_t)r * P + p] = pos[i];
}

}  // namespace

// =======================================================================================
// C ABI
// =======================================================================================
#define STREAM(s) reinterpret_cast<hipStream_t>(s)

#define DISPATCH_R(R, KERNEL, GRID, BLOCK, STREAMV, ...)                                 \
  do {                                                                                  \
    if ((R) <= 4) hipLaunchKernelGGL(KERNEL<4>, GRID, BLOCK, 0, STREAMV, __VA_ARGS__);   \
    else if ((R) <= 8) hipLaunchKernelGGL(KERNEL<8>, GRID, BLOCK, 0, STREAMV, __VA_ARGS__); \
    else hipLaunchKernelGGL(KERNEL<16>, GRID, BLOCK, 0, STREAMV, __VA_ARGS__);          \
  } while (0)

extern "C" {

QSC_API int qsc_version(void) { return 2; }  // 2: position-order factors are [Pp][RP]

QSC_API int qsc_rank_pad(int32_t R) {
  return (R < 1 || R > QSC_MAX_R) ? 0 : (R <= 4 ? 4 : (R <= 8 ? 8 : 16));
}

QSC_API const char* qsc_error_string(int code) {
  if (code == QSC_OK) return "success";
  if (code == QSC_EINVAL) return "invalid argument";
  if (code == QSC_EUNSUPPORTED) return "configuration not supported by this build";
  return hipGetErrorString((hipError_t)code);
}

QSC_API int qsc_device_check(int dev) {
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return (int)e;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return QSC_EINVAL;
  return QSC_OK;
}

static bool model_ok(const qsc_model* m) {
  return m && m->nbounds >= 2 && m->nbounds <= QSC_MAX_BOUNDS && m->sigma > 0.0;
}

QSC_API int qsc_quantize(const float* X, const float* noise, int64_t n, const qsc_model* m,
                         int64_t* Y, void* stream) {
  if (!model_ok(m) || n < 0 || (n > 0 && (!X || !noise || !Y))) return QSC_EINVAL;
  if (n == 0) return QSC_OK;
  Bounds B;
  for (int i = 0; i < m->nbounds; ++i) B.b[i] = m->bounds[i];
  hipLaunchKernelGGL(quantize_kernel, dim3(grid_for(n, 4, 8192)), dim3(kBlock), 0,
                     STREAM(stream), X, noise, n, B, m->nbounds, (float)m->sigma,
                     (float)m->offset, m->log_model, Y);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_bin_codes(const float* x, int64_t n, const qsc_model* m, int64_t* Y,
                          void* stream) {
  if (!model_ok(m) || n < 0 || (n > 0 && (!x || !Y))) return QSC_EINVAL;
  if (n == 0) return QSC_OK;
  Bounds B;
  for (int i = 0; i < m->nbounds; ++i) B.b[i] = m->bounds[i];
  hipLaunchKernelGGL(quantize_kernel, dim3(grid_for(n, 4, 8192)), dim3(kBlock), 0,
                     STREAM(stream), x, (const float*)nullptr, n, B, m->nbounds, 0.0f, 0.0f, 0,
                     Y);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_prob_probit(const int64_t* Y, const float* Xhat, int64_t n, const qsc_model* m,
                            float* P, void* stream) {
  if (!model_ok(m) || n < 0 || (n > 0 && (!Y || !Xhat || !P))) return QSC_EINVAL;
  if (n == 0) return QSC_OK;
  Edges E;
  make_edges(m, &E);
  hipLaunchKernelGGL(prob_probit_kernel, dim3(grid_for(n, 4, 8192)), dim3(kBlock), 0,
                     STREAM(stream), Y, Xhat, n, E, make_probit(m), (const float*)nullptr, P);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_prob_probit_bwd(const int64_t* Y, const float* Xhat, const float* gP, int64_t n,
                                const qsc_model* m, float* gX, void* stream) {
  if (!model_ok(m) || n < 0 || (n > 0 && (!Y || !Xhat || !gP || !gX))) return QSC_EINVAL;
  if (n == 0) return QSC_OK;
  Edges E;
  make_edges(m, &E);
  hipLaunchKernelGGL(prob_probit_kernel, dim3(grid_for(n, 4, 8192)), dim3(kBlock), 0,
                     STREAM(stream), Y, Xhat, n, E, make_probit(m), gP, gX);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_f_probit(const float* y, int64_t n, double sigma, float* out, void* stream) {
  if (n < 0 || sigma <= 0.0 || (n > 0 && (!y || !out))) return QSC_EINVAL;
  if (n == 0) return QSC_OK;
  qsc_model m{};
  m.nbounds = 2;
  m.sigma = sigma;
  hipLaunchKernelGGL(f_probit_kernel, dim3(grid_for(n, 4, 8192)), dim3(kBlock), 0,
                     STREAM(stream), y, n, make_probit(&m), out);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_obs_from_ordinal(const int64_t* Y, int64_t n, const qsc_model* m, float* out,
                                 void* stream) {
  if (!model_ok(m) || n < 0 || (n > 0 && (!Y || !out))) return QSC_EINVAL;
  if (n == 0) return QSC_OK;
  Bounds B;
  for (int i = 0; i < m->nbounds; ++i) B.b[i] = m->bounds[i];
  hipLaunchKernelGGL(ordinal_kernel, dim3(grid_for(n, 4, 8192)), dim3(kBlock), 0,
                     STREAM(stream), Y, n, B, m->nbounds, out);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_pack_codes(const int64_t* Y, const float* Wx, int64_t n, int32_t nbins,
                           uint8_t* codes, int32_t* bad, void* stream) {
  if (n < 0 || nbins < 1 || nbins > QSC_MAX_BOUNDS - 1 || (n > 0 && (!Y || !codes || !bad)))
    return QSC_EINVAL;
  if (n == 0) return QSC_OK;
  hipLaunchKernelGGL(pack_codes_kernel, dim3(grid_for(n, 4, 8192)), dim3(kBlock), 0,
                     STREAM(stream), Y, Wx, n, nbins, codes, bad);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_reconstruct(const float* S, const float* C, int32_t R, int32_t P, int32_t K,
                            float* T, void* stream) {
  if (R < 1 || R > QSC_MAX_R || P < 0 || K < 0 || ((int64_t)P * K > 0 && (!S || !C || !T)))
    return QSC_EINVAL;
  if ((int64_t)P * K == 0) return QSC_OK;
  dim3 grid((unsigned)ceil_div(ceil_div(P, 4), kBlock), (unsigned)ceil_div(K, kRecK));
  DISPATCH_R(R, reconstruct_kernel, grid, dim3(kBlock), STREAM(stream), S, C, R, P, K, T);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API size_t qsc_reconstruct_bwd_workspace_bytes(int32_t R, int32_t P, int32_t K) {
  return (size_t)ceil_div(P, kBwdChunk) * R * K * sizeof(float);
}

QSC_API int qsc_reconstruct_bwd(const float* gT, const float* S, const float* C, int32_t R,
                                int32_t P, int32_t K, float* dS, float* dC, void* ws,
                                size_t ws_bytes, void* stream) {
  if (R < 1 || R > QSC_MAX_R || P < 1 || K < 1 || !gT) return QSC_EINVAL;
  if (dS) {
    if (!C) return QSC_EINVAL;
    DISPATCH_R(R, reconstruct_bwd_s_kernel, dim3((unsigned)ceil_div(P, kBlock)), dim3(kBlock),
               STREAM(stream), gT, C, R, P, K, dS);
    QSC_CHECK_LAUNCH();
  }
  if (dC) {
    if (!S || !ws || ws_bytes < qsc_reconstruct_bwd_workspace_bytes(R, P, K)) return QSC_EINVAL;
    const int nch = (int)ceil_div(P, kBwdChunk);
    float* part = (float*)ws;
    DISPATCH_R(R, reconstruct_bwd_c_kernel, dim3((unsigned)nch, (unsigned)K), dim3(kBlock),
               STREAM(stream), gT, S, R, P, K, part);
    QSC_CHECK_LAUNCH();
    const int64_t n = (int64_t)R * K;
    hipLaunchKernelGGL(sum_partials_kernel, dim3((unsigned)ceil_div(n, kBlock)), dim3(kBlock), 0,
                       STREAM(stream), part, nch, n, dC);
    QSC_CHECK_LAUNCH();
  }
  return QSC_OK;
}

QSC_API size_t qsc_reduce_workspace_bytes(int64_t n) {
  (void)n;
  return (size_t)kReduceBlocks * 2 * sizeof(double);
}

QSC_API int qsc_diff_sumsq(const float* a, const float* b, int64_t n, int32_t use_log,
                           double offset, double* out2, void* ws, size_t ws_bytes,
                           void* stream) {
  if (n < 0 || !a || !b || !out2 || !ws || ws_bytes < qsc_reduce_workspace_bytes(n))
    return QSC_EINVAL;
  double* part = (double*)ws;
  hipLaunchKernelGGL(diff_sumsq_kernel, dim3(kReduceBlocks), dim3(kBlock), 0, STREAM(stream), a,
                     b, n, use_log, (float)offset, part);
  QSC_CHECK_LAUNCH();
  hipLaunchKernelGGL(finish_pairs_kernel, dim3(1), dim3(kBlock), 0, STREAM(stream), part,
                     kReduceBlocks, out2);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_map_diff_sumsq(const float* S, const float* C, const float* Ttrue, int32_t R,
                               int32_t P, int32_t K, int32_t use_log, double offset,
                               double* out2, void* ws, size_t ws_bytes, void* stream) {
  if (R < 1 || R > QSC_MAX_R || P < 1 || K < 1 || !S || !C || !Ttrue || !out2 || !ws ||
      ws_bytes < qsc_reduce_workspace_bytes(0))
    return QSC_EINVAL;
  double* part = (double*)ws;
  DISPATCH_R(R, map_diff_sumsq_kernel, dim3(kReduceBlocks), dim3(kBlock), STREAM(stream), S, C,
             Ttrue, R, P, K, use_log, (float)offset, part);
  QSC_CHECK_LAUNCH();
  hipLaunchKernelGGL(finish_pairs_kernel, dim3(1), dim3(kBlock), 0, STREAM(stream), part,
                     kReduceBlocks, out2);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_map_nmse_track(const float* S_pos, const int32_t* iperm, int32_t RP,
                               const float* C, const float* Ttrue, int32_t R, int32_t P,
                               int32_t K, int32_t use_log, double offset, const qsc_state* st,
                               int32_t every, double* hist, int32_t cap, void* ws,
                               size_t ws_bytes, void* stream) {
  if (R < 1 || R > QSC_MAX_R || RP < R || P < 1 || K < 1 || !S_pos || !iperm || !C || !Ttrue ||
      !st || every < 1 || !hist || cap < 0 || !ws || ws_bytes < qsc_reduce_workspace_bytes(0))
    return QSC_EINVAL;
  double* part = (double*)ws;
  DISPATCH_R(R, map_track_kernel, dim3(kReduceBlocks), dim3(kBlock), STREAM(stream), S_pos,
             iperm, RP, C, Ttrue, R, P, K, use_log, (float)offset, st, every, part);
  QSC_CHECK_LAUNCH();
  hipLaunchKernelGGL(track_finish_kernel, dim3(1), dim3(kBlock), 0, STREAM(stream), part,
                     kReduceBlocks, st, every, hist, cap);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_sumsq(const float* x, int64_t n, float* out, void* ws, size_t ws_bytes,
                      void* stream) {
  if (n < 0 || !x || !out || !ws || ws_bytes < qsc_reduce_workspace_bytes(n)) return QSC_EINVAL;
  double* part = (double*)ws;
  hipLaunchKernelGGL(sumsq_kernel, dim3(kReduceBlocks), dim3(kBlock), 0, STREAM(stream), x, n,
                     part);
  QSC_CHECK_LAUNCH();
  hipLaunchKernelGGL(sumsq_finish_kernel, dim3(1), dim3(kBlock), 0, STREAM(stream), part,
                     kReduceBlocks, out);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_perm_gather(const float* nat, const int32_t* perm, int32_t R, int32_t P,
                            int32_t Pp, float* pos, void* stream) {
  const int RP = qsc_rank_pad(R);
  if (RP == 0 || P < 1 || Pp < P || !nat || !perm || !pos) return QSC_EINVAL;
  const int64_t n = (int64_t)RP * Pp;
  hipLaunchKernelGGL(perm_gather_kernel, dim3((unsigned)ceil_div(n, kBlock)), dim3(kBlock), 0,
                     STREAM(stream), nat, perm, R, RP, P, Pp, pos);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_perm_scatter(const float* pos, const int32_t* perm, int32_t R, int32_t P,
                             int32_t Pp, float* nat, void* stream) {
  const int RP = qsc_rank_pad(R);
  if (RP == 0 || P < 1 || Pp < P || !nat || !perm || !pos) return QSC_EINVAL;
  const int64_t n = (int64_t)RP * Pp;
  hipLaunchKernelGGL(perm_scatter_kernel, dim3((unsigned)ceil_div(n, kBlock)), dim3(kBlock), 0,
                     STREAM(stream), pos, perm, R, RP, P, Pp, nat);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

}  // extern "C"

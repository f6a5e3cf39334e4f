// qsc_map.hip — spatial loss fields of the synthetic radio-map generator.
//
// Reference (MATLAB, text only): qmc/generate_map.m:80-113
//     loss_f = @(x,d,alpha) min(1,(x/d).^(-alpha));  d0 = 2
//     loss_mat = abs(Xgrid - location)               (Xgrid = x + 1i*y on a unit grid)
//     shadow_linear = 10.^(shadow/10)                (shadow: Shadowing_data, dB)
//     Sc{rr} = loss_f(loss_mat,d0,alpha).*shadow_linear;  Sc{rr} = Sc{rr}/norm(Sc{rr},'fro')
//     if dB: Sc{rr} = real(10*log10(Sc{rr}))
// The correlated shadowing field itself is drawn by circulant embedding + FFT on the host side
// of the package (maps.py); this file composes path loss x shadowing for all R emitters in one
// pass over the grid, reduces each field's squared norm in a fixed order (f64), and
// normalises.  HBM-bound elementwise work: 4 B read + 4 B written per pixel and emitter
// (+ one re-read for the normalisation).
#include <algorithm>

#include "qsc_common.cuh"

using namespace qsc;

namespace {

constexpr int kMapBlock = 256;

// S[r][i*J + j] = min(1, (d/d0)^-alpha_r) * 10^(shadow/10); part[r][blk] = block sum of S^2
__global__ void __launch_bounds__(kMapBlock) map_compose_kernel(
    const float* __restrict__ shadow, const float* __restrict__ loc,
    const float* __restrict__ alpha, int I, int J, float res, float d0, float* __restrict__ S,
    double* __restrict__ part) {
  __shared__ double sh[kMapBlock / 64];
  const int r = blockIdx.y;
  const int64_t P = (int64_t)I * J;
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float lx = loc[2 * r], ly = loc[2 * r + 1], a = alpha[r];
  double sq = 0.0;
  if (p < P) {
    const int i = (int)(p / J), j = (int)(p % J);
    const float dx = (float)j * res - lx, dy = (float)i * res - ly;
    const float d = sqrtf(dx * dx + dy * dy);
    // (d/d0)^(-alpha) >= 1 for d <= d0 (incl. d = 0, where pow gives +inf): min(1, .) = 1.
    // Both factors as one hardware exp2 (v_exp_f32 / v_log_f32, ~1 ulp):
    //   (d/d0)^-alpha * 10^(z/10) = 2^(-alpha log2(d/d0) + z log2(10)/10)
    const float lp = d > d0 ? -a * __builtin_amdgcn_logf(d / d0) : 0.0f;
    const float v =
        __builtin_amdgcn_exp2f(__builtin_fmaf(shadow[(int64_t)r * P + p], 0.33219280948873623f, lp));
    S[(int64_t)r * P + p] = v;
    sq = (double)v * (double)v;
  }
  sq = block_sum(sq, sh);
  if (threadIdx.x == 0) part[(int64_t)r * gridDim.x + blockIdx.x] = sq;
}

// inv[r] = 1 / ||S[r]||_F from the block partials (one workgroup per field, fixed order)
__global__ void __launch_bounds__(kMapBlock) map_norm_kernel(const double* __restrict__ part,
                                                             int nblk, float* __restrict__ inv,
                                                             float* __restrict__ norms) {
  __shared__ double sh[kMapBlock / 64];
  const int r = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) s += part[(int64_t)r * nblk + b];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    const double n = sqrt(s);
    inv[r] = n > 0.0 ? (float)(1.0 / n) : 0.0f;
    if (norms) norms[r] = (float)n;
  }
}

// S[r] *= inv[r], then optionally 10 log10
__global__ void __launch_bounds__(kMapBlock) map_normalize_kernel(const float* __restrict__ inv,
                                                                  int64_t P, int db,
                                                                  float* __restrict__ S) {
  const int r = blockIdx.y;
  const float sc = inv[r];
  float4* s4 = reinterpret_cast<float4*>(S + (int64_t)r * P);
  const int64_t P4 = (P % 4 == 0) ? P / 4 : 0;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < P4;
       q += (int64_t)gridDim.x * blockDim.x) {
    float4 v = s4[q];
    v.x *= sc;
    v.y *= sc;
    v.z *= sc;
    v.w *= sc;
    if (db) {
      v.x = 10.0f * log10f(v.x);
      v.y = 10.0f * log10f(v.y);
      v.z = 10.0f * log10f(v.z);
      v.w = 10.0f * log10f(v.w);
    }
    s4[q] = v;
  }
  for (int64_t p = 4 * P4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P;
       p += (int64_t)gridDim.x * blockDim.x) {
    float v = S[(int64_t)r * P + p] * sc;
    if (db) v = 10.0f * log10f(v);
    S[(int64_t)r * P + p] = v;
  }
}

}  // namespace

#define STREAM(s) reinterpret_cast<hipStream_t>(s)

extern "C" {

QSC_API size_t qsc_map_compose_workspace_bytes(int32_t R, int32_t I, int32_t J) {
  if (R < 1 || I < 1 || J < 1) return 0;
  return (size_t)R * ceil_div((int64_t)I * J, kMapBlock) * sizeof(double) + (size_t)R * 4;
}

QSC_API int qsc_map_compose(const float* shadow, const float* loc, const float* alpha, int32_t R,
                            int32_t I, int32_t J, float res, float d0, int32_t db, float* S,
                            float* norms, void* ws, size_t ws_bytes, void* stream) {
  if (R < 1 || I < 1 || J < 1 || !shadow || !loc || !alpha || !S || !ws || !(d0 > 0.0f) ||
      !(res > 0.0f) || ws_bytes < qsc_map_compose_workspace_bytes(R, I, J))
    return QSC_EINVAL;
  const int64_t P = (int64_t)I * J;
  const int nblk = (int)ceil_div(P, kMapBlock);
  hipStream_t s = STREAM(stream);
  hipLaunchKernelGGL(map_compose_kernel, dim3(nblk, R), dim3(kMapBlock), 0, s, shadow, loc, alpha,
                     I, J, res, d0, S, (double*)ws);
  QSC_CHECK_LAUNCH();
  float* inv = reinterpret_cast<float*>((char*)ws + (size_t)R * nblk * sizeof(double));
  hipLaunchKernelGGL(map_norm_kernel, dim3(R), dim3(kMapBlock), 0, s, (const double*)ws, nblk,
                     inv, norms);
  QSC_CHECK_LAUNCH();
  const int nb2 = (int)std::min<int64_t>(ceil_div(P, 4 * kMapBlock), 1024);
  hipLaunchKernelGGL(map_normalize_kernel, dim3(nb2, R), dim3(kMapBlock), 0, s,
                     (const float*)inv, P, db, S);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

}  // extern "C"

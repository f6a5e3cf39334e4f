// qsc_gram.hip — R x R normal equations on MFMA (gfx950 v_mfma_f32_16x16x4_f32).
//
// Reference (MATLAB, text only): backup/algorithms/NMF_SPA.m:18-19
//     pseudo_inverse_S = inv(Sm'*Sm)*Sm';  C = pseudo_inverse_S*Tm
// and the regularised least-squares C-update of backup/algorithms/joint_opt_ae.m:404-416
//     A = [Q'; lambda*I], c = argmin ||A c - [y; 0]||   (here without the non-negativity)
// i.e. C^T = (G + lambda^2 I)^-1 B with G = S_w S^T (R x R) and B = S_w T^T (R x K), both
// contractions over the I*J pixels.  Those contractions are the only GEMM-shaped work of the
// path, so they run on the f32-input MFMA (exact f32, one rounding per product):
//   lane l holds A[i = l&15][k = l>>4] and B[k = l>>4][j = l&15];
//   D[i][j] (16x16) lives as col = l&15, row = 4*(l>>4) + reg.
// Pixel slot k of one MFMA is pixel p0 + 4*(l>>4) + m for the m-th of four MFMAs fed by one
// 16-byte load, so A and B of a product always refer to the same pixel.
#include "qsc_common.cuh"

using namespace qsc;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kGBlock = 256;  // 4 waves
constexpr int kGBlocks = 512; // fixed grid: fixed summation order

__device__ __forceinline__ float4 ld4(const float* p, int64_t i, int64_t n) {
  if (i + 4 <= n) return *reinterpret_cast<const float4*>(p + i);
  float t[4];
  for (int q = 0; q < 4; ++q) t[q] = (i + q < n) ? p[i + q] : 0.0f;
  return make_float4(t[0], t[1], t[2], t[3]);
}

// rows_a: R rows of S (row = l&15); rows_b: either S (Gram) or 16 rows of T starting at k0.
// partial[blk][16][16] per block (waves summed in fixed order through LDS)
__global__ void __launch_bounds__(kGBlock) gram_kernel(const float* __restrict__ S,
                                                       const float* __restrict__ Bm,
                                                       const float* __restrict__ w, int R,
                                                       int P, int nb_rows, int64_t ldb,
                                                       int aligned,
                                                       float* __restrict__ partial) {
  __shared__ float red[4][16 * 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = lane & 15, kslot = lane >> 4;
  const int jb = blockIdx.y * 16;  // B row block (T rows = frequency bins)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const bool arow = row < R;
  const bool brow = (jb + row) < nb_rows;
  const float* a_ptr = S + (int64_t)row * P;
  const float* b_ptr = Bm + (int64_t)(jb + row) * ldb;
  // each wave iteration consumes 16 pixels (4 per k-slot, 4 MFMAs)
  const int64_t step = (int64_t)gridDim.x * 4 * 16;
  for (int64_t p0 = ((int64_t)blockIdx.x * 4 + wave) * 16; p0 < P; p0 += step) {
    const int64_t p = p0 + 4 * kslot;
    float4 a = arow ? (aligned ? *reinterpret_cast<const float4*>(a_ptr + p) : ld4(a_ptr, p, P))
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    if (!aligned && p >= P) a = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 b = brow ? (aligned ? *reinterpret_cast<const float4*>(b_ptr + p) : ld4(b_ptr, p, P))
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    if (w) {
      const float4 wv = aligned ? *reinterpret_cast<const float4*>(w + p) : ld4(w, p, P);
      a.x *= wv.x;
      a.y *= wv.y;
      a.z *= wv.z;
      a.w *= wv.w;
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  }
  // D[i][j]: col j = lane&15, row i = 4*(lane>>4) + reg
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) red[wave][(4 * kslot + reg) * 16 + row] = acc[reg];
  __syncthreads();
  for (int e = threadIdx.x; e < 256; e += blockDim.x) {
    const float v = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
    partial[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 256 + e] = v;
  }
}

// out[i][jb + j] for i < R, jb + j < nb_rows: sum of partials over blocks in a fixed order.
// Grid (nby, 4): a workgroup owns 64 of the 256 tile elements; its 4 waves take interleaved
// quarters of the blocks (memory-level parallelism), combined in a fixed order through LDS.
__global__ void __launch_bounds__(256) gram_reduce_kernel(const float* __restrict__ partial,
                                                          int nblk, int R, int nb_rows,
                                                          float* __restrict__ out) {
  __shared__ float sh[4][64];
  const int q = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int e = blockIdx.y * 64 + l;  // 16x16 element
  const int jb = blockIdx.x * 16;
  const float* src = partial + (int64_t)blockIdx.x * nblk * 256 + e;
  float s = 0.0f;
  for (int b = q; b < nblk; b += 4) s += src[(int64_t)b * 256];
  sh[q][l] = s;
  __syncthreads();
  if (q == 0) {
    const float t = ((sh[0][l] + sh[1][l]) + sh[2][l]) + sh[3][l];
    const int i = e >> 4, j = e & 15;
    if (i < R && jb + j < nb_rows) out[(int64_t)i * nb_rows + jb + j] = t;
  }
}

// X[R][K] = (G + lambda I)^-1 B, Cholesky in double, one workgroup
__global__ void __launch_bounds__(256) chol_solve_kernel(const float* __restrict__ G,
                                                         const float* __restrict__ B, int R,
                                                         int K, float lambda,
                                                         float* __restrict__ X) {
  __shared__ double L[QSC_MAX_R][QSC_MAX_R];
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = 1;
    for (int i = 0; i < R; ++i)
      for (int j = 0; j <= i; ++j) {
        double s = (double)G[i * R + j] + ((i == j) ? (double)lambda : 0.0);
        for (int q = 0; q < j; ++q) s -= L[i][q] * L[j][q];
        if (i == j) {
          if (s <= 0.0) ok = 0;
          L[i][i] = sqrt(s > 0.0 ? s : 1e-300);
        } else {
          L[i][j] = s / L[j][j];
        }
      }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    double y[QSC_MAX_R];
    for (int i = 0; i < R; ++i) {
      double s = B[(int64_t)i * K + k];
      for (int q = 0; q < i; ++q) s -= L[i][q] * y[q];
      y[i] = s / L[i][i];
    }
    for (int i = R - 1; i >= 0; --i) {
      double s = y[i];
      for (int q = i + 1; q < R; ++q) s -= L[q][i] * y[q];
      y[i] = s / L[i][i];
    }
    for (int i = 0; i < R; ++i) X[(int64_t)i * K + k] = ok ? (float)y[i] : __builtin_nanf("");
  }
}

}  // namespace

#define STREAM(s) reinterpret_cast<hipStream_t>(s)

extern "C" {

QSC_API size_t qsc_gram_workspace_bytes(int32_t R, int32_t P, int32_t K) {
  (void)R;
  (void)P;
  const int64_t nby = ceil_div(K > R ? K : R, 16);
  return (size_t)kGBlocks * nby * 256 * sizeof(float);
}

QSC_API int qsc_gram(const float* S, const float* w, int32_t R, int32_t P, float* G, void* ws,
                     size_t ws_bytes, void* stream) {
  if (R < 1 || R > QSC_MAX_R || P < 1 || !S || !G || !ws ||
      ws_bytes < (size_t)kGBlocks * 256 * sizeof(float))
    return QSC_EINVAL;
  const int aligned = (P % 16) == 0;
  hipLaunchKernelGGL(gram_kernel, dim3(kGBlocks, 1), dim3(kGBlock), 0, STREAM(stream), S, S, w, R,
                     P, R, (int64_t)P, aligned, (float*)ws);
  QSC_CHECK_LAUNCH();
  hipLaunchKernelGGL(gram_reduce_kernel, dim3(1, 4), dim3(256), 0, STREAM(stream), (const float*)ws,
                     kGBlocks, R, R, G);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_gram_rhs(const float* S, const float* T, const float* w, int32_t R, int32_t P,
                         int32_t K, float* B, void* ws, size_t ws_bytes, void* stream) {
  if (R < 1 || R > QSC_MAX_R || P < 1 || K < 1 || !S || !T || !B || !ws ||
      ws_bytes < qsc_gram_workspace_bytes(R, P, K))
    return QSC_EINVAL;
  const int aligned = (P % 16) == 0;
  const unsigned nby = (unsigned)ceil_div(K, 16);
  hipLaunchKernelGGL(gram_kernel, dim3(kGBlocks, nby), dim3(kGBlock), 0, STREAM(stream), S, T, w,
                     R, P, K, (int64_t)P, aligned, (float*)ws);
  QSC_CHECK_LAUNCH();
  hipLaunchKernelGGL(gram_reduce_kernel, dim3(nby, 4), dim3(256), 0, STREAM(stream),
                     (const float*)ws, kGBlocks, R, K, B);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_chol_solve(const float* G, const float* B, int32_t R, int32_t K, float lambda,
                           float* X, void* stream) {
  if (R < 1 || R > QSC_MAX_R || K < 1 || !G || !B || !X) return QSC_EINVAL;
  hipLaunchKernelGGL(chol_solve_kernel, dim3(1), dim3(256), 0, STREAM(stream), G, B, R, K,
                     lambda, X);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

}  // extern "C"

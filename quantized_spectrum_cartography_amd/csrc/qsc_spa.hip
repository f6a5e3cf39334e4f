// qsc_spa.hip — SPA warm start and the non-negative C-update.
//
// Reference (MATLAB, text only):
//   backup/algorithms/NMF_SPA.m:1-29   [C, Sm] = NMF_SPA(T, R): column-sum normalisation of
//                                      Tm = T', SPA picks R columns (frequency bins), C from the
//                                      pseudo-inverse of the picked columns, ColumnPositive,
//                                      C >= 0, unit-norm columns of C, Sm scaled by the norms
//   backup/algorithms/NMF_SPA.m:31-56  K = SPA(X, r): greedy max-norm column + projection
//   backup/algorithms/joint_opt_ae.m:404-417  C-update: per bin k, c = lsqnonneg([Q'; lambda I],
//                                      [y_k; 0])
//
// MI355X design.  The only O(K^2 * P) work is the K x K Gram of the data (T w) T^T: a SYRK on
// the f32 MFMA (v_mfma_f32_16x16x4_f32, exact f32 products), 64 x 64 output tiles, upper
// triangle of tile pairs only, the pixel axis split over enough chunks to fill 256 CUs, and a
// fixed-order chunk reduction (deterministic).  SPA then runs in Gram form: the residual
// R = (I - sum u u^T) X never materialises; with H = X^T X the projection is the rank-1 update
// H <- H - h_j h_j^T / H_jj, and only diag(H) and the picked columns are kept (O(R^2 K)).
// The C fit needs G[sel, sel] and G[sel, :] of the same Gram, so the data are read once.
// NNLS: Lawson-Hanson in normal-equation form (Bro & de Jong's FNNLS), one thread per bin k,
// R <= 16; same minimiser as lsqnonneg on the augmented matrix (strictly convex for lambda > 0).
#include <algorithm>
#include <cfloat>
#include <type_traits>

#include "qsc_common.cuh"

using namespace qsc;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kSyTile = 64;
constexpr int kSyBlock = 256;       // 4 waves, each a 32 x 32 quarter of the tile
constexpr int kSyTargetBlocks = 768;  // ~3 workgroups per CU
constexpr int kSpaMaxK = 4096;      // diag(H) in LDS (double)
constexpr int kNnlsThreads = 16;    // bins per workgroup (per-thread LDS factor storage)

__device__ __forceinline__ float4 ld4b(const float* p, int64_t i, int64_t n, bool vec) {
  if (vec && i + 4 <= n) return *reinterpret_cast<const float4*>(p + i);
  float t[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) t[q] = (i + q < n) ? p[i + q] : 0.0f;
  return make_float4(t[0], t[1], t[2], t[3]);
}

__device__ __forceinline__ void pair_of(int pair, int nt, int& ti, int& tj) {
  int t = 0;
  while (pair >= nt - t) {
    pair -= nt - t;
    ++t;
  }
  ti = t;
  tj = t + pair;
}

// partial[chunk][pair][64][64] = sum over the chunk's pixels of (T w)[ti-rows] T[tj-rows]^T.
// Grid: x = tile pair (fastest), y = pixel chunk, so the pairs that share a chunk's rows run
// together and the chunk is read from HBM once (the other pairs hit L2 / Infinity Cache).
// Each 64-pixel stage of the A (ti) and B (tj) row blocks is loaded with coalesced 16-byte
// loads (16 lanes per 256-byte row segment), the next stage is prefetched into registers while
// the MFMAs consume the current one out of LDS; wave w owns the 32 x 32 quarter
// (w >> 1, w & 1) of the tile = 2 x 2 MFMA 16 x 16 accumulators.
// F64: the same products on v_mfma_f64_16x16x4_f64 (f32 data widened, f64 accumulation) for
// the SPA, whose residual test (max ||r||^2 > 1e-12, NMF_SPA.m:40) needs a Gram accurate far
// below f32 rounding.
constexpr int kSyStage = 64;              // pixels per LDS stage
constexpr int kSyPitch = kSyStage + 4;    // LDS row pitch (floats)
constexpr int kSyLoads = kSyTile * kSyStage / 4 / kSyBlock;  // float4 per thread per block

template <bool F64>
__global__ void __launch_bounds__(kSyBlock) syrk_kernel(const float* __restrict__ T,
                                                        const float* __restrict__ w, int K,
                                                        int64_t P, int nt, int64_t csz,
                                                        int npairs, int vec,
                                                        void* __restrict__ partial_,
                                                        double* __restrict__ rs_part) {
  using Acc = typename std::conditional<F64, f64x4, f32x4>::type;
  using Out = typename std::conditional<F64, double, float>::type;
  __shared__ __attribute__((aligned(16))) float As[kSyTile * kSyPitch];
  __shared__ __attribute__((aligned(16))) float Bs[kSyTile * kSyPitch];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = lane & 15, kslot = lane >> 4;
  int ti, tj;
  pair_of(blockIdx.x, nt, ti, tj);
  const bool diag = ti == tj;
  const int64_t p_lo = (int64_t)blockIdx.y * csz;
  const int64_t p_hi = p_lo + csz < P ? p_lo + csz : P;
  // this thread's load slots: float4 f = threadIdx.x + 256 q -> row f >> 4, pixel 4 (f & 15)
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 ra[kSyLoads], rb[kSyLoads];
  auto fetch = [&](int64_t s0) {
#pragma unroll
    for (int q = 0; q < kSyLoads; ++q) {
      const int f = threadIdx.x + kSyBlock * q;
      const int r = f >> 4;
      const int64_t p = s0 + 4 * (f & 15);
      const int gra = ti * kSyTile + r, grb = tj * kSyTile + r;
      float4 va = gra < K ? ld4b(T + (int64_t)gra * P, p, p_hi, vec) : z4;
      if (w) {
        const float4 wv = ld4b(w, p, p_hi, vec);
        va.x *= wv.x;
        va.y *= wv.y;
        va.z *= wv.z;
        va.w *= wv.w;
      }
      ra[q] = va;
      if (!diag) rb[q] = grb < K ? ld4b(T + (int64_t)grb * P, p, p_hi, vec) : z4;
    }
  };
  Acc acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = Acc{0, 0, 0, 0};
  // diagonal tile: B = unweighted rows of the same block; keep both (the weight is on A only)
  float4 rbd[kSyLoads];
  auto fetch_diag_b = [&](int64_t s0) {
#pragma unroll
    for (int q = 0; q < kSyLoads; ++q) {
      const int f = threadIdx.x + kSyBlock * q;
      const int r = f >> 4;
      const int64_t p = s0 + 4 * (f & 15);
      const int g = ti * kSyTile + r;
      rbd[q] = (w && g < K) ? ld4b(T + (int64_t)g * P, p, p_hi, vec) : z4;
    }
  };
  if (p_lo < p_hi) {
    fetch(p_lo);
    if (diag && w) fetch_diag_b(p_lo);
  }
  const float* Bsrc = (diag && !w) ? As : Bs;
  const int ar = (wave >> 1) * 32, br = (wave & 1) * 32;
  // diagonal tiles also yield the (weighted) row sums of their block (the SPA's column-sum
  // normaliser), so the data are read once: wave 0, lane = row, summed out of LDS
  const bool do_rs = rs_part != nullptr && diag && wave == 0;
  double rsum = 0.0;
  for (int64_t s0 = p_lo; s0 < p_hi; s0 += kSyStage) {
#pragma unroll
    for (int q = 0; q < kSyLoads; ++q) {
      const int f = threadIdx.x + kSyBlock * q;
      *reinterpret_cast<float4*>(As + (f >> 4) * kSyPitch + 4 * (f & 15)) = ra[q];
      if (!diag) *reinterpret_cast<float4*>(Bs + (f >> 4) * kSyPitch + 4 * (f & 15)) = rb[q];
      else if (w) *reinterpret_cast<float4*>(Bs + (f >> 4) * kSyPitch + 4 * (f & 15)) = rbd[q];
    }
    __syncthreads();
    if (s0 + kSyStage < p_hi) {
      fetch(s0 + kSyStage);
      if (diag && w) fetch_diag_b(s0 + kSyStage);
    }
    if (do_rs) {
      float rl = 0.0f;  // 64 products of the stage in f32, then into the f64 total
#pragma unroll
      for (int c = 0; c < kSyStage; c += 4) {
        const float4 v = *reinterpret_cast<const float4*>(As + lane * kSyPitch + c);
        rl += (v.x + v.y) + (v.z + v.w);
      }
      rsum += (double)rl;
    }
#pragma unroll
    for (int sub = 0; sub < kSyStage / 16; ++sub) {
      float4 a[2], b[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        a[x] = *reinterpret_cast<const float4*>(As + (ar + 16 * x + row) * kSyPitch + 16 * sub +
                                                4 * kslot);
        b[x] = *reinterpret_cast<const float4*>(Bsrc + (br + 16 * x + row) * kSyPitch +
                                                16 * sub + 4 * kslot);
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          if constexpr (F64) {
            acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)a[x].x, (double)b[y].x,
                                                            acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)a[x].y, (double)b[y].y,
                                                            acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)a[x].z, (double)b[y].z,
                                                            acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)a[x].w, (double)b[y].w,
                                                            acc[x][y], 0, 0, 0);
          } else {
            acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x].x, b[y].x, acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x].y, b[y].y, acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x].z, b[y].z, acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x].w, b[y].w, acc[x][y], 0, 0, 0);
          }
        }
    }
    __syncthreads();
  }
  // D[i][j]: col j = lane&15; row i = 4*(lane>>4) + reg (f32), (lane>>4) + 4*reg (f64)
  Out* out = reinterpret_cast<Out*>(partial_) +
             ((int64_t)blockIdx.y * npairs + blockIdx.x) * (kSyTile * kSyTile);
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int i = ar + x * 16 + (F64 ? kslot + 4 * reg : 4 * kslot + reg);
        const int j = br + y * 16 + row;
        out[i * kSyTile + j] = acc[x][y][reg];
      }
  if (do_rs && ti * kSyTile + lane < K)
    rs_part[(int64_t)blockIdx.y * K + ti * kSyTile + lane] = rsum;
}

// G (K x K, both triangles) = sum over chunks in a fixed order (4 interleaved partial sums
// for memory-level parallelism, combined in a fixed order); grid (npairs, 16): one thread per
// tile element.  A diagonal tile is written from its upper half only, so G is exactly
// symmetric.
template <typename Out>
__global__ void __launch_bounds__(256) syrk_reduce_kernel(const Out* __restrict__ partial,
                                                          int nchunks, int npairs, int nt, int K,
                                                          Out* __restrict__ G) {
  int ti, tj;
  pair_of(blockIdx.x, nt, ti, tj);
  const int e = blockIdx.y * 256 + threadIdx.x;
  const int i = e / kSyTile, j = e % kSyTile;
  const int gi = ti * kSyTile + i, gj = tj * kSyTile + j;
  if (gi >= K || gj >= K || (ti == tj && i > j)) return;
  const int64_t stride = (int64_t)npairs * (kSyTile * kSyTile);
  const Out* src = partial + (int64_t)blockIdx.x * (kSyTile * kSyTile) + e;
  Out s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int c = 0;
  for (; c + 4 <= nchunks; c += 4) {
    s0 += src[(int64_t)c * stride];
    s1 += src[(int64_t)(c + 1) * stride];
    s2 += src[(int64_t)(c + 2) * stride];
    s3 += src[(int64_t)(c + 3) * stride];
  }
  for (; c < nchunks; ++c) s0 += src[(int64_t)c * stride];
  const Out s = (s0 + s1) + (s2 + s3);
  G[(int64_t)gi * K + gj] = s;
  G[(int64_t)gj * K + gi] = s;
}

// n[k] = sum over chunks of the syrk kernel's row-sum partials (fixed order)
__global__ void __launch_bounds__(256) rowsum_reduce_kernel(const double* __restrict__ rs_part,
                                                            int nchunks, int K,
                                                            double* __restrict__ n) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  double s = 0.0;
  for (int c = 0; c < nchunks; ++c) s += rs_part[(int64_t)c * K + k];
  n[k] = s;
}

// SPA in Gram form on the column-sum-normalised data (NMF_SPA.m:31-56).  One workgroup.
//   Hn[a][b] = G[a][b] / (n_a n_b);  dg = diag(residual Gram);  V[i] = i-th residual column of
//   Hn divided by sqrt of its norm, so that dg <- dg - V[i]^2 and h_j = Hn[:, j] - V^T V[:, j].
__global__ void __launch_bounds__(1024) spa_select_kernel(const double* __restrict__ G,
                                                          const double* __restrict__ n, int K,
                                                          int R, double* __restrict__ V,
                                                          int32_t* __restrict__ sel,
                                                          int32_t* __restrict__ count) {
  __shared__ double dg[kSpaMaxK];
  __shared__ double bv[16];
  __shared__ int bi[16];
  __shared__ int jsel;
  __shared__ double djsel;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  for (int k = tid; k < K; k += blockDim.x) {
    const double nk = n[k];
    dg[k] = nk != 0.0 ? G[(int64_t)k * K + k] / (nk * nk) : 0.0;
  }
  __syncthreads();
  int m = 0;
  for (int i = 0; i < R; ++i) {
    // argmax of dg, first index on ties (MATLAB max)
    double best = -1.0;
    int bidx = K;
    for (int k = tid; k < K; k += blockDim.x)
      if (dg[k] > best) {
        best = dg[k];
        bidx = k;
      }
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bidx, o, 64);
      if (ov > best || (ov == best && oi < bidx)) {
        best = ov;
        bidx = oi;
      }
    }
    if (lane == 0) {
      bv[wave] = best;
      bi[wave] = bidx;
    }
    __syncthreads();
    if (tid == 0) {
      double b = bv[0];
      int j = bi[0];
      for (int q = 1; q < nw; ++q)
        if (bv[q] > b || (bv[q] == b && bi[q] < j)) {
          b = bv[q];
          j = bi[q];
        }
      jsel = (b > 1e-12 && j < K) ? j : -1;  // while ... max(normR) > 1e-12
      djsel = b;
    }
    __syncthreads();
    const int j = jsel;
    if (j < 0) break;
    const double rs = 1.0 / sqrt(djsel);
    const double nj = n[j];
    for (int k = tid; k < K; k += blockDim.x) {
      const double nk = n[k];
      double h = (nk != 0.0) ? G[(int64_t)k * K + j] / (nk * nj) : 0.0;
      for (int q = 0; q < i; ++q) h -= V[(int64_t)q * K + k] * V[(int64_t)q * K + j];
      const double v = h * rs;
      V[(int64_t)i * K + k] = v;
    }
    __syncthreads();  // V[i] complete (workgroup-scope visibility of the global writes)
    for (int k = tid; k < K; k += blockDim.x) {
      const double v = V[(int64_t)i * K + k];
      const double d = dg[k] - v * v;
      dg[k] = d > 0.0 ? d : 0.0;
    }
    if (tid == 0) sel[i] = j;
    m = i + 1;
    __syncthreads();
  }
  for (int i = m + tid; i < R; i += blockDim.x) sel[i] = -1;
  if (tid == 0) *count = m;
}

// C (R x K, rows >= count zero) and d (R): NMF_SPA.m:17-26 in Gram form.
//   C' = inv(Sm'Sm) Sm' Tm = inv(G[sel,sel]) G[sel,:];  ColumnPositive (sign flip of a column
//   whose sum is negative);  C(C < 0) = 0;  [C, d] = ColumnNormalization(C)
__global__ void __launch_bounds__(256) spa_fit_kernel(const double* __restrict__ G,
                                                      const int32_t* __restrict__ sel,
                                                      const int32_t* __restrict__ count, int K,
                                                      int R, float* __restrict__ C,
                                                      float* __restrict__ d) {
  __shared__ double L[QSC_MAX_R][QSC_MAX_R];
  __shared__ double sh[4];
  __shared__ int ok;
  __shared__ double flip, scale;
  const int m = *count;
  if (threadIdx.x == 0) {
    ok = 1;
    for (int i = 0; i < m; ++i)
      for (int j = 0; j <= i; ++j) {
        double s = G[(int64_t)sel[i] * K + sel[j]];
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
    for (int i = 0; i < m; ++i) {
      double s = G[(int64_t)sel[i] * K + k];
      for (int q = 0; q < i; ++q) s -= L[i][q] * y[q];
      y[i] = s / L[i][i];
    }
    for (int i = m - 1; i >= 0; --i) {
      double s = y[i];
      for (int q = i + 1; q < m; ++q) s -= L[q][i] * y[q];
      y[i] = s / L[i][i];
    }
    for (int i = 0; i < R; ++i)
      C[(int64_t)i * K + k] = (i < m) ? (ok ? (float)y[i] : __builtin_nanf("")) : 0.0f;
  }
  for (int r = 0; r < R; ++r) {
    double s = 0.0;
    for (int k = threadIdx.x; k < K; k += blockDim.x) s += (double)C[(int64_t)r * K + k];
    s = block_sum(s, sh);
    if (threadIdx.x == 0) flip = (s < 0.0) ? -1.0 : 1.0;
    __syncthreads();
    double q2 = 0.0;
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
      float c = (float)(flip * (double)C[(int64_t)r * K + k]);
      c = c < 0.0f ? 0.0f : c;
      C[(int64_t)r * K + k] = c;
      q2 += (double)c * (double)c;
    }
    q2 = block_sum(q2, sh);
    if (threadIdx.x == 0) {
      const double nrm = sqrt(q2);
      d[r] = (float)nrm;
      scale = nrm > 0.0 ? 1.0 / nrm : 1.0;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < K; k += blockDim.x)
      C[(int64_t)r * K + k] = (float)((double)C[(int64_t)r * K + k] * scale);
    __syncthreads();
  }
}

// S[r][p] = mask(p) * T[sel_r][p] * d_r  (Sm = Tm(:, idx) .* d, transposed), zero rows >= count
__global__ void __launch_bounds__(256) spa_rows_kernel(const float* __restrict__ T,
                                                       const float* __restrict__ w,
                                                       const int32_t* __restrict__ sel,
                                                       const float* __restrict__ d, int64_t P,
                                                       int R, float* __restrict__ S) {
  const int r = blockIdx.y;
  const int j = sel[r];
  const float dr = d[r];
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P;
       p += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.0f;
    if (j >= 0 && (!w || w[p] != 0.0f)) v = T[(int64_t)j * P + p] * dr;
    S[(int64_t)r * P + p] = v;
  }
}

// ---------------------------------------------------------------------------------------
// NNLS (joint_opt_ae.m:409-417): x_k = argmin_{x >= 0} x^T (G + lambda I) x / 2 - b_k^T x,
// b_k = B[:, k].  Per-thread passive-set factors live in LDS as [slot][thread].
// ---------------------------------------------------------------------------------------
struct NnlsLds {
  double* L;   // R*R per thread
  double* x;   // R
  double* s;   // R
  double* b;   // R
  int* idx;    // R
};

__global__ void __launch_bounds__(kNnlsThreads) nnls_kernel(const float* __restrict__ G,
                                                             const float* __restrict__ B, int R,
                                                             int K, float lambda,
                                                             float* __restrict__ X) {
  extern __shared__ double lds[];
  constexpr int NT = kNnlsThreads;
  const int t = threadIdx.x;
  const int k = blockIdx.x * NT + t;
  double* Gs = lds;                             // R*R shared
  double* L = Gs + R * R;                       // [R*R][NT]
  double* x = L + (size_t)R * R * NT;           // [R][NT]
  double* s = x + (size_t)R * NT;
  double* b = s + (size_t)R * NT;
  double* w = b + (size_t)R * NT;
  int* idx = reinterpret_cast<int*>(w + (size_t)R * NT);  // [R][NT]
  for (int e = t; e < R * R; e += NT)
    Gs[e] = (double)G[e] + ((e / R == e % R) ? (double)lambda : 0.0);
  __syncthreads();
  if (k >= K) return;
#define AT(arr, i) arr[(size_t)(i) * NT + t]
  double bmax = 0.0;
  for (int i = 0; i < R; ++i) {
    AT(b, i) = (double)B[(int64_t)i * K + k];
    AT(x, i) = 0.0;
    AT(w, i) = AT(b, i);
    bmax = fmax(bmax, fabs(AT(b, i)));
  }
  const double tol = 10.0 * (double)FLT_EPSILON * (double)R * fmax(bmax, 1e-30);
  uint32_t passive = 0;
  bool fail = false;
  // s_P = G_PP^-1 b_P (Cholesky), s_Z = 0; false if G_PP is not positive definite
  auto solve_passive = [&]() -> bool {
    int mm = 0;
    for (int i = 0; i < R; ++i)
      if (passive >> i & 1u) AT(idx, mm++) = i;
    for (int a = 0; a < mm; ++a)
      for (int c = 0; c <= a; ++c) {
        double v = Gs[AT(idx, a) * R + AT(idx, c)];
        for (int q = 0; q < c; ++q) v -= AT(L, a * R + q) * AT(L, c * R + q);
        if (a == c) {
          if (!(v > 0.0)) return false;
          AT(L, a * R + a) = sqrt(v);
        } else {
          AT(L, a * R + c) = v / AT(L, c * R + c);
        }
      }
    for (int i = 0; i < R; ++i) AT(s, i) = 0.0;
    double y[QSC_MAX_R];
    for (int a = 0; a < mm; ++a) {
      double v = AT(b, AT(idx, a));
      for (int q = 0; q < a; ++q) v -= AT(L, a * R + q) * y[q];
      y[a] = v / AT(L, a * R + a);
    }
    for (int a = mm - 1; a >= 0; --a) {
      double v = y[a];
      for (int q = a + 1; q < mm; ++q) v -= AT(L, q * R + a) * y[q];
      y[a] = v / AT(L, a * R + a);
      AT(s, AT(idx, a)) = y[a];
    }
    return true;
  };
  for (int outer = 0; outer < 3 * R && !fail; ++outer) {
    int j = -1;
    double wbest = tol;
    for (int i = 0; i < R; ++i)
      if (!(passive >> i & 1u) && AT(w, i) > wbest) {
        wbest = AT(w, i);
        j = i;
      }
    if (j < 0) break;
    passive |= 1u << j;
    for (int inner = 0; inner <= R; ++inner) {
      if (!solve_passive()) {
        fail = true;
        break;
      }
      bool feasible = true;
      for (int i = 0; i < R; ++i)
        if ((passive >> i & 1u) && AT(s, i) <= 0.0) feasible = false;
      if (feasible) break;
      // step toward s until the first passive coordinate hits zero; it (and any other that
      // reaches <= 0) leaves the passive set
      double alpha = 2.0;
      int amin = -1;
      for (int i = 0; i < R; ++i)
        if ((passive >> i & 1u) && AT(s, i) <= 0.0) {
          const double xi = AT(x, i);
          const double a = xi / (xi - AT(s, i));
          if (a < alpha) {
            alpha = a;
            amin = i;
          }
        }
      for (int i = 0; i < R; ++i) {
        const double xi = AT(x, i) + alpha * (AT(s, i) - AT(x, i));
        AT(x, i) = xi;
        if ((passive >> i & 1u) && (i == amin || xi <= 0.0)) {
          passive &= ~(1u << i);
          AT(x, i) = 0.0;
        }
      }
    }
    if (fail) break;
    for (int i = 0; i < R; ++i) AT(x, i) = (passive >> i & 1u) ? AT(s, i) : 0.0;
    for (int i = 0; i < R; ++i) {
      double v = AT(b, i);
      for (int c = 0; c < R; ++c) v -= Gs[i * R + c] * AT(x, c);
      AT(w, i) = v;
    }
  }
  for (int i = 0; i < R; ++i)
    X[(int64_t)i * K + k] = fail ? __builtin_nanf("") : (float)AT(x, i);
#undef AT
}

__global__ void __launch_bounds__(256) cast_kernel(const double* __restrict__ a, int64_t n,
                                                   float* __restrict__ b) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    b[i] = (float)a[i];
}

struct SyrkPlan {
  int nt, npairs, nchunks;
  int64_t csz;
};

SyrkPlan syrk_plan(int K, int64_t P) {
  SyrkPlan pl;
  pl.nt = (int)ceil_div(K, kSyTile);
  pl.npairs = pl.nt * (pl.nt + 1) / 2;
  int64_t nc = ceil_div(kSyTargetBlocks, pl.npairs);
  nc = nc < 1 ? 1 : nc;
  const int64_t maxc = ceil_div(P, 64);
  nc = nc > maxc ? maxc : nc;
  pl.csz = round_up(ceil_div(P, nc), 64);
  pl.nchunks = (int)ceil_div(P, pl.csz);
  return pl;
}

size_t align_up(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

#define STREAM(s) reinterpret_cast<hipStream_t>(s)

extern "C" {

QSC_API size_t qsc_syrk_workspace_bytes(int32_t K, int32_t P) {
  if (K < 1 || P < 1) return 0;
  const SyrkPlan pl = syrk_plan(K, P);
  return (size_t)pl.nchunks * pl.npairs * kSyTile * kSyTile * sizeof(float);
}

QSC_API int qsc_syrk(const float* T, const float* w, int32_t K, int32_t P, float* G, void* ws,
                     size_t ws_bytes, void* stream) {
  if (K < 1 || P < 1 || !T || !G || !ws || ws_bytes < qsc_syrk_workspace_bytes(K, P))
    return QSC_EINVAL;
  const SyrkPlan pl = syrk_plan(K, P);
  const int vec = (P % 4 == 0) && ((uintptr_t)T % 16 == 0) && (!w || (uintptr_t)w % 16 == 0);
  hipLaunchKernelGGL(syrk_kernel<false>, dim3(pl.npairs, pl.nchunks), dim3(kSyBlock), 0,
                     STREAM(stream), T, w, K, (int64_t)P, pl.nt, pl.csz, pl.npairs, vec, ws,
                     (double*)nullptr);
  QSC_CHECK_LAUNCH();
  hipLaunchKernelGGL(syrk_reduce_kernel<float>, dim3(pl.npairs, 16), dim3(256), 0, STREAM(stream),
                     (const float*)ws, pl.nchunks, pl.npairs, pl.nt, K, G);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

// f64 Gram for the SPA (workspace: 2 x the f32 form's partials)
static int syrk64(const float* T, const float* w, int K, int P, double* G, double* n, void* ws,
                  hipStream_t s) {
  const SyrkPlan pl = syrk_plan(K, P);
  const int vec = (P % 4 == 0) && ((uintptr_t)T % 16 == 0) && (!w || (uintptr_t)w % 16 == 0);
  double* rs = reinterpret_cast<double*>((char*)ws + 2 * qsc_syrk_workspace_bytes(K, P));
  hipLaunchKernelGGL(syrk_kernel<true>, dim3(pl.npairs, pl.nchunks), dim3(kSyBlock), 0, s, T, w,
                     K, (int64_t)P, pl.nt, pl.csz, pl.npairs, vec, ws, rs);
  QSC_CHECK_LAUNCH();
  hipLaunchKernelGGL(syrk_reduce_kernel<double>, dim3(pl.npairs, 16), dim3(256), 0, s,
                     (const double*)ws, pl.nchunks, pl.npairs, pl.nt, K, G);
  QSC_CHECK_LAUNCH();
  hipLaunchKernelGGL(rowsum_reduce_kernel, dim3((unsigned)ceil_div(K, 256)), dim3(256), 0, s,
                     (const double*)rs, pl.nchunks, K, n);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API size_t qsc_spa_workspace_bytes(int32_t K, int32_t P, int32_t R) {
  if (K < 1 || P < 1 || R < 1) return 0;
  const SyrkPlan pl = syrk_plan(K, P);
  return align_up(2 * qsc_syrk_workspace_bytes(K, P) + (size_t)pl.nchunks * K * 8) +
         align_up((size_t)K * K * 8) +
         align_up((size_t)K * 8) + align_up((size_t)R * K * 8) + align_up((size_t)R * 4);
}

QSC_API int qsc_spa(const float* T, const float* w, int32_t K, int32_t P, int32_t R,
                    int32_t* sel, int32_t* count, float* C, float* S, float* G_out, void* ws,
                    size_t ws_bytes, void* stream) {
  if (K < 1 || K > kSpaMaxK || P < 1 || R < 1 || R > QSC_MAX_R || R > K || !T || !sel ||
      !count || !C || !S || !ws || ws_bytes < qsc_spa_workspace_bytes(K, P, R))
    return QSC_EINVAL;
  char* p = (char*)ws;
  void* syws = p;
  p += align_up(2 * qsc_syrk_workspace_bytes(K, P) + (size_t)syrk_plan(K, P).nchunks * K * 8);
  double* G = (double*)p;
  p += align_up((size_t)K * K * 8);
  double* n = (double*)p;
  p += align_up((size_t)K * 8);
  double* V = (double*)p;
  p += align_up((size_t)R * K * 8);
  float* d = (float*)p;
  hipStream_t s = STREAM(stream);
  const int e = syrk64(T, w, K, P, G, n, syws, s);
  if (e != QSC_OK) return e;
  hipLaunchKernelGGL(spa_select_kernel, dim3(1), dim3(1024), 0, s, (const double*)G,
                     (const double*)n, K, R, V, sel, count);
  QSC_CHECK_LAUNCH();
  hipLaunchKernelGGL(spa_fit_kernel, dim3(1), dim3(256), 0, s, (const double*)G,
                     (const int32_t*)sel, (const int32_t*)count, K, R, C, d);
  QSC_CHECK_LAUNCH();
  const unsigned gx = (unsigned)std::min<int64_t>(ceil_div(P, 256), 1024);
  hipLaunchKernelGGL(spa_rows_kernel, dim3(gx, R), dim3(256), 0, s, T, w, (const int32_t*)sel,
                     (const float*)d, (int64_t)P, R, S);
  QSC_CHECK_LAUNCH();
  if (G_out) {
    hipLaunchKernelGGL(cast_kernel, dim3(256), dim3(256), 0, s, (const double*)G, (int64_t)K * K,
                       G_out);
    QSC_CHECK_LAUNCH();
  }
  return QSC_OK;
}

QSC_API int qsc_nnls(const float* G, const float* B, int32_t R, int32_t K, float lambda,
                     float* X, void* stream) {
  if (R < 1 || R > QSC_MAX_R || K < 1 || !G || !B || !X || !(lambda >= 0.0f)) return QSC_EINVAL;
  const size_t shm = (size_t)R * R * 8 + (size_t)kNnlsThreads * ((size_t)R * R + 4 * R) * 8 +
                     (size_t)kNnlsThreads * R * 4;
  hipLaunchKernelGGL(nnls_kernel, dim3((unsigned)ceil_div(K, kNnlsThreads)), dim3(kNnlsThreads),
                     shm, STREAM(stream), G, B, R, K, lambda, X);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

}  // extern "C"

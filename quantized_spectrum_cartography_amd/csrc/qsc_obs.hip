// qsc_obs.hip — one-time packing of the observation tensor into the two sliced sparse formats
// read by the fused passes (layout documented in include/qsc.h, qsc_obs_desc).
//
// Why: the reference evaluates the likelihood on every (k, p) entry and multiplies the
// unobserved ones by Wx = 0 (qmc/qmc.ipynb :572, Wx ~ Bernoulli(f) per entry at :493).  At
// f = 0.1 that is 90 % wasted arithmetic and, on a 64-lane wavefront, 64-way divergence.  The
// passes instead walk only observed entries, one lane per pixel (S-pass) or per frequency bin
// (C-pass), so every gradient sum stays in registers.  Pixels are re-ordered by observation
// count (stable sort) so the 64 lanes of a slice carry near-equal work.
#include <hipcub/hipcub.hpp>

#include <vector>

#include "qsc_common.cuh"
#include "qsc_sched.cuh"

using namespace qsc;

namespace {

constexpr int kBlock = 256;

__global__ void __launch_bounds__(kBlock) count_kernel(const uint8_t* __restrict__ codes, int K,
                                                       int P, int* __restrict__ cnt) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= P) return;
  int c = 0;
  for (int k = 0; k < K; ++k) c += codes[(int64_t)k * P + p] != QSC_UNOBSERVED;
  cnt[p] = c;
}

__global__ void iota_kernel(int* __restrict__ v, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = i;
}

__global__ void fill_int_kernel(int* __restrict__ v, int n, int val) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = val;
}

// S-format slice widths: QSC_SLICE * round4(max count in the slice)
__global__ void __launch_bounds__(kBlock) s_width_kernel(const int* __restrict__ perm,
                                                         const int* __restrict__ cnt, int P,
                                                         int nslices, int* __restrict__ width,
                                                         int64_t* __restrict__ sizes) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nslices) return;
  int m = 0;
  for (int l = 0; l < QSC_SLICE; ++l) {
    const int p = perm[s * QSC_SLICE + l];
    if (p >= 0 && p < P) m = max(m, cnt[p]);
  }
  m = (m + 3) & ~3;
  width[s] = m;
  sizes[s] = (int64_t)m * QSC_SLICE;
}

// C-format layout of one pixel tile (one block per tile): per-bin counts via LDS integer atomics
// (order-independent), the tile's bins ordered by count, descending, ties by k (padding bins
// K..Kp-1 count -1, so they come last) -> c_kmap, and per-slice widths (the slice's first, i.e.
// longest, list rounded up to chunks of 4).  Sorting makes the 64 lists a C-pass wave walks in
// lockstep near-equal in length (include/qsc.h, C-format).
__global__ void __launch_bounds__(kBlock) c_layout_kernel(const uint8_t* __restrict__ codes,
                                                          const int* __restrict__ perm, int K,
                                                          int P, int PT, int nks,
                                                          int* __restrict__ width,
                                                          int64_t* __restrict__ sizes,
                                                          int* __restrict__ kmap) {
  extern __shared__ int lcnt[];  // [Kp] counts, then [Kp] bin order
  const int Kp = nks * 64;
  int* lord = lcnt + Kp;
  const int t = blockIdx.x;
  for (int i = threadIdx.x; i < Kp; i += blockDim.x) lcnt[i] = i < K ? 0 : -1;
  __syncthreads();
  for (int ql = threadIdx.x; ql < PT; ql += blockDim.x) {
    const int p = perm[tile_pos(t, ql, gridDim.x)];  // grid = one block per tile
    if (p < 0 || p >= P) continue;
    for (int k = 0; k < K; ++k)
      if (codes[(int64_t)k * P + p] != QSC_UNOBSERVED) atomicAdd(&lcnt[k], 1);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < Kp; k += blockDim.x) {
    const int c = lcnt[k];
    int rank = 0;
    for (int k2 = 0; k2 < Kp; ++k2) {
      const int c2 = lcnt[k2];
      rank += (c2 > c) || (c2 == c && k2 < k);
    }
    lord[rank] = k;
    kmap[(int64_t)t * Kp + rank] = k;
  }
  __syncthreads();
  for (int ks = threadIdx.x; ks < nks; ks += blockDim.x) {
    int m = max(lcnt[lord[ks * 64]], 0);
    m = (m + 3) & ~3;
    width[(int64_t)t * nks + ks] = m;
    sizes[(int64_t)t * nks + ks] = (int64_t)m * 64;
  }
}

template <typename E>
struct EntryTraits;
template <>
struct EntryTraits<uint16_t> {
  static constexpr int kBits = 12;
  static constexpr uint32_t kPad = 15;
};
template <>
struct EntryTraits<uint32_t> {
  static constexpr int kBits = 24;
  static constexpr uint32_t kPad = 255;
};

// chunked column-major slot of entry j of lane `lane` in a list group of `lanes` lanes
__device__ __forceinline__ int64_t slot(int64_t base, int lanes, int lane, int j) {
  return base + (int64_t)(j >> 2) * (lanes * 4) + lane * 4 + (j & 3);
}

// Entry values (include/qsc.h): code-field form  idx | code << KBITS  (pad: code PAD), or the
// signed-row form (rowfmt 1)  idx + (code == 1 ? sr_off(rows) : 0)  (pad: row 2 sr_off(rows)),
// where `rows` is the table's row count, K for the S-format and PT for the C-format
template <typename E>
__device__ __forceinline__ E entry_of(uint32_t idx, uint32_t code, int sr, int rows) {
  using Tr = EntryTraits<E>;
  return sr ? (E)(idx + (code == 1 ? (uint32_t)sr_off(rows) : 0u)) : (E)(idx | (code << Tr::kBits));
}
template <typename E>
__host__ __device__ __forceinline__ E pad_of(int sr, int rows) {
  using Tr = EntryTraits<E>;
  return sr ? (E)(2u * (uint32_t)sr_off(rows)) : (E)(Tr::kPad << Tr::kBits);
}
template <typename E>
__host__ __device__ __forceinline__ SchedFmt sched_fmt(int sr, int rows) {
  SchedFmt f;
  f.pad_base = (uint32_t)pad_of<E>(sr, rows);
  f.rows = (uint32_t)rows;
  f.sr = sr;
  f.bits = EntryTraits<E>::kBits;
  return f;
}

// Bank-conflict-free list order (qsc_sched.cuh), one wave per 16-lane group of one list block
// (S-format: a slice's 32 position lists = 2 groups; C-format: a (tile, k-slice) block's 64 bin
// lists = 4 groups), its scratch in LDS, worked by lane 0 (a serial edge colouring, run once
// per packing).  `in` is a copy of the naturally ordered entries, `out` the packed array; blocks
// of lists longer than Wcap keep their natural order.
template <typename E>
__global__ void __launch_bounds__(64) sched_kernel(const E* __restrict__ in, E* __restrict__ out,
                                                   const int* __restrict__ width,
                                                   const int64_t* __restrict__ off, int lanes,
                                                   int Wcap, SchedFmt f) {
  extern __shared__ __attribute__((aligned(16))) char scratch[];
  const int groups = lanes / kSchedLanes;
  const int li = blockIdx.x / groups, g = blockIdx.x - li * groups;
  if (threadIdx.x != 0) return;
  const int W = width[li];
  const int64_t base = off[li];
  auto slot = [&](int i, int j) -> int64_t {
    return base + (int64_t)(j >> 2) * (lanes * 4) + b128_group_lane(g, i) * 4 + (j & 3);
  };
  bool ok = true;
  if (W > 0) {
    auto get = [&](int i, int j) -> uint32_t { return (uint32_t)in[slot(i, j)]; };
    auto put = [&](int i, int c, uint32_t v) { out[slot(i, c)] = (E)v; };
    ok = W <= Wcap && sched_group(scratch, W, f, get, put);
  }
  if (ok) return;
  for (int i = 0; i < kSchedLanes; ++i)
    for (int j = 0; j < W; ++j) out[slot(i, j)] = in[slot(i, j)];
}

__global__ void width_max_kernel(const int* __restrict__ w, int n, int* __restrict__ out) {
  __shared__ int sh[256];
  int m = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) m = max(m, w[i]);
  sh[threadIdx.x] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] = max(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sh[0];
}

// pad entries after the last list (read-ahead tail, QSC_ENTRY_TAIL)
template <typename E>
__global__ void tail_fill_kernel(E* __restrict__ ent, int64_t start, int n, int sr, int rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ent[start + i] = pad_of<E>(sr, rows);
}

template <typename E>
__global__ void __launch_bounds__(kBlock) s_fill_kernel(const uint8_t* __restrict__ codes,
                                                        const int* __restrict__ perm, int K,
                                                        int P, int Pp,
                                                        const int* __restrict__ width,
                                                        const int64_t* __restrict__ off,
                                                        E* __restrict__ ent, int sr) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Pp) return;
  const int s = q / QSC_SLICE, lane = q % QSC_SLICE;
  const int W = width[s];
  const int64_t base = off[s];
  const int p = perm[q];
  int j = 0;
  if (p >= 0 && p < P) {
    for (int k = 0; k < K; ++k) {
      const uint8_t c = codes[(int64_t)k * P + p];
      if (c != QSC_UNOBSERVED)
        ent[slot(base, QSC_SLICE, lane, j++)] = entry_of<E>((uint32_t)k, c, sr, K);
    }
  }
  for (; j < W; ++j) ent[slot(base, QSC_SLICE, lane, j)] = pad_of<E>(sr, K);
}

template <typename E>
__global__ void __launch_bounds__(kBlock) c_fill_kernel(const uint8_t* __restrict__ codes,
                                                        const int* __restrict__ perm, int K,
                                                        int P, int PT, int nks,
                                                        const int* __restrict__ width,
                                                        const int64_t* __restrict__ off,
                                                        const int* __restrict__ kmap,
                                                        E* __restrict__ ent, int sr) {
  const int t = blockIdx.x;
  for (int kk = threadIdx.x; kk < nks * 64; kk += blockDim.x) {
    const int ks = kk >> 6, lane = kk & 63;
    const int64_t wi = (int64_t)t * nks + ks;
    const int W = width[wi];
    const int64_t base = off[wi];
    const int k = kmap[(int64_t)t * nks * 64 + kk];  // the bin of this lane (count-sorted)
    int j = 0;
    if (k < K) {
      for (int ql = 0; ql < PT; ++ql) {
        const int p = perm[tile_pos(t, ql, gridDim.x)];  // grid = one block per tile
        if (p < 0 || p >= P) continue;
        const uint8_t c = codes[(int64_t)k * P + p];
        if (c != QSC_UNOBSERVED)
          ent[slot(base, 64, lane, j++)] = entry_of<E>((uint32_t)ql, c, sr, PT);
      }
    }
    for (; j < W; ++j) ent[slot(base, 64, lane, j)] = pad_of<E>(sr, PT);
  }
}

struct LayoutWs {
  int64_t* s_sizes;
  int64_t* c_sizes;
  int64_t* totals;  // [3]: s_entries, c_entries, nnz
  void* cub;
  size_t cub_bytes;
};

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

size_t cub_scan_bytes(int n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (int64_t*)nullptr, (int64_t*)nullptr, n);
  return b;
}
size_t cub_reduce_bytes(int n) {
  size_t b = 0;
  (void)hipcub::DeviceReduce::Sum(nullptr, b, (int*)nullptr, (int64_t*)nullptr, n);
  return b;
}

}  // namespace

#define STREAM(s) reinterpret_cast<hipStream_t>(s)

extern "C" {

QSC_API int qsc_obs_count(const uint8_t* codes, int32_t K, int32_t P, int32_t* cnt, void* stream) {
  if (K < 1 || P < 1 || !codes || !cnt) return QSC_EINVAL;
  hipLaunchKernelGGL(count_kernel, dim3((unsigned)ceil_div(P, kBlock)), dim3(kBlock), 0,
                     STREAM(stream), codes, K, P, cnt);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API size_t qsc_obs_order_workspace_bytes(int32_t P) {
  size_t b = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, b, (int*)nullptr, (int*)nullptr,
                                               (int*)nullptr, (int*)nullptr, P);
  return align_up(b) + 3 * align_up((size_t)P * sizeof(int));
}

QSC_API int qsc_obs_order(const int32_t* cnt, int32_t P, int32_t Pp, int32_t* perm, void* ws,
                          size_t ws_bytes, void* stream) {
  if (P < 1 || Pp < P || !cnt || !perm || !ws || ws_bytes < qsc_obs_order_workspace_bytes(P))
    return QSC_EINVAL;
  size_t cub_b = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, cub_b, (int*)nullptr, (int*)nullptr,
                                               (int*)nullptr, (int*)nullptr, P);
  char* w = (char*)ws;
  void* cub = w;
  w += align_up(cub_b);
  int* keys_out = (int*)w;
  w += align_up((size_t)P * sizeof(int));
  int* vals_in = (int*)w;
  hipStream_t s = STREAM(stream);
  hipLaunchKernelGGL(iota_kernel, dim3((unsigned)ceil_div(P, kBlock)), dim3(kBlock), 0, s, vals_in, P);
  QSC_CHECK_LAUNCH();
  hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(cub, cub_b, cnt, keys_out, vals_in,
                                                              perm, P, 0, 32, s);
  if (e != hipSuccess) return (int)e;
  if (Pp > P) {
    hipLaunchKernelGGL(fill_int_kernel, dim3((unsigned)ceil_div(Pp - P, kBlock)), dim3(kBlock), 0,
                       s, perm + P, Pp - P, -1);
    QSC_CHECK_LAUNCH();
  }
  return QSC_OK;
}

QSC_API size_t qsc_obs_layout_workspace_bytes(int32_t K, int32_t P, int32_t PT) {
  const int64_t Pp = round_up(P, PT > 0 ? PT : 64);
  const int64_t ns = Pp / QSC_SLICE;
  const int64_t nt = ceil_div(Pp, PT > 0 ? PT : 64);
  const int64_t nc = nt * ceil_div(K, 64);
  size_t cb = cub_scan_bytes((int)(ns + 1));
  cb = std::max(cb, cub_scan_bytes((int)(nc + 1)));
  cb = std::max(cb, cub_reduce_bytes(P));
  return align_up((ns + 1) * 8) + align_up((nc + 1) * 8) + align_up(3 * 8) + align_up(cb);
}

QSC_API int qsc_obs_layout(const uint8_t* codes, int32_t K, int32_t P, int32_t PT, int32_t nbins,
                           const int32_t* perm, const int32_t* cnt, int32_t* s_width,
                           int64_t* s_off, int32_t* c_width, int64_t* c_off, int32_t* c_kmap,
                           void* ws, size_t ws_bytes, qsc_obs_desc* desc, void* stream) {
  if (K < 1 || P < 1 || PT < 64 || (PT & 63) || nbins < 1 || nbins > QSC_MAX_BOUNDS - 1 ||
      !codes || !perm || !cnt || !s_width || !s_off || !c_width || !c_off || !c_kmap || !desc ||
      !ws || ws_bytes < qsc_obs_layout_workspace_bytes(K, P, PT))
    return QSC_EINVAL;
  const int Pp = (int)round_up(P, PT);  // whole tiles; padding positions carry no entries
  const int ns = Pp / QSC_SLICE, nt = Pp / PT, nks = (int)ceil_div(K, 64);
  // c_layout_kernel's LDS (counts + order, 2 ints per bin) against the device's own limit
  int dev = 0, lds_max = 64 * 1024;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess &&
        v > 0)
      lds_max = v;
  }
  if ((int64_t)nks * 64 * 2 * sizeof(int) > lds_max) return QSC_EINVAL;
  const int wide = (K > 4096 || PT > 4096 || nbins > 15) ? 1 : 0;
  if (wide && ((int64_t)K >= (1 << 24) || (int64_t)PT >= (1 << 24))) return QSC_EINVAL;
  char* w = (char*)ws;
  int64_t* s_sizes = (int64_t*)w;
  w += align_up((size_t)(ns + 1) * 8);
  int64_t* c_sizes = (int64_t*)w;
  w += align_up((size_t)(nt * nks + 1) * 8);
  int64_t* totals = (int64_t*)w;
  w += align_up(3 * 8);
  void* cub = w;
  size_t cub_b = ws_bytes - (size_t)(w - (char*)ws);
  hipStream_t s = STREAM(stream);
  hipLaunchKernelGGL(s_width_kernel, dim3((unsigned)ceil_div(ns, kBlock)), dim3(kBlock), 0, s,
                     perm, cnt, P, ns, s_width, s_sizes);
  QSC_CHECK_LAUNCH();
  QSC_TRY(hipMemsetAsync(s_sizes + ns, 0, 8, s));
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(cub, cub_b, s_sizes, s_off, ns + 1, s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(c_layout_kernel, dim3((unsigned)nt), dim3(kBlock), nks * 64 * 2 * sizeof(int),
                     s, codes, perm, K, P, PT, nks, c_width, c_sizes, c_kmap);
  QSC_CHECK_LAUNCH();
  QSC_TRY(hipMemsetAsync(c_sizes + (int64_t)nt * nks, 0, 8, s));
  cub_b = ws_bytes - (size_t)((char*)cub - (char*)ws);
  e = hipcub::DeviceScan::ExclusiveSum(cub, cub_b, c_sizes, c_off, nt * nks + 1, s);
  if (e != hipSuccess) return (int)e;
  cub_b = ws_bytes - (size_t)((char*)cub - (char*)ws);
  e = hipcub::DeviceReduce::Sum(cub, cub_b, cnt, totals + 2, P, s);
  if (e != hipSuccess) return (int)e;
  QSC_TRY(hipMemcpyAsync(totals, s_off + ns, 8, hipMemcpyDeviceToDevice, s));
  QSC_TRY(hipMemcpyAsync(totals + 1, c_off + (int64_t)nt * nks, 8, hipMemcpyDeviceToDevice, s));
  int64_t host_tot[3];
  e = hipMemcpyAsync(host_tot, totals, sizeof(host_tot), hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return (int)e;
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) return (int)e;
  desc->K = K;
  desc->P = P;
  desc->Pp = Pp;
  desc->PT = PT;
  desc->ntiles = nt;
  desc->nks = nks;
  desc->wide = wide;
  desc->nbins = nbins;
  desc->s_entries = host_tot[0] + QSC_ENTRY_TAIL;
  desc->c_entries = host_tot[1] + QSC_ENTRY_TAIL;
  desc->nnz = host_tot[2];
  desc->rowfmt = 0;
  desc->reserved_ = 0;
  return QSC_OK;
}

QSC_API int qsc_obs_fill(const uint8_t* codes, const qsc_obs_desc* d, const int32_t* perm,
                         const int32_t* s_width, const int64_t* s_off, const int32_t* c_width,
                         const int64_t* c_off, const int32_t* c_kmap, void* s_entries,
                         void* c_entries, void* stream) {
  if (!d || !codes || !perm || !s_width || !s_off || !c_width || !c_off || !c_kmap ||
      !s_entries || !c_entries || d->s_entries < QSC_ENTRY_TAIL || d->c_entries < QSC_ENTRY_TAIL)
    return QSC_EINVAL;
  // signed rows: narrow entries, every row index (up to the last pad row) representable
  const int sr = d->rowfmt == 1 ? 1 : 0;
  if (d->rowfmt != 0 && (d->rowfmt != 1 || d->wide || (int64_t)sr_rows(d->K) > 0x10000 ||
                         (int64_t)sr_rows(d->PT) > 0x10000 || d->nbins != 2))
    return QSC_EINVAL;
  hipStream_t s = STREAM(stream);
  const dim3 tg((QSC_ENTRY_TAIL + kBlock - 1) / kBlock), tb(kBlock);
  if (d->wide) {
    hipLaunchKernelGGL(tail_fill_kernel<uint32_t>, tg, tb, 0, s, (uint32_t*)s_entries,
                       d->s_entries - QSC_ENTRY_TAIL, QSC_ENTRY_TAIL, 0, d->K);
    hipLaunchKernelGGL(tail_fill_kernel<uint32_t>, tg, tb, 0, s, (uint32_t*)c_entries,
                       d->c_entries - QSC_ENTRY_TAIL, QSC_ENTRY_TAIL, 0, d->PT);
    hipLaunchKernelGGL(s_fill_kernel<uint32_t>, dim3((unsigned)ceil_div(d->Pp, kBlock)),
                       dim3(kBlock), 0, s, codes, perm, d->K, d->P, d->Pp, s_width, s_off,
                       (uint32_t*)s_entries, 0);
    QSC_CHECK_LAUNCH();
    hipLaunchKernelGGL(c_fill_kernel<uint32_t>, dim3((unsigned)d->ntiles), dim3(kBlock), 0, s,
                       codes, perm, d->K, d->P, d->PT, d->nks, c_width, c_off, c_kmap,
                       (uint32_t*)c_entries, 0);
  } else {
    hipLaunchKernelGGL(tail_fill_kernel<uint16_t>, tg, tb, 0, s, (uint16_t*)s_entries,
                       d->s_entries - QSC_ENTRY_TAIL, QSC_ENTRY_TAIL, sr, d->K);
    hipLaunchKernelGGL(tail_fill_kernel<uint16_t>, tg, tb, 0, s, (uint16_t*)c_entries,
                       d->c_entries - QSC_ENTRY_TAIL, QSC_ENTRY_TAIL, sr, d->PT);
    hipLaunchKernelGGL(s_fill_kernel<uint16_t>, dim3((unsigned)ceil_div(d->Pp, kBlock)),
                       dim3(kBlock), 0, s, codes, perm, d->K, d->P, d->Pp, s_width, s_off,
                       (uint16_t*)s_entries, sr);
    QSC_CHECK_LAUNCH();
    hipLaunchKernelGGL(c_fill_kernel<uint16_t>, dim3((unsigned)d->ntiles), dim3(kBlock), 0, s,
                       codes, perm, d->K, d->P, d->PT, d->nks, c_width, c_off, c_kmap,
                       (uint16_t*)c_entries, sr);
  }
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API size_t qsc_obs_schedule_workspace_bytes(const qsc_obs_desc* d) {
  if (!d || d->s_entries < 0 || d->c_entries < 0) return 0;
  const size_t eb = d->wide ? 4 : 2;
  return align_up((size_t)std::max(d->s_entries, d->c_entries) * eb) + 256;
}

QSC_API int qsc_obs_schedule(const qsc_obs_desc* d, const int32_t* s_width, const int64_t* s_off,
                             const int32_t* c_width, const int64_t* c_off, void* s_entries,
                             void* c_entries, void* ws, size_t ws_bytes, void* stream) {
  if (!d || !s_width || !s_off || !c_width || !c_off || !s_entries || !c_entries || !ws ||
      ws_bytes < qsc_obs_schedule_workspace_bytes(d) || (d->rowfmt != 0 && d->rowfmt != 1))
    return QSC_EINVAL;
  hipStream_t s = STREAM(stream);
  const size_t eb = d->wide ? 4 : 2;
  char* copy = (char*)ws;
  int* wmax = (int*)(copy + align_up((size_t)std::max(d->s_entries, d->c_entries) * eb));
  const int sr = d->rowfmt == 1 ? 1 : 0;
  for (int fmt = 0; fmt < 2; ++fmt) {
    // fmt 0: S-format (slices of QSC_SLICE position lists, rows = K); 1: C-format (64 bin
    // lists per (tile, k-slice) block, rows = PT)
    const int nl = fmt == 0 ? d->Pp / QSC_SLICE : d->ntiles * d->nks;
    const int lanes = fmt == 0 ? QSC_SLICE : 64;
    const int rows = fmt == 0 ? d->K : d->PT;
    const int* width = fmt == 0 ? s_width : c_width;
    const int64_t* off = fmt == 0 ? s_off : c_off;
    void* ent = fmt == 0 ? s_entries : c_entries;
    const int64_t n = fmt == 0 ? d->s_entries : d->c_entries;
    if (nl < 1 || n < 1) continue;
    hipLaunchKernelGGL(width_max_kernel, dim3(1), dim3(256), 0, s, width, nl, wmax);
    QSC_CHECK_LAUNCH();
    int host_w = 0;
    QSC_TRY(hipMemcpyAsync(&host_w, wmax, sizeof(int), hipMemcpyDeviceToHost, s));
    QSC_TRY(hipStreamSynchronize(s));
    const int wcap = std::min(host_w, kSchedMaxW);
    if (wcap < 1) continue;
    QSC_TRY(hipMemcpyAsync(copy, ent, (size_t)n * eb, hipMemcpyDeviceToDevice, s));
    const dim3 grid((unsigned)((int64_t)nl * (lanes / kSchedLanes)));
    const size_t shm = sched_scratch_bytes(wcap);
    if (d->wide)
      hipLaunchKernelGGL(sched_kernel<uint32_t>, grid, dim3(64), shm, s, (const uint32_t*)copy,
                         (uint32_t*)ent, width, off, lanes, wcap, sched_fmt<uint32_t>(0, rows));
    else
      hipLaunchKernelGGL(sched_kernel<uint16_t>, grid, dim3(64), shm, s, (const uint16_t*)copy,
                         (uint16_t*)ent, width, off, lanes, wcap, sched_fmt<uint16_t>(sr, rows));
    QSC_CHECK_LAUNCH();
  }
  return QSC_OK;
}

QSC_API int qsc_sched_lists_host(const uint32_t* in, uint32_t* out, int32_t W, int32_t rowfmt,
                                 int32_t rows, int32_t wide) {
  if (!in || !out || W < 0 || rows < 1 || (rowfmt != 0 && rowfmt != 1) || (rowfmt && wide))
    return QSC_EINVAL;
  const SchedFmt f = wide ? sched_fmt<uint32_t>(0, rows) : sched_fmt<uint16_t>(rowfmt, rows);
  if (W == 0) return QSC_OK;
  std::vector<unsigned char> scratch(sched_scratch_bytes(W) + 16);
  auto get = [&](int i, int j) -> uint32_t { return in[(size_t)i * W + j]; };
  auto put = [&](int i, int c, uint32_t v) { out[(size_t)i * W + c] = v; };
  if (sched_group(scratch.data(), W, f, get, put)) return QSC_OK;
  for (size_t i = 0; i < (size_t)kSchedLanes * W; ++i) out[i] = in[i];
  return 1;  // kept the natural order (W > kSchedMaxW)
}

}  // extern "C"

// Per-iteration cost of the global dependency of the alternating solver (every tile's dC partial
// -> C update -> every tile), with no pass arithmetic:
//   pair    : two launches per iteration (a 256 x 1024-thread "tile" kernel that writes an 8 KB
//             partial per workgroup, then a 32-workgroup "finish" kernel that reduces the 256
//             partials in a fixed order), captured in a hipGraph: today's kernel boundary form
//   barrier : ONE persistent launch, a grid barrier per iteration (8 group counters + 1 top
//             counter, relaxed agent-scope atomics, polled with agent-scope loads)
//   greduce : ONE persistent launch, per iteration every workgroup writes its 8 KB partial
//             write-through, the last arrival of each of 16 tile groups sums its group's 16
//             partials in a fixed order (write-through), and after the barrier EVERY workgroup
//             sums the 16 group partials itself (the same fixed order: bit-identical C on every
//             workgroup, no finish launch)
// Every poll is bounded (a timeout sets a fault word and the kernel leaves); the grid is at most
// one workgroup per CU and its co-residency is checked with the occupancy API first.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/grid_sync.hip -o tools/micro/grid_sync
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int kThreads = 1024;
constexpr int kCols = 2048;        // R x K floats of one partial (C3: 8 x 256)
constexpr int kGroups = 16;        // tile groups (vw = tile % 16)
constexpr long kMaxPolls = 1 << 22;

__device__ __forceinline__ unsigned long long ld_acq(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// grid barrier: 8 group counters on separate 128-B lines, the last arrival of a group bumps the
// top counter; everyone polls the top counter.  Counters count up for the life of the buffer.
__device__ bool grid_barrier(unsigned long long* ctr, int it, int* fault) {
  __shared__ int ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    ok = 1;
    const int g = blockIdx.x & 7;
    const unsigned long long ng = (gridDim.x - g + 7) / 8;
    const unsigned long long v =
        __hip_atomic_fetch_add(ctr + 16 * g, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v + 1 == (unsigned long long)(it + 1) * ng)
      __hip_atomic_fetch_add(ctr + 16 * 8, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long n = 0;
    while (ld_acq(ctr + 16 * 8) < (unsigned long long)(it + 1) * 8) {
      if (++n > kMaxPolls) {
        atomicExch(fault, 1);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return ok != 0;
}

__global__ void __launch_bounds__(kThreads) k_barrier(unsigned long long* ctr, int iters,
                                                       int* fault) {
  for (int it = 0; it < iters; ++it)
    if (!grid_barrier(ctr, it, fault)) return;
}

// greduce: partials [tile][kCols], group partials [g][kCols], result C [kCols] per workgroup
__global__ void __launch_bounds__(kThreads) k_greduce(unsigned long long* ctr, float* part,
                                                       float* gpart, float* out, int iters,
                                                       int* fault) {
  const int t = blockIdx.x, nt = gridDim.x, tid = threadIdx.x;
  __shared__ int last;
  float c0 = 1.0f + t, c1 = 2.0f + t;
  for (int it = 0; it < iters; ++it) {
    // the tile's partial (2 columns per thread), written through to the device-coherent level
    st_wt(part + (size_t)t * kCols + tid, c0 * 0.5f + it);
    st_wt(part + (size_t)t * kCols + tid + kThreads, c1 * 0.5f + it);
    __builtin_amdgcn_s_waitcnt(0);  // (vmcnt/vscnt: the stores have left)
    __syncthreads();
    const int g = t % kGroups;
    const int ng = (nt - g + kGroups - 1) / kGroups;
    if (tid == 0) {
      const unsigned long long v = __hip_atomic_fetch_add(ctr + 16 * (9 + g), 1ull,
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (v + 1 == (unsigned long long)(it + 1) * ng);
    }
    __syncthreads();
    if (last) {  // the group's partial, tiles g, g + 16, ... in order
      float a0 = 0.0f, a1 = 0.0f;
      for (int j = g; j < nt; j += kGroups) {
        a0 += ld_wt(part + (size_t)j * kCols + tid);
        a1 += ld_wt(part + (size_t)j * kCols + tid + kThreads);
      }
      st_wt(gpart + (size_t)g * kCols + tid, a0);
      st_wt(gpart + (size_t)g * kCols + tid + kThreads, a1);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (tid == 0)
        __hip_atomic_fetch_add(ctr + 16 * 8, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // wait for all 16 group partials
    if (tid == 0) {
      long n = 0;
      while (ld_acq(ctr + 16 * 8) < (unsigned long long)(it + 1) * kGroups) {
        if (++n > kMaxPolls) {
          atomicExch(fault, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    float s0 = 0.0f, s1 = 0.0f;
    for (int gg = 0; gg < kGroups; ++gg) {
      s0 += ld_wt(gpart + (size_t)gg * kCols + tid);
      s1 += ld_wt(gpart + (size_t)gg * kCols + tid + kThreads);
    }
    c0 = s0 * 1e-6f;
    c1 = s1 * 1e-6f;
    if (*fault) return;
    // every workgroup must have read the group partials before any rewrites them
    if (!grid_barrier(ctr + 16 * 32, it, fault)) return;
  }
  if (t == 0) {
    out[tid] = c0;
    out[tid + kThreads] = c1;
  }
}

// one launch per iteration: head = every workgroup sums the 16 group partials of the previous
// launch (plain loads: the kernel boundary publishes them), body = write this tile's partial
// write-through, tail = the last arrival of each group sums its group's 16 partials (sc1 buffer
// loads, all in flight) into this launch's group record (ping-pong: gin / gout)
__device__ __forceinline__ float ld_sc1(const float* base, unsigned off_bytes) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0,
                                                                     0x7fffffff, 0x00020000);
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off_bytes, 0, 16));  // sc1
}
__global__ void __launch_bounds__(kThreads) k_one(unsigned long long* ctr, float* part,
                                                   const float* gin, float* gout, float* cout) {
  const int t = blockIdx.x, nt = gridDim.x, tid = threadIdx.x;
  __shared__ int last;
  float s0 = 0.0f, s1 = 0.0f;
  {
    float v0[kGroups], v1[kGroups];
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
      v0[g] = gin[(size_t)g * kCols + tid];
      v1[g] = gin[(size_t)g * kCols + tid + kThreads];
    }
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
      s0 += v0[g];
      s1 += v1[g];
    }
  }
  if (t == 0) {
    cout[tid] = s0 * 1e-6f;
    cout[tid + kThreads] = s1 * 1e-6f;
  }
  st_wt(part + (size_t)t * kCols + tid, s0 * 0.5f + t);
  st_wt(part + (size_t)t * kCols + tid + kThreads, s1 * 0.5f + t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int g = t % kGroups;
  const int ng = (nt - g + kGroups - 1) / kGroups;
  if (tid == 0) {
    const unsigned long long v = __hip_atomic_fetch_add(ctr + 16 * g, 1ull, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
    last = ((v + 1) % (unsigned long long)ng) == 0;
  }
  __syncthreads();
  if (last) {
    float a0[kGroups], a1[kGroups];
#pragma unroll
    for (int j = 0; j < kGroups; ++j) {
      const int tt = min(g + j * kGroups, nt - 1);
      a0[j] = ld_sc1(part, (unsigned)(((size_t)tt * kCols + tid) * 4));
      a1[j] = ld_sc1(part, (unsigned)(((size_t)tt * kCols + tid + kThreads) * 4));
    }
    float x0 = 0.0f, x1 = 0.0f;
#pragma unroll
    for (int j = 0; j < kGroups; ++j)
      if (g + j * kGroups < nt) {
        x0 += a0[j];
        x1 += a1[j];
      }
    gout[(size_t)g * kCols + tid] = x0;
    gout[(size_t)g * kCols + tid + kThreads] = x1;
  }
}

// pair form: tile kernel + finish kernel
__global__ void __launch_bounds__(kThreads) k_tile(const float* cin, float* part) {
  const int t = blockIdx.x, tid = threadIdx.x;
  part[(size_t)t * kCols + tid] = cin[tid] * 0.5f + t;
  part[(size_t)t * kCols + tid + kThreads] = cin[tid + kThreads] * 0.5f + t;
}
__global__ void __launch_bounds__(kThreads) k_finish(const float* part, int nt, float* cout) {
  // 32 workgroups x 64 columns, 16 waves each summing tiles w, w + 16, ... then in order
  __shared__ float red[16][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
  float a = 0.0f;
  for (int j = w; j < nt; j += 16) a += part[(size_t)j * kCols + col];
  red[w][threadIdx.x & 63] = a;
  __syncthreads();
  if (w == 0) {
    float s = 0.0f;
    for (int i = 0; i < 16; ++i) s += red[i][threadIdx.x];
    cout[col] = s * 1e-6f;
  }
}

int main() {
  int dev = 0, ncu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  int occ_b = 0, occ_g = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_b, k_barrier, kThreads, 0));
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_g, k_greduce, kThreads, 0));
  const int nt = ncu;  // one workgroup per CU
  printf("CUs %d, occupancy barrier %d greduce %d, grid %d x %d\n", ncu, occ_b, occ_g, nt, kThreads);
  if (occ_b < 1 || occ_g < 1) return 2;
  unsigned long long* ctr;
  float *part, *gpart, *out, *cbuf;
  int* fault;
  CHECK(hipMalloc(&ctr, 1 << 16));
  CHECK(hipMalloc(&part, (size_t)nt * kCols * 4));
  CHECK(hipMalloc(&gpart, (size_t)kGroups * kCols * 4));
  CHECK(hipMalloc(&out, kCols * 4));
  CHECK(hipMalloc(&cbuf, kCols * 4));
  CHECK(hipMalloc(&fault, 4));
  CHECK(hipMemset(fault, 0, 4));
  CHECK(hipMemset(cbuf, 0, kCols * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int iters = 400;
  float ms = 0;

  // pair form in a graph
  hipGraph_t graph;
  hipGraphExec_t exec;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < iters; ++i) {
    hipLaunchKernelGGL(k_tile, dim3(nt), dim3(kThreads), 0, s, cbuf, part);
    hipLaunchKernelGGL(k_finish, dim3(kCols / 64), dim3(kThreads), 0, s, part, nt, cbuf);
  }
  CHECK(hipStreamEndCapture(s, &graph));
  CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  CHECK(hipGraphLaunch(exec, s));
  CHECK(hipStreamSynchronize(s));
  CHECK(hipEventRecord(e0, s));
  CHECK(hipGraphLaunch(exec, s));
  CHECK(hipEventRecord(e1, s));
  CHECK(hipEventSynchronize(e1));
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  printf("pair (tile + finish launches, hipGraph): %7.2f us / iteration\n", ms * 1e3f / iters);

  // one launch per iteration (head combine + group tail), ping-pong group records, in a graph
  {
    float* g2;
    CHECK(hipMalloc(&g2, (size_t)2 * kGroups * kCols * 4));
    CHECK(hipMemset(g2, 0, (size_t)2 * kGroups * kCols * 4));
    CHECK(hipMemset(ctr, 0, 1 << 16));
    hipGraph_t g1;
    hipGraphExec_t x1;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < iters; ++i) {
      float* gi = g2 + (size_t)(i & 1) * kGroups * kCols;
      float* go = g2 + (size_t)((i + 1) & 1) * kGroups * kCols;
      hipLaunchKernelGGL(k_one, dim3(nt), dim3(kThreads), 0, s, ctr, part, gi, go, cbuf);
    }
    CHECK(hipStreamEndCapture(s, &g1));
    CHECK(hipGraphInstantiate(&x1, g1, nullptr, nullptr, 0));
    CHECK(hipGraphLaunch(x1, s));
    CHECK(hipStreamSynchronize(s));
    CHECK(hipEventRecord(e0, s));
    CHECK(hipGraphLaunch(x1, s));
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("one launch (head combine + group tail, hipGraph): %7.2f us / iteration\n",
           ms * 1e3f / iters);
  }

  for (int rep = 0; rep < 2; ++rep) {
    CHECK(hipMemsetAsync(ctr, 0, 1 << 16, s));
    CHECK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(k_barrier, dim3(nt), dim3(kThreads), 0, s, ctr, iters, fault);
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    int f = 0;
    CHECK(hipMemcpy(&f, fault, 4, hipMemcpyDeviceToHost));
    printf("barrier (persistent, 8 + 1 counters): %7.2f us / iteration  fault %d\n",
           ms * 1e3f / iters, f);
    if (f) return 3;
    CHECK(hipMemsetAsync(ctr, 0, 1 << 16, s));
    CHECK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(k_greduce, dim3(nt), dim3(kThreads), 0, s, ctr, part, gpart, out, iters,
                       fault);
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipMemcpy(&f, fault, 4, hipMemcpyDeviceToHost));
    printf("greduce (persistent, group partials + per-WG reduce): %7.2f us / iteration  fault %d\n",
           ms * 1e3f / iters, f);
    if (f) return 3;
  }
  return 0;
}

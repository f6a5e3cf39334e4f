// First-load latency at a kernel's start (diagnostic, round 5): 256 workgroups of 1024 threads
// (the fused launch's grid) each read one 8 KB buffer (the C the fused launch stages), then a
// second 8 KB buffer, stamping the realtime clock (100 MHz) before and after each wait.  Cases:
//   written  : the buffer was written by the kernel just before (as cfinish writes C)
//   stale    : the buffer was last written long ago (several kernels before)
//   hot      : the same kernel run twice back to back, buffer untouched in between
// plus the same with each thread's row of a 32 MB array (the first-slice burst) in flight.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/first_load.hip -o tools/micro/first_load
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr int kBlocks = 256, kThreads = 1024;

__global__ void writer(float* c, int n, float v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) c[i] = v + i;
}

// t[4 * block + j]: j = 0 start, 1 after the first load landed, 2 after the burst landed
__global__ void __launch_bounds__(kThreads) reader(const float4* c, const float4* big, int nbig,
                                                   int burst, unsigned long long* t, float* sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
  if (burst) {
    const int i = (blockIdx.x * kThreads + threadIdx.x) % nbig;
    b = big[i];  // issued first, like the early waves' first-slice reads
  }
  const float4 x = c[threadIdx.x & 511];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const float s = x.x + x.y + x.z + x.w + b.x + b.y;
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    t[4 * blockIdx.x + 0] = t0;
    t[4 * blockIdx.x + 1] = t1;
  }
  if (s == 12345.678f) sink[blockIdx.x] = s;
}

static void report(const char* name, const std::vector<unsigned long long>& t) {
  unsigned long long g0 = ~0ull;
  for (int b = 0; b < kBlocks; ++b) g0 = std::min(g0, t[4 * b]);
  std::vector<double> lat, fin;
  for (int b = 0; b < kBlocks; ++b) {
    lat.push_back((t[4 * b + 1] - t[4 * b]) / 100.0);  // us (100 MHz)
    fin.push_back((t[4 * b + 1] - g0) / 100.0);
  }
  std::sort(lat.begin(), lat.end());
  std::sort(fin.begin(), fin.end());
  std::printf("%-28s block start->loaded+barrier: p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f us | "
              "from grid start: p50 %5.2f max %5.2f us\n",
              name, lat[kBlocks / 10], lat[kBlocks / 2], lat[kBlocks * 9 / 10], lat[kBlocks - 1],
              fin[kBlocks / 2], fin[kBlocks - 1]);
}

int main() {
  const int nc = 2048, nbig = 32 << 20 >> 4;  // 8 KB of floats; 32 MB of float4
  float *c, *c2, *sink;
  float4* big;
  unsigned long long* t;
  CHECK(hipMalloc(&c, nc * 4));
  CHECK(hipMalloc(&c2, nc * 4));
  CHECK(hipMalloc(&big, (size_t)nbig * 16));
  CHECK(hipMalloc(&sink, kBlocks * 4));
  CHECK(hipMalloc(&t, kBlocks * 4 * 8));
  CHECK(hipMemset(big, 0, (size_t)nbig * 16));
  std::vector<unsigned long long> h(kBlocks * 4);
  for (int burst = 0; burst < 2; ++burst) {
    for (int rep = 0; rep < 3; ++rep) {
      // written: the previous kernel wrote c
      hipLaunchKernelGGL(writer, dim3(34), dim3(1024), 0, 0, c, nc, 1.0f * rep);
      hipLaunchKernelGGL(reader, dim3(kBlocks), dim3(kThreads), 0, 0, (const float4*)c,
                         (const float4*)big, nbig, burst, t, sink);
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(h.data(), t, h.size() * 8, hipMemcpyDeviceToHost));
      report(burst ? "written, +burst" : "written", h);
      // stale: c2 was written before the previous several kernels
      hipLaunchKernelGGL(writer, dim3(34), dim3(1024), 0, 0, c2, nc, 2.0f);
      for (int k = 0; k < 4; ++k)
        hipLaunchKernelGGL(writer, dim3(34), dim3(1024), 0, 0, c, nc, 3.0f);
      hipLaunchKernelGGL(reader, dim3(kBlocks), dim3(kThreads), 0, 0, (const float4*)c2,
                         (const float4*)big, nbig, burst, t, sink);
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(h.data(), t, h.size() * 8, hipMemcpyDeviceToHost));
      report(burst ? "stale, +burst" : "stale", h);
      // hot: read twice back to back
      hipLaunchKernelGGL(reader, dim3(kBlocks), dim3(kThreads), 0, 0, (const float4*)c2,
                         (const float4*)big, nbig, burst, t, sink);
      hipLaunchKernelGGL(reader, dim3(kBlocks), dim3(kThreads), 0, 0, (const float4*)c2,
                         (const float4*)big, nbig, burst, t, sink);
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(h.data(), t, h.size() * 8, hipMemcpyDeviceToHost));
      report(burst ? "hot, +burst" : "hot", h);
    }
  }
  return 0;
}

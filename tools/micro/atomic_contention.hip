// Arrival-ticket cost: every workgroup of an N-workgroup grid takes one relaxed agent-scope
// atomic increment at about the same time, on ONE counter (the fused finish's ticket) or on one
// of 8 counters on separate 128-B lines (a per-group ticket).  Kernel time against N, against the
// same grid without the atomic.  Diagnostic for the fused-finish tail.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/atomic_contention.hip -o tools/micro/atomic_contention
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

// mode 0: no atomic; 1: one counter; 2: counter blockIdx % 8 (128-B apart); 3: one counter, and
// the last arrival increments a second one (two-level form: 8 group counters + 1)
__global__ void tickets(unsigned long long* ctr, int mode, int* out) {
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long v = 0;
    if (mode == 1) {
      v = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (mode == 2 || mode == 3) {
      const int g = blockIdx.x & 7;
      v = __hip_atomic_fetch_add(ctr + 16 * g, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned ng = (gridDim.x - g + 7) / 8;
      if (mode == 3 && (v % ng) == ng - 1)
        v = __hip_atomic_fetch_add(ctr + 16 * 8, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    out[blockIdx.x] = (int)v;
  }
}

int main() {
  unsigned long long* ctr;
  int* out;
  CHECK(hipMalloc(&ctr, 4096));
  CHECK(hipMemset(ctr, 0, 4096));
  CHECK(hipMalloc(&out, 1 << 16));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 200;
  for (int n : {64, 256, 512, 1024, 2048}) {
    float us[4];
    for (int mode = 0; mode < 4; ++mode) {
      for (int w = 0; w < 10; ++w) hipLaunchKernelGGL(tickets, dim3(n), dim3(256), 0, 0, ctr, mode, out);
      CHECK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(tickets, dim3(n), dim3(256), 0, 0, ctr, mode, out);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      us[mode] = ms * 1e3f / reps;
    }
    printf("N %5d  plain %6.2f us  one counter %6.2f us (+%5.2f)  8 counters %6.2f us (+%5.2f)  "
           "8 + 1 %6.2f us (+%5.2f)\n", n, us[0], us[1], us[1] - us[0], us[2], us[2] - us[0], us[3],
           us[3] - us[0]);
  }
  CHECK(hipFree(ctr));
  CHECK(hipFree(out));
  return 0;
}

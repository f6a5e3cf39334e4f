// Calibration: issue rate of the fused passes' per-entry probit arithmetic on gfx950, with the
// operands in registers (no memory), at 1..8 waves per SIMD.  Prints ns per entry-wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../quantized_spectrum_cartography_amd/csrc/qsc_common.cuh"
using namespace qsc;

template <int ILP>
__global__ void __launch_bounds__(256) kern(float* out, int iters, Lik lk) {
  float acc[8] = {0}, own[8];
  for (int r = 0; r < 8; ++r) own[r] = 0.01f * (threadIdx.x + r);
  float nll = 0.f;
  float t0[ILP];
  for (int u = 0; u < ILP; ++u) t0[u] = 0.1f * u + 1e-3f * threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < ILP; ++u) {
      float o[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) o[r] = own[r] + t0[u];
      float t = o[0] * own[0];
#pragma unroll
      for (int r = 1; r < 8; ++r) t = __builtin_fmaf(o[r], own[r], t);
      float l2, g;
      lik_grad<LIK_ONEBIT, false>(t, (it + u) & 1, nullptr, lk, l2, g);
      nll -= l2;
#pragma unroll
      for (int r = 0; r < 8; ++r) acc[r] = __builtin_fmaf(g, o[r], acc[r]);
      t0[u] += 1e-4f;
    }
  }
  float s = nll;
  for (int r = 0; r < 8; ++r) s += acc[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  qsc_model m{};
  m.nbounds = 3; m.log_model = 0; m.sigma = 0.5; m.bounds[0] = 0; m.bounds[1] = 0.5f; m.bounds[2] = 2;
  Lik lk = make_lik(&m);
  int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out; hipMalloc(&out, 256 * 4 * 8 * 1024 * 4);
  const int iters = 256;
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int wps = 1; wps <= 8; wps *= 2) {
    dim3 grid(ncu * wps);  // 256-thread blocks = one wave per SIMD each
    for (int ilp = 1; ilp <= 4; ilp *= 2) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        if (ilp == 1) kern<1><<<grid, 256>>>(out, iters * 4, lk);
        if (ilp == 2) kern<2><<<grid, 256>>>(out, iters * 2, lk);
        if (ilp == 4) kern<4><<<grid, 256>>>(out, iters, lk);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        double entries_per_wave = iters * 4.0;  // entry evaluations per lane
        if (rep) printf("waves/SIMD %d ILP %d: %.3f ms, %.2f ns per entry per SIMD (all waves), %.1f cyc@2.4GHz\n",
                        wps, ilp, ms, ms * 1e6 / (entries_per_wave * wps),
                        ms * 1e6 / (entries_per_wave * wps) * 2.4);
      }
    }
  }
  return 0;
}

// Probe: do fp32 MFMA (v_mfma_f32_32x32x2_f32) and fp32 VALU FMA (v_pk_fma_f32) issued by
// different waves of one SIMD run concurrently? 512-thread workgroups, one per CU (8 waves:
// two per SIMD); waves 0-3 run MFMA chains, waves 4-7 packed-FMA chains, or either alone.
// Concurrent units show as mode 2 taking ~max(mode 0, mode 1), shared ones as ~the sum.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int MODE>   // 0: MFMA waves only, 1: VALU waves only, 2: both
__global__ __launch_bounds__(512) void k_mix(float* out, int n) {
  const int w = threadIdx.x >> 6;
  float s = 0.f;
  if (w < 4 && MODE != 1) {
    f32x16 acc0 = {}, acc1 = {};
    float a = threadIdx.x * 1e-3f, b = 1.0f;
    for (int i = 0; i < n; ++i) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, acc1, 0, 0, 0);
      }
    }
    for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r];
  } else if (w >= 4 && MODE != 0) {
    // per MFMA pair of the other waves (2 x 4096 flops): 32 v_pk_fma_f32 (32 x 256 flops)
    f32x2 acc[16];
    for (int j = 0; j < 16; ++j) acc[j] = f32x2{threadIdx.x * 1e-3f + j, 0.5f * j};
    const f32x2 a = {1.0001f, 0.9999f}, b = {1e-4f, -1e-4f};
    for (int i = 0; i < n; ++i) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = __builtin_elementwise_fma(acc[j], a, b);
      }
    }
    for (int j = 0; j < 16; ++j) s += acc[j].x + acc[j].y;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  const int n = 4000;
  float* out;
  hipMalloc(&out, 4096 * 512 * 4);
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(k_mix<0>, dim3(256), dim3(512), 0, 0, out, n);
      else if (mode == 1) hipLaunchKernelGGL(k_mix<1>, dim3(256), dim3(512), 0, 0, out, n);
      else hipLaunchKernelGGL(k_mix<2>, dim3(256), dim3(512), 0, 0, out, n);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      // flops per launch of each side: 256 WGs x 4 waves x n x 16 MFMA x 4096 (= VALU side)
      const double fl = 256.0 * 4 * n * 16 * 4096.0;
      const double tot = mode == 2 ? 2 * fl : fl;
      if (rep == 2)
        printf("mode %d (%s): %.3f ms  %.1f TF/s\n", mode, mode == 0 ? "MFMA" : mode == 1 ? "VALU" : "both", ms,
               tot / (ms * 1e-3) / 1e12);
    }
  }
  float h[4];
  hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
  printf("sink %g\n", h[0]);
  return 0;
}

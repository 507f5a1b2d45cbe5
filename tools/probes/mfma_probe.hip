// Probe: cycles per v_mfma_f32_32x32x2_f32 on one chain vs two independent chains,
// with 1 or 2 waves per SIMD, and the shader clock under that load
// (s_memtime cycles / s_memrealtime 100 MHz ticks).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CHAINS>
__global__ __launch_bounds__(256) void k_probe(float* out, long long* clk, int n) {
  f32x16 acc0 = {}, acc1 = {};
  float a = threadIdx.x * 1e-3f, b = 1.0f;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc0, 0, 0, 0);
      if (CHAINS == 2) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, acc1, 0, 0, 0);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

int main() {
  const int n = 2000;
  float* out; long long* clk;
  hipMalloc(&out, 4096 * 256 * 4); hipMalloc(&clk, 4096 * 16);
  long long h[8192];
  for (int chains = 1; chains <= 2; ++chains) {
    for (int bpc = 1; bpc <= 2; ++bpc) {     // 256-thread blocks per CU = waves per SIMD
      const int nb = 256 * bpc;
      for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        if (chains == 1) hipLaunchKernelGGL(k_probe<1>, dim3(nb), dim3(256), 0, 0, out, clk, n);
        else hipLaunchKernelGGL(k_probe<2>, dim3(nb), dim3(256), 0, 0, out, clk, n);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, clk, nb * 16, hipMemcpyDeviceToHost);
        double cyc = 0, rt = 0;
        for (int i = 0; i < nb; ++i) { cyc += h[2 * i]; rt += h[2 * i + 1]; }
        cyc /= nb; rt /= nb;
        const double mfma_per_wave = (double)n * 8 * chains;
        const double flops = mfma_per_wave * 32 * 32 * 2 * 2 * 4 * nb;   // 4 waves per block
        if (rep == 1)
          printf("chains=%d waves/SIMD=%d: %.1f cyc per MFMA per wave, clock %.2f GHz, %.1f TFLOP/s (event %.3f ms)\n",
                 chains, bpc, cyc / mfma_per_wave, cyc / (rt * 10.0) , flops / (ms * 1e-3) / 1e12, ms);
      }
    }
  }
  return 0;
}

// Dependent-chain latency of fp64 VALU ops on one wave (the one-workgroup fp64 solves of
// csrc/epc_kernels.hip are chains of these): ITERS x {op} where each op consumes the previous
// result; s_memtime clocks per op. Also LDS load -> use -> store chains.
// Usage: f64_latency_probe ITERS
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void k_chain(int iters, int mode, double a, double b, unsigned long long* out, double* sink) {
  __shared__ double buf[256];
  double x = a + threadIdx.x * 1e-9;
  float xf = (float)x;
  buf[threadIdx.x] = x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (mode == 0) {
    for (int i = 0; i < iters; ++i) x = fma(x, b, a);
  } else if (mode == 1) {
    for (int i = 0; i < iters; ++i) x = __builtin_amdgcn_rcp(x + a);
  } else if (mode == 2) {
    for (int i = 0; i < iters; ++i) xf = fmaf(xf, (float)b, (float)a);
  } else if (mode == 3) {
    for (int i = 0; i < iters; ++i) {
      const int j = ((int)(x * 0.0) + i) & 255;
      x = buf[(threadIdx.x + j) & 255] * b + a;
    }
  } else {
    for (int i = 0; i < iters; ++i) x = 1.0 / (x + a);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) *out = t1 - t0;
  sink[threadIdx.x] = x + xf;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4096;
  unsigned long long* out;
  double* sink;
  if (hipMalloc(&out, 8) != hipSuccess || hipMalloc(&sink, 256 * 8) != hipSuccess) return 1;
  const char* names[] = {"fma_f64 chain", "rcp_f64 chain (+add)", "fma_f32 chain", "LDS load -> fma -> address chain",
                         "IEEE f64 division chain (+add)"};
  for (int mode = 0; mode < 5; ++mode) {
    unsigned long long best = ~0ull;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, iters, mode, 0.5, 0.999, out, sink);
      unsigned long long h = 0;
      if (hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      best = h < best ? h : best;
    }
    printf("%-36s %.1f clocks per step (one wave)\n", names[mode], (double)best / iters);
  }
  return 0;
}

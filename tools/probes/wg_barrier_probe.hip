// Cost of one workgroup barrier by workgroup size on one CU (the one-workgroup fp64 solves of
// csrc/epc_kernels.hip run ~2 barriers per tridiagonalisation step): a single workgroup of NT
// threads runs ITERS x {LDS store, barrier, LDS load} and reports shader clocks per iteration
// from s_memtime; mode 1 drops the barrier (the LDS round trip alone).
// Usage: wg_barrier_probe NT ITERS  -> prints clocks per iteration for mode 0 and 1.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(1024) void k_probe(int iters, int mode, unsigned long long* out, double* sink) {
  __shared__ double buf[1024];
  double acc = threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    buf[threadIdx.x] = acc;
    if (mode == 0) __syncthreads();
    acc += buf[(threadIdx.x + 64) % blockDim.x];
    if (mode == 0) __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) *out = t1 - t0;
  sink[threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: %s NT ITERS\n", argv[0]); return 2; }
  const int nt = atoi(argv[1]), iters = atoi(argv[2]);
  unsigned long long* out;
  double* sink;
  hipMalloc(&out, 8);
  hipMalloc(&sink, 1024 * 8);
  for (int mode = 0; mode < 2; ++mode) {
    unsigned long long best = ~0ull;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(k_probe, dim3(1), dim3(nt), 0, 0, iters, mode, out, sink);
      unsigned long long h = 0;
      hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
      best = h < best ? h : best;
    }
    printf("NT %4d mode %d (%s): %.1f clocks per iteration (2 barriers + LDS round trip)\n", nt, mode,
           mode == 0 ? "barriers" : "no barrier", (double)best / iters);
  }
  return 0;
}

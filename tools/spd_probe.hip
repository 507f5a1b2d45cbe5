// Timing probe of the SPD-inverse kernels (csrc/spd_kernels.hip) at the C3 shape:
// 16 problems of R = 1141 (nbk = 36), per-kernel hipEvent times over repeated launches,
// plus phase-isolating variants of the panel kernel.
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 tools/spd_probe.hip -o tools/spd_probe.bin
#include <cstdio>
#include <cstring>
#include <vector>

#include "../admm-quantization_amd/csrc/spd_kernels.hip"

using namespace admmq;

__global__ __launch_bounds__(256) void k_probe_diag(const ProbDesc* __restrict__ probs, int k) {
  const ProbDesc& p = probs[blockIdx.y];
  const int i = k + blockIdx.x;
  if (k >= p.nbk || i >= p.nbk) return;
  __shared__ double lkk[NB * LS];
  __shared__ int err;
  if (threadIdx.x == 0) err = 0;
  load_block(lkk, p.A64, p.ldm, k, k);
  __syncthreads();
  chol32(lkk, &err);
  if (i == k) store_block(p.D64, NB, k, 0, lkk);
}

__global__ __launch_bounds__(256) void k_probe_trinv(const ProbDesc* __restrict__ probs, int k) {
  const ProbDesc& p = probs[blockIdx.y];
  const int i = k + blockIdx.x;
  if (k >= p.nbk || i >= p.nbk) return;
  __shared__ double lkk[NB * LS], x[NB * LS];
  __shared__ int err;
  if (threadIdx.x == 0) err = 0;
  load_block(lkk, p.A64, p.ldm, k, k);
  __syncthreads();
  chol32(lkk, &err);
  trinv32(lkk, x);
  if (i == k) store_block(p.D64, NB, k, 0, x);
}

__global__ __launch_bounds__(256) void k_probe_load(const ProbDesc* __restrict__ probs, int k) {
  const ProbDesc& p = probs[blockIdx.y];
  const int i = k + blockIdx.x;
  if (k >= p.nbk || i >= p.nbk) return;
  __shared__ double lkk[NB * LS];
  load_block(lkk, p.A64, p.ldm, k, k);
  __syncthreads();
  if (i == k) store_block(p.D64, NB, k, 0, lkk);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const int nprob = 16, R = 1141, nbk = (R + 31) / 32, ldm = nbk * 32;
  std::vector<ProbDesc> h(nprob);
  std::vector<double> a((size_t)ldm * ldm, 0.0);
  for (int r = 0; r < ldm; ++r)
    for (int c = 0; c < ldm; ++c) a[(size_t)r * ldm + c] = r == c ? (double)ldm : 1.0 / (1.0 + r + c);
  for (int p = 0; p < nprob; ++p) {
    ::memset(&h[p], 0, sizeof(ProbDesc));
    CK(hipMalloc(&h[p].A64, a.size() * 8));
    CK(hipMalloc(&h[p].L64, a.size() * 8));
    CK(hipMalloc(&h[p].D64, (size_t)nbk * 32 * 32 * 8));
    CK(hipMalloc(&h[p].M, (size_t)ldm * ldm * 4));
    CK(hipMalloc(&h[p].flags, 16));
    CK(hipMemset(h[p].flags, 0, 16));
    CK(hipMemcpy(h[p].A64, a.data(), a.size() * 8, hipMemcpyHostToDevice));
    h[p].R = R; h[p].ldm = ldm; h[p].nbk = nbk;
  }
  ProbDesc* d;
  CK(hipMalloc(&d, nprob * sizeof(ProbDesc)));
  CK(hipMemcpy(d, h.data(), nprob * sizeof(ProbDesc), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto&& launch, int reps) {
    launch();
    (void)hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %9.2f us/launch\n", name, 1000.0 * ms / reps);
  };
  const int reps = 50;
  timeit("load+store (k=0)", [&] { hipLaunchKernelGGL(k_probe_load, dim3(nbk, nprob), dim3(256), 0, 0, d, 0); }, reps);
  timeit("chol32 (k=0)", [&] { hipLaunchKernelGGL(k_probe_diag, dim3(nbk, nprob), dim3(256), 0, 0, d, 0); }, reps);
  timeit("chol32+trinv32 (k=0)", [&] { hipLaunchKernelGGL(k_probe_trinv, dim3(nbk, nprob), dim3(256), 0, 0, d, 0); }, reps);
  timeit("k_chol_panel (k=0)", [&] { hipLaunchKernelGGL(k_chol_panel, dim3(nbk, nprob), dim3(256), 0, 0, d, 0); }, reps);
  timeit("k_chol_panel (k=30)", [&] { hipLaunchKernelGGL(k_chol_panel, dim3(nbk - 30, nprob), dim3(256), 0, 0, d, 30); }, reps);
  timeit("k_chol_update (k=0)", [&] {
    const int n = nbk - 1;
    hipLaunchKernelGGL(k_chol_update, dim3(n * (n + 1) / 2, nprob), dim3(256), 0, 0, d, 0); }, reps);
  timeit("k_chol_update (k=30)", [&] {
    const int n = nbk - 31;
    hipLaunchKernelGGL(k_chol_update, dim3(n * (n + 1) / 2, nprob), dim3(256), 0, 0, d, 30); }, reps);
  timeit("empty-ish (k=nbk)", [&] { hipLaunchKernelGGL(k_chol_panel, dim3(1, nprob), dim3(256), 0, 0, d, nbk); }, reps);
  for (int p = 0; p < nprob; ++p) CK(hipMemcpy(h[p].A64, a.data(), a.size() * 8, hipMemcpyHostToDevice));
  timeit("launch_spd_inverse (all)", [&] {
    launch_spd_inverse(d, nprob, nbk, 0); }, 5);
  timeit("k_diag_inv", [&] { hipLaunchKernelGGL(k_diag_inv, dim3(nbk, nprob), dim3(256), 0, 0, d); }, reps);
  timeit("k_linv_cols", [&] {
    hipLaunchKernelGGL(k_linv_cols, dim3((nbk - 1) * (NB / kLinvCols), nprob), dim3(1024),
                       (size_t)(nbk + 1) * NB * kLinvCols * sizeof(double), 0, d); }, 10);
  timeit("k_minv", [&] { hipLaunchKernelGGL(k_minv, dim3(nbk * (nbk + 1) / 2, nprob), dim3(256), 0, 0, d); }, 10);
  CK(hipDeviceSynchronize());
  return 0;
}

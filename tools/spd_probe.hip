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

// chol32 with the column broadcast through LDS instead of two readlanes per (c, s): the
// same operations in the same order (same bits); A/B of the panel's serial chain
__device__ void chol32_lds(double* a, int* err, double* colb) {
  if (threadIdx.x < NB) {
    const int r = threadIdx.x;
    double row[NB];
#pragma unroll
    for (int s = 0; s < NB; ++s) row[s] = a[r * LS + s];
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      const double d = readlane_d(row[c], c);
      if (r == 0 && !(d > 0.0)) *err = 1;
      const double sd = sqrt(d);
      const double l = r > c ? row[c] / sd : (r == c ? sd : 0.0);
      row[c] = l;
      colb[r] = l;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int s = c + 1; s < NB; ++s) row[s] -= l * colb[s];
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int s = 0; s < NB; ++s) a[r * LS + s] = s <= r ? row[s] : 0.0;
  }
  __syncthreads();
}
__global__ __launch_bounds__(256) void k_probe_diag_lds(const ProbDesc* __restrict__ probs, int k) {
  const ProbDesc& p = probs[blockIdx.y];
  const int i = k + blockIdx.x;
  if (k >= p.nbk || i >= p.nbk) return;
  __shared__ double lkk[NB * LS], colb[NB];
  __shared__ int err;
  if (threadIdx.x == 0) err = 0;
  load_block(lkk, p.A64, p.ldm, k, k);
  __syncthreads();
  chol32_lds(lkk, &err, colb);
  if (i == k) store_block(p.D64 + 32 * 32 * 64, NB, k, 0, lkk);
}
// trinv32 with each row's l entries read into registers before its FMA chains (the same
// operations in the same order: same bits)
__device__ __forceinline__ void trinv32_pre(const double* l, double* x) {   // (now the product form)
  if (threadIdx.x < NB) {
    const int c = threadIdx.x;
    double rinv[NB], col[NB];
#pragma unroll
    for (int r = 0; r < NB; ++r) rinv[r] = 1.0 / l[r * LS + r];
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      double lr[NB];
#pragma unroll
      for (int t = 0; t < r; ++t) lr[t] = l[r * LS + t];
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int t = 0; t + 1 < r; t += 2) {
        s0 += lr[t] * col[t];
        s1 += lr[t + 1] * col[t + 1];
      }
      if (r & 1) s0 += lr[r - 1] * col[r - 1];
      col[r] = r < c ? 0.0 : (r == c ? rinv[r] : -(s0 + s1) * rinv[r]);
    }
#pragma unroll
    for (int r = 0; r < NB; ++r) x[r * LS + c] = col[r];
  }
  __syncthreads();
}
__global__ __launch_bounds__(256) void k_probe_trinv_pre(const ProbDesc* __restrict__ probs, int k) {
  const ProbDesc& p = probs[blockIdx.y];
  const int i = k + blockIdx.x;
  if (k >= p.nbk || i >= p.nbk) return;
  __shared__ double lkk[NB * LS], x[NB * LS];
  __shared__ int err;
  if (threadIdx.x == 0) err = 0;
  load_block(lkk, p.A64, p.ldm, k, k);
  __syncthreads();
  chol32(lkk, &err);
  trinv32_pre(lkk, x);
  if (i == k) store_block(p.D64 + 32 * 32 * 32, NB, k, 0, x);
}
__global__ void k_cmp(const double* a, const double* b, int n, int* bad) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (__double_as_longlong(a[i]) != __double_as_longlong(b[i])) atomicAdd(bad, 1);
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
    CK(hipMalloc(&h[p].D64, (size_t)(nbk + 64) * 32 * 32 * 8));
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
  timeit("chol32 LDS broadcast (k=0)", [&] { hipLaunchKernelGGL(k_probe_diag_lds, dim3(nbk, nprob), dim3(256), 0, 0, d, 0); }, reps);
  {
    int* bad;
    CK(hipMalloc(&bad, 4));
    CK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_cmp, dim3(4), dim3(256), 0, 0, h[0].D64, h[0].D64 + 32 * 32 * 64, 32 * 32, bad);
    int hb = -1;
    CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    printf("chol32 vs LDS-broadcast form: %d differing doubles of the k=0 diagonal block\n", hb);
  }
  timeit("chol32+trinv32 (k=0)", [&] { hipLaunchKernelGGL(k_probe_trinv, dim3(nbk, nprob), dim3(256), 0, 0, d, 0); }, reps);
  timeit("chol32+trinv32_pre (k=0)", [&] { hipLaunchKernelGGL(k_probe_trinv_pre, dim3(nbk, nprob), dim3(256), 0, 0, d, 0); }, reps);
  {
    int* bad;
    CK(hipMalloc(&bad, 4));
    CK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_cmp, dim3(4), dim3(256), 0, 0, h[0].D64, h[0].D64 + 32 * 32 * 32, 32 * 32, bad);
    int hb = -1;
    CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    printf("trinv32 vs preloaded-row form: %d differing doubles of the k=0 inverse block\n", hb);
  }
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

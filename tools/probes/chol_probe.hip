// Latency probe of the 32 x 32 diagonal-block factorisation of the blocked fp64 Cholesky
// (csrc/spd_kernels.hip chol32 + trinv32: the serial chain of every panel step; one
// k_chol_panel launch per block column, ~25 us each at R = 1141). Variants with the same
// arithmetic in the same order (same bits) or a different summation order (stated):
//   chol32            the product form: l_s broadcast by two v_readlane per (c, s) (the
//                     compiler keeps ~60 of them live in SGPRs and spills them to VGPR lanes)
//   chol32_shfl       the same operations, l_s broadcast by ds_bpermute (VGPRs, no SGPRs)
//   trinv32           column c by thread c, two interleaved FMA chains per row
//   trinv32_w8        column c by 8 threads, each a strided part of every row's sum, summed
//                     by DPP (another summation order: other bits)
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 tools/probes/chol_probe.hip -o tools/probes/chol_probe
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../admm-quantization_amd/csrc/spd_kernels.hip"  // (its chol32 is now the w64 form below)

using namespace admmq;

// (shfl_d comes with spd_kernels.hip; since round 6 its chol32 is the 64-lane form chol32_w64
// below, so "chol32" here measures that; the round-6 numbers of the one-row-per-lane form
// are in profiles/r06_chol_probe.txt)
__device__ void chol32_shfl(double* a, int* err) {
  if (threadIdx.x < 64) {   // the whole wave takes part in the shuffles; lanes >= 32 idle otherwise
    const int r = threadIdx.x & 31;
    double row[NB];
#pragma unroll
    for (int s = 0; s < NB; ++s) row[s] = a[r * LS + s];
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      const double d = readlane_d(row[c], c);
      if (threadIdx.x == 0 && !(d > 0.0)) *err = 1;
      const double sd = sqrt(d);
      const double l = r > c ? row[c] / sd : (r == c ? sd : 0.0);
      row[c] = l;
#pragma unroll
      for (int s = c + 1; s < NB; ++s) row[s] -= l * shfl_d(l, s);
    }
    if (threadIdx.x < 32)
#pragma unroll
      for (int s = 0; s < NB; ++s) a[r * LS + s] = s <= r ? row[s] : 0.0;
  }
  __syncthreads();
}

// chol32 on all 64 lanes: lane (r, h) = r + 32 h holds row r's columns 2 j + h; each step's
// rank-1 update is ~half as many instructions per lane (the same operations per element:
// same bits). l_s comes from lane s (which holds l for row s in both halves).
__device__ void chol32_w64(double* a, int* err) {
  if (threadIdx.x < 64) {
    const int r = threadIdx.x & 31, h = threadIdx.x >> 5;
    double rw[NB / 2];
#pragma unroll
    for (int j = 0; j < NB / 2; ++j) rw[j] = a[r * LS + 2 * j + h];
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      // row r's entry c lives in lane r + 32 (c & 1), slot c >> 1
      const double rc = shfl_d(rw[c >> 1], r + 32 * (c & 1));
      const double d = readlane_d(rw[c >> 1], c + 32 * (c & 1));
      if (threadIdx.x == 0 && !(d > 0.0)) *err = 1;
      const double sd = sqrt(d);
      const double l = r > c ? rc / sd : (r == c ? sd : 0.0);
      if ((c & 1) == h) rw[c >> 1] = l;
#pragma unroll
      for (int j = 0; j < NB / 2; ++j) {
        if (2 * j + 1 <= c) continue;   // (uniform: both columns of slot j at or before c)
        const int sc = 2 * j + h;       // this lane's column of slot j
        const double ls = shfl_d(l, sc);
        if (sc > c) rw[j] -= l * ls;
      }
    }
#pragma unroll
    for (int j = 0; j < NB / 2; ++j) {
      const int sc = 2 * j + h;
      a[r * LS + sc] = sc <= r ? rw[j] : 0.0;
    }
  }
  __syncthreads();
}

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double sum8_d(double v) {
  v += dpp_d<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);   // row_half_mirror
  return v;
}
// column c = tid >> 3 by the 8 threads j = tid & 7: thread j sums the row's terms t = j (mod 8)
// (it holds col[t] for those t: cq[t / 8]); every thread of the group gets the sum
__device__ __forceinline__ void trinv32_w8(const double* l, double* x) {
  const int c = threadIdx.x >> 3, j = threadIdx.x & 7;
  double cq[NB / 8];
#pragma unroll
  for (int q = 0; q < NB / 8; ++q) cq[q] = 0.0;
#pragma unroll
  for (int r = 0; r < NB; ++r) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NB / 8; ++q) {
      const int t = 8 * q + j;
      if (8 * q < r) s = fma(t < r ? l[r * LS + t] : 0.0, cq[q], s);
    }
    s = sum8_d(s);
    const double v = r < c ? 0.0 : (r == c ? 1.0 / l[r * LS + r] : -s / l[r * LS + r]);
    if ((r & 7) == j) cq[r >> 3] = v;
  }
#pragma unroll
  for (int q = 0; q < NB / 8; ++q) x[(8 * q + j) * LS + c] = cq[q];
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_p_chol(const ProbDesc* __restrict__ probs, int k, int variant) {
  const ProbDesc& p = probs[blockIdx.y];
  const int i = k + blockIdx.x;
  if (k >= p.nbk || i >= p.nbk) return;
  __shared__ double lkk[NB * LS], x[NB * LS];
  __shared__ int err;
  if (threadIdx.x == 0) err = 0;
  load_block(lkk, p.A64, p.ldm, k, k);
  __syncthreads();
  if (variant & 8) chol32_w64(lkk, &err);
  else if (variant & 1) chol32_shfl(lkk, &err);
  else chol32(lkk, &err);
  if (variant & 4) {
    if (variant & 2) trinv32_w8(lkk, x);
    else trinv32(lkk, x);
  }
  if (i == k) store_block(p.D64 + (size_t)32 * 32 * 64 * (variant + 1), NB, k, 0, (variant & 4) ? x : lkk);
}

__global__ void k_cmp(const double* a, const double* b, int n, int* bad, double* maxrel) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (__double_as_longlong(a[i]) != __double_as_longlong(b[i])) atomicAdd(bad, 1);
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const int nprob = 1, R = 1141, nbk = (R + 31) / 32, ldm = nbk * 32;
  std::vector<ProbDesc> h(nprob);
  std::vector<double> a((size_t)ldm * ldm, 0.0);
  for (int r = 0; r < ldm; ++r)
    for (int c = 0; c < ldm; ++c) a[(size_t)r * ldm + c] = r == c ? (double)ldm : 1.0 / (1.0 + r + c);
  for (int p = 0; p < nprob; ++p) {
    ::memset(&h[p], 0, sizeof(ProbDesc));
    CK(hipMalloc(&h[p].A64, a.size() * 8));
    CK(hipMalloc(&h[p].L64, a.size() * 8));
    CK(hipMalloc(&h[p].D64, (size_t)(nbk + 64 * 17) * 32 * 32 * 8));
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
    printf("%-40s %9.2f us/launch\n", name, 1000.0 * ms / reps);
  };
  const int reps = 200;
  const char* names[16] = {"chol32", "chol32_shfl", "", "", "chol32 + trinv32", "chol32_shfl + trinv32", "chol32 + trinv32_w8",
                           "chol32_shfl + trinv32_w8", "chol32_w64", "", "", "", "chol32_w64 + trinv32", "", "", ""};
  for (int v : {0, 1, 8, 4, 5, 12, 6, 7})
    timeit(names[v], [&] { hipLaunchKernelGGL(k_p_chol, dim3(nbk, nprob), dim3(256), 0, 0, d, 0, v); }, reps);
  timeit("k_chol_panel (k=0)", [&] { hipLaunchKernelGGL(k_chol_panel, dim3(nbk, nprob), dim3(256), 0, 0, d, 0); }, reps);
  int* bad;
  CK(hipMalloc(&bad, 4));
  auto cmp = [&](int va, int vb) {
    CK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_cmp, dim3(4), dim3(256), 0, 0, h[0].D64 + (size_t)32 * 32 * 64 * (va + 1),
                       h[0].D64 + (size_t)32 * 32 * 64 * (vb + 1), 32 * 32, bad, nullptr);
    int hb = -1;
    CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    printf("%s vs %s: %d differing doubles\n", names[va], names[vb], hb);
    return 0;
  };
  cmp(0, 1);
  cmp(0, 8);
  cmp(4, 5);
  cmp(4, 12);
  cmp(4, 6);
  CK(hipDeviceSynchronize());
  return 0;
}

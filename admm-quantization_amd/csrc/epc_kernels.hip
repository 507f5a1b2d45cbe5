// The EPC step's Lagrange multiplier on the device (cp_anc, source/parafac_epc.py:61-74;
// admmq.parafac_epc): the scalar root search that ran on the host after every mode step's
// R x R eigendecomposition, with two host synchronisations per step.
#include <cmath>
#include <cstdint>

#include "../../include/admmq.h"
#include "admmq_internal.h"

namespace admmq {

// The root mu >= 0 of normY2 - sum_i c_i (s_i + 2 mu) / (s_i + mu)^2 = delta2 by doubling
// the bracket from max(s) and 200 bisection steps to fp64 resolution; the sum over i in a
// fixed order (thread-strided partials, then the 4 waves' sums in order). One workgroup:
// the host no longer waits for c and s every mode step.
__device__ double epc_err(const double* c, const double* sv, int n, double mu, double normY2, double* red) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double acc = 0.0;
  for (int i = tid; i < n; i += 256) {
    const double d = sv[i] + mu;
    acc += c[i] * (sv[i] + 2.0 * mu) / (d * d);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  __syncthreads();   // red reused across calls
  if (lane == 0) red[w] = acc;
  __syncthreads();
  return normY2 - (((red[0] + red[1]) + red[2]) + red[3]);
}

__global__ __launch_bounds__(256) void k_epc_mu(const double* __restrict__ c, const double* __restrict__ sv, int n,
                                                double normY2, double delta2, double* __restrict__ mu_out) {
  __shared__ double red[4];
  __shared__ double smax[4];
  double mx = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) mx = fmax(mx, sv[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) smax[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmax(fmax(smax[0], smax[1]), fmax(smax[2], smax[3]));
  double result = 0.0;
  if (!(epc_err(c, sv, n, 0.0, normY2, red) >= delta2)) {
    double hi = fmax(mx, 1e-300);
    while (epc_err(c, sv, n, hi, normY2, red) < delta2 && hi < 1e300) hi *= 2.0;
    double lo = 0.0;
    for (int it = 0; it < 200; ++it) {
      const double mid = 0.5 * (lo + hi);
      if (mid <= lo || mid >= hi) break;
      if (epc_err(c, sv, n, mid, normY2, red) < delta2) lo = mid;
      else hi = mid;
    }
    result = lo;
  }
  if (threadIdx.x == 0) *mu_out = result;
}

// ---------------------------------------------------------------------------
// The R x R normal-equation solves of the CP-ALS / EPC initialiser on one workgroup
// (n <= kSpdSmallMax: the fp64 matrix in LDS), replacing tensorly parafac's solve and
// cp_anc's eigendecomposition (source/parafac_epc.py:42, :61-74; admmq.parafac_epc):
//
//   k_spd_solve64   X = F G^-1 (the CP-ALS update U_m = F G^-1, G = Hadamard of the Grams);
//   k_epc_step64    X = F (G + mu I)^-1 with mu >= 0 the root of the EPC error equation
//                   e(mu) = ||Y||^2 - <F, X> - mu ||X||^2 = delta^2 (the eigen form's
//                   ||Y||^2 - sum_j c_j (s_j + 2 mu) / (s_j + mu)^2 with G = V diag(s) V^T,
//                   c_j = |F v_j|^2), found by Newton steps on e, e'(mu) = 2 mu ||X L^-T||^2,
//                   safeguarded by the bracket [lo, hi] (bisection / doubling), each from a
//                   fresh Cholesky of G + mu I; mu = 0 when e(0) >= delta^2 already (the LS
//                   step keeps the error).
//
// Cholesky (right-looking, one column per step, one workgroup barrier per step): the lower
// triangle holds the matrix being factored; L's column j is written, scaled, into row j of
// the upper triangle (never read by a trailing update) and its diagonal into dg[j]. The
// right-hand sides are the rows of F: a 16-lane group of one wave owns a row, lane c the
// entries i = c (mod 16) in registers; forward and backward substitution run down the
// columns with the pivot value broadcast inside the group by a shuffle, so they need no
// workgroup barrier.
constexpr int kSpdSmallMax = 140;   // 140^2 doubles = 156.8 KB of LDS
constexpr int kSpdThreads = 1024;
constexpr int kSpdGroup = 16;                            // lanes per right-hand-side row
constexpr int kSpdRowsPerPass = kSpdThreads / kSpdGroup;  // 64 rows at a time
constexpr int kSpdPer = (kSpdSmallMax + kSpdGroup - 1) / kSpdGroup;   // entries per lane (9)

// A <- G + shift I (lower triangle and diagonal), then its Cholesky factor; false (uniform
// over the workgroup) if a pivot is not positive and finite
__device__ bool spd_chol_lds(const double* __restrict__ G, int n, double shift, double* A, double* dg) {
  const int tid = threadIdx.x;
  for (int e = tid; e < n * n; e += kSpdThreads) {
    const int i = e / n, k = e - i * n;
    if (k <= i) A[e] = G[e] + (i == k ? shift : 0.0);
  }
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    const double d = A[j * n + j];
    if (!(d > 0.0) || !(d < __builtin_huge_val())) return false;   // every thread reads the same d
    const double r = 1.0 / d, isq = 1.0 / sqrt(d);
    if (tid == 0) dg[j] = sqrt(d);
    for (int i = j + 1 + tid; i < n; i += kSpdThreads) A[j * n + i] = A[i * n + j] * isq;   // L[i][j]
    for (int i = j + 1 + (tid >> 3); i < n; i += kSpdThreads / 8) {
      const double li = A[i * n + j] * r;
      for (int k = j + 1 + (tid & 7); k <= i; k += 8) A[i * n + k] -= li * A[k * n + j];
    }
    __syncthreads();
  }
  return true;
}

// One right-hand-side row per 16-lane group: x (this lane's entries i = c + 16 q) <- x A^-1
// with A = L L^T: forward L z = x, then backward L^T y = z. FWD_ONLY: z only (x L^-T).
template <bool FWD_ONLY>
__device__ __forceinline__ void spd_row_solve(const double* A, const double* dg, int n, double (&x)[kSpdPer]) {
  const int lane = threadIdx.x & 63, c = lane & (kSpdGroup - 1), base = lane & ~(kSpdGroup - 1);
  for (int j = 0; j < n; ++j) {   // z_j = x_j / L_jj, then x_i -= L[i][j] z_j for i > j
    const int qj = j / kSpdGroup;
    double zj = 0.0;
#pragma unroll
    for (int q = 0; q < kSpdPer; ++q)
      if (q == qj) zj = x[q] / dg[j];
    zj = __shfl(zj, base + (j & (kSpdGroup - 1)), 64);
#pragma unroll
    for (int q = 0; q < kSpdPer; ++q) {
      const int i = c + kSpdGroup * q;
      if (i == j) x[q] = zj;
      else if (i > j && i < n) x[q] -= A[j * n + i] * zj;
    }
  }
  if (FWD_ONLY) return;
  for (int j = n - 1; j >= 0; --j) {   // y_j = z_j / L_jj, then z_i -= L[j][i] y_j for i < j
    const int qj = j / kSpdGroup;
    double yj = 0.0;
#pragma unroll
    for (int q = 0; q < kSpdPer; ++q)
      if (q == qj) yj = x[q] / dg[j];
    yj = __shfl(yj, base + (j & (kSpdGroup - 1)), 64);
#pragma unroll
    for (int q = 0; q < kSpdPer; ++q) {
      const int i = c + kSpdGroup * q;
      if (i == j) x[q] = yj;
      else if (i < j) x[q] -= A[i * n + j] * yj;
    }
  }
}

__device__ __forceinline__ void spd_load_row(const double* __restrict__ F, int row, int m, int n, double (&x)[kSpdPer]) {
  const int c = threadIdx.x & (kSpdGroup - 1);
#pragma unroll
  for (int q = 0; q < kSpdPer; ++q) {
    const int i = c + kSpdGroup * q;
    x[q] = (row < m && i < n) ? F[(size_t)row * n + i] : 0.0;
  }
}

// Block sum (every thread's v; the result in every thread), 16 waves
__device__ __forceinline__ double spd_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < kSpdThreads / 64; ++w) t += red[w];
  return t;
}

__global__ __launch_bounds__(kSpdThreads) void k_spd_solve64(const double* __restrict__ G, const double* __restrict__ F,
                                                             int m, int n, double* __restrict__ X,
                                                             int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double A[];
  __shared__ double dg[kSpdSmallMax];
  const bool ok = spd_chol_lds(G, n, 0.0, A, dg);
  if (!ok) {
    if (threadIdx.x == 0 && info) *info = 1;
    return;
  }
  for (int r0 = 0; r0 < m; r0 += kSpdRowsPerPass) {
    const int row = r0 + (int)(threadIdx.x / kSpdGroup);
    double x[kSpdPer];
    spd_load_row(F, row, m, n, x);
    spd_row_solve<false>(A, dg, n, x);
    const int c = threadIdx.x & (kSpdGroup - 1);
    if (row < m)
#pragma unroll
      for (int q = 0; q < kSpdPer; ++q) {
        const int i = c + kSpdGroup * q;
        if (i < n) X[(size_t)row * n + i] = x[q];
      }
  }
  if (threadIdx.x == 0 && info) *info = 0;
}

// e(mu), e'(mu) and X = F (G + mu I)^-1 (into X when `store`); false if G + mu I is not SPD
__device__ bool epc_eval(const double* __restrict__ G, const double* __restrict__ F, int m, int n, double mu,
                         double normY2, double* A, double* dg, double* red, double* X, bool store, double& e,
                         double& de) {
  if (!spd_chol_lds(G, n, mu, A, dg)) return false;
  double fx = 0.0, xx = 0.0, ww = 0.0;
  const int c = threadIdx.x & (kSpdGroup - 1);
  for (int r0 = 0; r0 < m; r0 += kSpdRowsPerPass) {
    const int row = r0 + (int)(threadIdx.x / kSpdGroup);
    double f[kSpdPer], x[kSpdPer];
    spd_load_row(F, row, m, n, f);
#pragma unroll
    for (int q = 0; q < kSpdPer; ++q) x[q] = f[q];
    spd_row_solve<false>(A, dg, n, x);
#pragma unroll
    for (int q = 0; q < kSpdPer; ++q) { fx += f[q] * x[q]; xx += x[q] * x[q]; }
    if (store && row < m)
#pragma unroll
      for (int q = 0; q < kSpdPer; ++q) {
        const int i = c + kSpdGroup * q;
        if (i < n) X[(size_t)row * n + i] = x[q];
      }
    if (mu > 0.0) {   // ||X L^-T||^2: forward solves of the rows of X
      spd_row_solve<true>(A, dg, n, x);
#pragma unroll
      for (int q = 0; q < kSpdPer; ++q) ww += x[q] * x[q];
    }
  }
  fx = spd_block_sum(fx, red);
  xx = spd_block_sum(xx, red);
  ww = spd_block_sum(ww, red);
  e = normY2 - fx - mu * xx;
  de = 2.0 * mu * ww;
  return true;
}

// mu_io: in, a warm start (the previous step's mu of this mode, <= 0: none); out, mu.
// info (may be NULL): 0 ok, 1 no SPD G + mu I on the bracket.
__global__ __launch_bounds__(kSpdThreads) void k_epc_step64(const double* __restrict__ G, const double* __restrict__ F,
                                                            int m, int n, double normY2, double delta2,
                                                            double* __restrict__ mu_io, double* __restrict__ X,
                                                            int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double A[];
  __shared__ double dg[kSpdSmallMax];
  __shared__ double red[kSpdThreads / 64];
  double tr = 0.0;   // trace(G) / n: the scale of the bracket's first step
  for (int i = threadIdx.x; i < n; i += kSpdThreads) tr += G[(size_t)i * n + i];
  tr = spd_block_sum(tr, red) / (double)n;
  const double warm = *mu_io;
  double e = 0.0, de = 0.0;
  double mu = 0.0, lo = 0.0, hi = __builtin_huge_val();
  double xmu = -1.0;   // the mu whose X = F (G + mu I)^-1 is in X
  bool have = false;   // (e, de) are those of mu
  // mu = 0 (the least-squares step) unless a warm start already shows the root above it
  bool need0 = true;
  if (warm > 0.0) {
    if (epc_eval(G, F, m, n, warm, normY2, A, dg, red, X, true, e, de)) {
      mu = xmu = warm; have = true;
      if (e < delta2) { lo = warm; need0 = false; }
      else hi = warm;
    }
  }
  if (need0) {
    double e0, de0;
    const bool ok0 = epc_eval(G, F, m, n, 0.0, normY2, A, dg, red, X, true, e0, de0);
    if (ok0) xmu = 0.0;
    if (ok0 && e0 >= delta2) {   // the LS step already keeps the error: mu = 0
      if (threadIdx.x == 0) { *mu_io = 0.0; if (info) *info = 0; }
      return;
    }
    if (!have) {   // no bracket yet: double from a small multiple of trace(G) / n
      mu = tr > 0.0 ? tr * 0x1p-20 : 1e-300;
      for (int it = 0; it < 2100; ++it) {
        if (!epc_eval(G, F, m, n, mu, normY2, A, dg, red, X, true, e, de)) { mu *= 2.0; continue; }
        have = true; xmu = mu;
        if (e < delta2) { lo = mu; mu *= 2.0; if (!(mu < 1e300)) break; }
        else { hi = mu; break; }
      }
    }
  }
  // safeguarded Newton on e(mu) = delta2 inside [lo, hi]: a Newton step (bisection, or
  // doubling while hi is unknown, when it leaves the bracket) until the step is below fp64
  // resolution, the bracket has collapsed, or e is within rounding of delta2. (e is flat near
  // mu = 0, e'(0) = 0, so a small |e - delta2| alone does not fix mu: the step size decides.)
  for (int it = 0; it < 100 && have; ++it) {
    if (hi < __builtin_huge_val() && !(hi - lo > 4.0 * 0x1p-52 * hi)) break;   // collapsed bracket
    double nx = de > 0.0 ? mu - (e - delta2) / de : -1.0;
    if (!(nx > lo && nx < hi)) nx = (hi < __builtin_huge_val()) ? 0.5 * (lo + hi) : 2.0 * fmax(mu, lo);
    if (fabs(nx - mu) <= 2.0 * 0x1p-52 * mu) break;   // converged to fp64 resolution
    double en, dn;
    if (!epc_eval(G, F, m, n, nx, normY2, A, dg, red, X, true, en, dn)) { lo = nx; continue; }
    mu = xmu = nx; e = en; de = dn;
    if (e < delta2) lo = mu; else hi = mu;
    if (fabs(e - delta2) <= 0x1p-52 * normY2) break;   // at the rounding floor of e
  }
  if (have && xmu != mu) {   // X must be that of the returned mu
    double en, dn;
    (void)epc_eval(G, F, m, n, mu, normY2, A, dg, red, X, true, en, dn);
  }
  if (threadIdx.x == 0) { *mu_io = mu; if (info) *info = have ? 0 : 1; }
}

}  // namespace admmq

using namespace admmq;

extern "C" {

int32_t admmq_epc_mu(const double* c, const double* s, int64_t n, double normY2, double delta2, double* mu,
                     void* stream) {
  if (!c || !s || !mu || n <= 0 || n > (1LL << 30)) return set_error(ADMMQ_ERR_ARG, "epc_mu: bad arguments");
  hipLaunchKernelGGL(k_epc_mu, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), c, s, (int)n, normY2, delta2, mu);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "epc_mu: launch failed");
}

int32_t admmq_spd_solve64(const double* G, const double* F, int64_t m, int64_t n, double* X, int32_t* info,
                          void* stream) {
  if (!G || !F || !X || m < 0 || n <= 0 || n > kSpdSmallMax || m > (1LL << 24))
    return set_error(ADMMQ_ERR_ARG, "spd_solve64: bad arguments (1 <= n <= 140)");
  if (m == 0) return ADMMQ_OK;
  const size_t lds = (size_t)n * n * sizeof(double);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_spd_solve64), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(k_spd_solve64, dim3(1), dim3(kSpdThreads), lds, static_cast<hipStream_t>(stream), G, F, (int)m,
                     (int)n, X, info);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "spd_solve64: launch failed");
}

int32_t admmq_epc_step64(const double* G, const double* F, int64_t m, int64_t n, double normY2, double delta2,
                         double* mu, double* X, int32_t* info, void* stream) {
  if (!G || !F || !X || !mu || m <= 0 || n <= 0 || n > kSpdSmallMax || m > (1LL << 24))
    return set_error(ADMMQ_ERR_ARG, "epc_step64: bad arguments (1 <= n <= 140)");
  const size_t lds = (size_t)n * n * sizeof(double);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_epc_step64), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(k_epc_step64, dim3(1), dim3(kSpdThreads), lds, static_cast<hipStream_t>(stream), G, F, (int)m,
                     (int)n, normY2, delta2, mu, X, info);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "epc_step64: launch failed");
}

}  // extern "C"

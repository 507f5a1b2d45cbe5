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

}  // namespace admmq

using namespace admmq;

extern "C" {

int32_t admmq_epc_mu(const double* c, const double* s, int64_t n, double normY2, double delta2, double* mu,
                     void* stream) {
  if (!c || !s || !mu || n <= 0 || n > (1LL << 30)) return set_error(ADMMQ_ERR_ARG, "epc_mu: bad arguments");
  hipLaunchKernelGGL(k_epc_mu, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), c, s, (int)n, normY2, delta2, mu);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "epc_mu: launch failed");
}

}  // extern "C"

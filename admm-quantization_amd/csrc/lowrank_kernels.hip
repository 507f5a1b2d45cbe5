// Quant + low-rank ADMM (scripts/factorize_lowrank.py:85-101, admm_iteration):
//
//   for j in 1 .. max_iter-1:
//     H_ = (rho (H + U) + W - H2) / (1 + rho)          k_lr_pre   (also X = H_ - U)
//     H  = proj(H_ - U)                                 caller: quantizer or rank projection
//     U += H - H_ ;  r = |H - H_|^2/|H|^2 ;  s = |H - H_prev|^2/|U|^2 ;  break if r, s < eps
//                                                       k_lr_post  (H_prev is the old H)
//
// Both kernels are elementwise streams (HBM-bound: pre 24 B/element, post 20 B/element
// + the projection's own pass; float4 when aligned); every float32 operation is in the reference's order.
// The break test runs on the device: post's blocks write fp64 partial sums, the last
// block to arrive sums them in block order (deterministic), tests r < eps and s < eps
// and sets the sticky `done` word; later pre/post launches see it and do nothing, so
// the caller queues all max_iter-1 iterations without a host round trip per iteration.
#include <algorithm>
#include <cstdint>
#include <initializer_list>
#include <string>

#include "../../include/admmq.h"
#include "admmq_internal.h"

namespace admmq {

constexpr int kLrBlocks = 1024;   // fixed grid: partial sums have a fixed order
constexpr int kLrThreads = 256;

struct LrState {
  int done, ticket, iters, pad_;
};

// V4: every pointer 16-byte aligned and n % 4 == 0 (the host checks): float4 streams
template <bool V4>
__global__ __launch_bounds__(kLrThreads) void k_lr_pre(const float* __restrict__ H, const float* __restrict__ U,
                                                       const float* __restrict__ W, const float* __restrict__ H2,
                                                       float* __restrict__ Hbar, float* __restrict__ X, long long n,
                                                       float rho, float den, const LrState* __restrict__ st) {
  if (st->done) return;
  auto one = [&](float h, float u, float w, float h2, float& hb, float& x) {
    const float hu = h + u;
    const float t = ((rho * hu + w) - h2) / den;   // (rho*(H + U) + W - H2) / (1 + rho)
    hb = t;
    x = t - u;
  };
  if constexpr (V4) {
    const long long n4 = n >> 2;
    for (long long q = (long long)blockIdx.x * kLrThreads + threadIdx.x; q < n4; q += (long long)gridDim.x * kLrThreads) {
      const float4 h = reinterpret_cast<const float4*>(H)[q], u = reinterpret_cast<const float4*>(U)[q];
      const float4 w = reinterpret_cast<const float4*>(W)[q], h2 = reinterpret_cast<const float4*>(H2)[q];
      float4 hb, x;
      one(h.x, u.x, w.x, h2.x, hb.x, x.x);
      one(h.y, u.y, w.y, h2.y, hb.y, x.y);
      one(h.z, u.z, w.z, h2.z, hb.z, x.z);
      one(h.w, u.w, w.w, h2.w, hb.w, x.w);
      reinterpret_cast<float4*>(Hbar)[q] = hb;
      reinterpret_cast<float4*>(X)[q] = x;
    }
  } else {
    for (long long e = (long long)blockIdx.x * kLrThreads + threadIdx.x; e < n; e += (long long)gridDim.x * kLrThreads)
      one(H[e], U[e], W[e], H2[e], Hbar[e], X[e]);
  }
}

__device__ __forceinline__ double lr_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <bool V4>
__global__ __launch_bounds__(kLrThreads) void k_lr_post(const float* __restrict__ Hn, const float* __restrict__ Hbar,
                                                        float* __restrict__ H, float* __restrict__ U, long long n,
                                                        float eps, LrState* __restrict__ st, double* __restrict__ part) {
  if (st->done) return;
  double s1 = 0.0, s2 = 0.0, s3 = 0.0, s4 = 0.0;
  auto one = [&](float hn, float hb, float hp, float& u) {
    const float d = hn - hb;
    u = u + d;                                   // U += H - H_
    const float dp = hn - hp;
    s1 += (double)d * d;                         // sum (H - H_)^2
    s2 += (double)hn * hn;                       // sum H^2
    s3 += (double)dp * dp;                       // sum (H - H_prev)^2
    s4 += (double)u * u;                         // sum U^2
  };
  // contiguous chunk per block: the block partials do not depend on the grid schedule
  if constexpr (V4) {
    const long long n4 = n >> 2;
    const long long per = (n4 + gridDim.x - 1) / gridDim.x;
    const long long b0 = (long long)blockIdx.x * per, b1 = min(n4, b0 + per);
    for (long long q = b0 + threadIdx.x; q < b1; q += kLrThreads) {
      const float4 hn = reinterpret_cast<const float4*>(Hn)[q], hb = reinterpret_cast<const float4*>(Hbar)[q];
      const float4 hp = reinterpret_cast<const float4*>(H)[q];
      float4 u = reinterpret_cast<const float4*>(U)[q];
      one(hn.x, hb.x, hp.x, u.x);
      one(hn.y, hb.y, hp.y, u.y);
      one(hn.z, hb.z, hp.z, u.z);
      one(hn.w, hb.w, hp.w, u.w);
      reinterpret_cast<float4*>(U)[q] = u;
      reinterpret_cast<float4*>(H)[q] = hn;
    }
  } else {
    const long long per = (n + gridDim.x - 1) / gridDim.x;
    const long long b0 = (long long)blockIdx.x * per, b1 = min(n, b0 + per);
    for (long long e = b0 + threadIdx.x; e < b1; e += kLrThreads) {
      const float hn = Hn[e], hb = Hbar[e], hp = H[e];
      float u = U[e];
      one(hn, hb, hp, u);
      U[e] = u;
      H[e] = hn;
    }
  }
  __shared__ double red[4][kLrThreads / 64];
  __shared__ int last;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  s1 = lr_wave_sum(s1); s2 = lr_wave_sum(s2); s3 = lr_wave_sum(s3); s4 = lr_wave_sum(s4);
  if (lane == 0) { red[0][w] = s1; red[1][w] = s2; red[2][w] = s3; red[3][w] = s4; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t[4] = {0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < kLrThreads / 64; ++q)
      for (int k = 0; k < 4; ++k) t[k] += red[k][q];
    double* mine = part + 4 * (size_t)blockIdx.x;
    for (int k = 0; k < 4; ++k) __hip_atomic_store(mine + k, t[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
    const int old = __hip_atomic_fetch_add(&st->ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old + 1 == (int)gridDim.x;
  }
  __syncthreads();
  if (!last) return;
  // the last block sums the partials in a fixed order: thread t the blocks t, t + 256, ...
  // ascending, then the wave sums and the four waves in order (one thread walking all
  // 4 x 1024 partials took ~200 us of dependent loads)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  double t[4] = {0.0, 0.0, 0.0, 0.0};
  for (unsigned b = threadIdx.x; b < gridDim.x; b += kLrThreads)
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] += __hip_atomic_load(part + 4 * (size_t)b + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int k = 0; k < 4; ++k) t[k] = lr_wave_sum(t[k]);
  __syncthreads();   // (red is reused)
  if (lane == 0) { red[0][w] = t[0]; red[1][w] = t[1]; red[2][w] = t[2]; red[3][w] = t[3]; }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double u[4] = {0.0, 0.0, 0.0, 0.0};
  for (int q = 0; q < kLrThreads / 64; ++q)
    for (int k = 0; k < 4; ++k) u[k] += red[k][q];
  st->ticket = 0;
  st->iters += 1;
  if (u[0] / u[1] < (double)eps && u[2] / u[3] < (double)eps) st->done = 1;
}

static size_t lr_bytes() { return 256 + (size_t)kLrBlocks * 4 * sizeof(double); }

static bool aligned16(std::initializer_list<const float*> ps) {
  for (const float* p : ps)
    if (reinterpret_cast<uintptr_t>(p) & 15) return false;
  return true;
}

// units = elements (scalar) or float4s (V4)
static int lr_grid(long long n) { return (int)std::max(1LL, std::min<long long>(kLrBlocks, (n + kLrThreads - 1) / kLrThreads)); }

}  // namespace admmq

using namespace admmq;

extern "C" {

size_t admmq_lowrank_workspace_size(int64_t n) { return n < 0 ? 0 : lr_bytes(); }

int32_t admmq_lowrank_reset(void* workspace, size_t workspace_bytes, void* stream) {
  if (!workspace || workspace_bytes < lr_bytes()) return set_error(ADMMQ_ERR_WORKSPACE, "lowrank: workspace too small");
  if (hipMemsetAsync(workspace, 0, sizeof(LrState), static_cast<hipStream_t>(stream)) != hipSuccess)
    return set_error(ADMMQ_ERR_HIP, "lowrank: reset failed");
  return ADMMQ_OK;
}

int32_t admmq_lowrank_pre(const float* H, const float* U, const float* W, const float* H2, float* Hbar, float* X,
                          int64_t n, float rho, void* workspace, size_t workspace_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!H || !U || !W || !H2 || !Hbar || !X))) return set_error(ADMMQ_ERR_ARG, "lowrank_pre: bad arguments");
  if (!workspace || workspace_bytes < lr_bytes()) return set_error(ADMMQ_ERR_WORKSPACE, "lowrank: workspace too small");
  if (n == 0) return ADMMQ_OK;
  const LrState* st = static_cast<const LrState*>(workspace);
  const bool v4 = n % 4 == 0 && aligned16({H, U, W, H2, Hbar, X});
  const int grid = lr_grid(v4 ? n / 4 : n);
  if (v4)
    hipLaunchKernelGGL(k_lr_pre<true>, dim3(grid), dim3(kLrThreads), 0, static_cast<hipStream_t>(stream), H, U, W, H2,
                       Hbar, X, (long long)n, rho, 1.0f + rho, st);
  else
    hipLaunchKernelGGL(k_lr_pre<false>, dim3(grid), dim3(kLrThreads), 0, static_cast<hipStream_t>(stream), H, U, W, H2,
                       Hbar, X, (long long)n, rho, 1.0f + rho, st);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "lowrank_pre: launch failed");
}

int32_t admmq_lowrank_post(const float* Hn, const float* Hbar, float* H, float* U, int64_t n, float eps,
                           void* workspace, size_t workspace_bytes, void* stream) {
  if (n <= 0 || !Hn || !Hbar || !H || !U) return set_error(ADMMQ_ERR_ARG, "lowrank_post: bad arguments");
  if (!workspace || workspace_bytes < lr_bytes()) return set_error(ADMMQ_ERR_WORKSPACE, "lowrank: workspace too small");
  LrState* st = static_cast<LrState*>(workspace);
  double* part = reinterpret_cast<double*>(static_cast<char*>(workspace) + 256);
  const bool v4 = n % 4 == 0 && aligned16({Hn, Hbar, H, U});
  const int grid = lr_grid(v4 ? n / 4 : n);
  if (v4)
    hipLaunchKernelGGL(k_lr_post<true>, dim3(grid), dim3(kLrThreads), 0, static_cast<hipStream_t>(stream), Hn, Hbar, H,
                       U, (long long)n, eps, st, part);
  else
    hipLaunchKernelGGL(k_lr_post<false>, dim3(grid), dim3(kLrThreads), 0, static_cast<hipStream_t>(stream), Hn, Hbar, H,
                       U, (long long)n, eps, st, part);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "lowrank_post: launch failed");
}

}  // extern "C"

// Two-stage exact MSE-minmax search (source/quantization.py:118-144).
//
// The reference tries 200 clipping candidates t_c with a full pass each. Its answer
// is the first-index argmin of the canonical SSE (oracle/quant_oracle.py). Here:
//
// stage 1  k_mse_hist   each element x visits only its <= 2^(bits-1) level
//                       breakpoints: for k = 1..|q(0)|, b_k = #{c : |q(c)| >= k}
//                       (q(c) = clamp(rint(fl(x/s_c))) is monotone in c, found with a
//                       linear estimate + exact IEEE checks), and adds |x| (fixed point)
//                       and 2k-1 into per-candidate suffix histograms h1/h2; plus sum x^2.
//          k_mse_select one block per job: T1(c) = sum_{b>c} h1[b], T2(c) = sum_{b>c} h2[b]
//                       give the exact-arithmetic SSE A(c) = S2 - 2 s T1 + s^2 T2 and a
//                       rigorous bound E(c) on |canonical - A| (oracle/stage1_model.py);
//                       S = {c : A - E <= min(A + E)} provably holds the argmin.
// stage 2  k_mse_sse    canonical SSE only for c in S (|S| = 1 almost always: then the
//                       kernel exits at once); exhaustive when |S| > kMaxSel or forced.
#include <cstdlib>

#include "quant_device.h"

namespace admmq {

__device__ __forceinline__ const MseView& mview(const ProbDesc* d, const QJob* q, int job) {
  return d ? d[job].mv : q[job].mv;
}

// rint(fl(a / s_c)) for a >= 0 via the reciprocal fast path + exact fallback.
__device__ __forceinline__ int level_of(float a, int c, const float* __restrict__ s_tab,
                                        const float* __restrict__ r_tab, float delta) {
  const float y = a * r_tab[c];
  float q = __builtin_rintf(y);
  if (__builtin_fabsf(__builtin_fabsf(y - q) - 0.5f) < delta) q = __builtin_rintf(a / s_tab[c]);
  return (int)q;
}

// VAR (timing ablation only, results wrong unless 0): 1 = no LDS histogram atomics,
// 2 = no global flush, 3 = neither.
template <int VAR>
__global__ __launch_bounds__(256) void k_mse_hist(const ProbDesc* __restrict__ d, const QJob* __restrict__ qj,
                                                  const Chunk* __restrict__ chunks, int ncand, int bits, int slot) {
  const Chunk ck = chunks[blockIdx.x];
  const MseView& v = mview(d, qj, ck.job);
  if (v.done && *v.done) return;
  const float mx = __uint_as_float(v.stat[4 * slot]);
  if (mse_degenerate(mx)) return;
  __shared__ float s_tab[kMaxStage1], r_tab[kMaxStage1];
  __shared__ unsigned long long h1[kMaxStage1 + 1];
  __shared__ unsigned h2[kMaxStage1 + 1];
  __shared__ double red[4];
  const int n = ncand;
  const int qmax = 1 << (bits - 1);
  const float den = (float)(2 * qmax - 1);
  for (int c = threadIdx.x; c < n; c += blockDim.x) {
    const float s = (2.0f * cand_t(mx, c, n)) / den;
    s_tab[c] = s;
    r_tab[c] = 1.0f / s;
  }
  for (int b = threadIdx.x; b <= n; b += blockDim.x) { h1[b] = 0ull; h2[b] = 0u; }
  __syncthreads();
  const float S0 = (float)(0.2 * (double)mx);
  const float E0 = (float)(1.2 * (double)mx);
  const float inv_step = (n > 1) ? (float)(n - 1) / (E0 - S0) : 0.f;
  const float delta = (float)(qmax + 1) * 0x1p-21f;
  int emx;
  (void)__builtin_frexpf(mx, &emx);
  const long long nterm = (long long)v.nelem * qmax;
  const int clt = 64 - __builtin_clzll((unsigned long long)(nterm > 1 ? nterm - 1 : 1));
  const int K1 = 61 - emx - clt;
  const long long total = (long long)v.rows * v.ld;
  const long long end = min((long long)ck.start + kHistElems, total);
  double s2 = 0.0;
  // b = n ("level >= k for every candidate") is by far the most common breakpoint for
  // small k: accumulate it in registers instead of 64-way-colliding LDS atomics.
  unsigned long long full1 = 0ull;
  unsigned full2 = 0u;
  for (long long e = (long long)ck.start + 4LL * threadIdx.x; e < end; e += 4LL * blockDim.x) {
    const float4 x4 = *reinterpret_cast<const float4*>(v.X + e);
    const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = xs[j];
      if (x == 0.f) continue;
      s2 += (double)x * (double)x;
      const float a = __builtin_fabsf(x);
      const int cap = (x > 0.f) ? qmax - 1 : qmax;
      const int k0 = min(level_of(a, 0, s_tab, r_tab, delta), cap);
      if (k0 <= 0) continue;
      const unsigned long long af = to_fixed(a, K1);
      // levels reached even at the largest candidate count for every c
      const int kfull = min(level_of(a, n - 1, s_tab, r_tab, delta), k0);
      if (kfull > 0) {
        full1 += af * (unsigned long long)kfull;
        full2 += (unsigned)(kfull * kfull);        // sum_{k<=kfull} (2k-1)
      }
      int bprev = n;
      for (int k = kfull + 1; k <= k0; ++k) {
        // |q(c)| >= k  <=>  t_c <~ a*den/(2k-1);  t_c ~ S0 + c*step
        const float tau = a * den * __builtin_amdgcn_rcpf((float)(2 * k - 1));   // estimate only
        const float ce = (tau - S0) * inv_step;
        int b = (ce >= (float)n) ? n - 1 : (ce < 0.f ? 1 : (int)ce + 1);
        b = min(max(b, 1), min(bprev, n - 1));
        while (b < n - 1 && level_of(a, b, s_tab, r_tab, delta) >= k) ++b;
        while (b > 1 && level_of(a, b - 1, s_tab, r_tab, delta) < k) --b;
        bprev = b;
        if constexpr (VAR & 1) {
          full1 += af ^ (unsigned long long)b;
        } else {
          atomicAdd(&h1[b], af);
          atomicAdd(&h2[b], (unsigned)(2 * k - 1));
        }
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s2 += __shfl_xor(s2, off);
    full1 += __shfl_xor(full1, off);
    full2 += (unsigned)__shfl_xor((int)full2, off);
  }
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = s2;
    atomicAdd(&h1[n], full1);
    atomicAdd(&h2[n], full2);
  }
  __syncthreads();
  unsigned long long* g1 = v.h1 + (size_t)slot * (n + 1);
  unsigned long long* g2 = v.h2 + (size_t)slot * (n + 1);
  if constexpr ((VAR & 2) == 0) {
    for (int b = threadIdx.x; b <= n; b += blockDim.x) {
      if (h1[b]) atomicAdd(&g1[b], h1[b]);
      if (h2[b]) atomicAdd(&g2[b], (unsigned long long)h2[b]);
    }
  } else {
    if (threadIdx.x == 0 && h1[n] == 12345) g1[0] = h2[0];
  }
  if (threadIdx.x == 0) atomicAdd(&v.s2[slot], red[0] + red[1] + red[2] + red[3]);
}

// One wave per job. Lane l owns the consecutive candidate block [l*P, l*P+P) with
// P = ceil(n/64): suffix sums come from a per-lane pass plus a wave-level exclusive
// suffix scan, the set S is built in ascending order from a prefix count over lanes.
__global__ __launch_bounds__(64) void k_mse_select(const ProbDesc* __restrict__ d, const QJob* __restrict__ qj,
                                                   int ncand, int bits, int slot, int force_all) {
  const MseView& v = mview(d, qj, blockIdx.x);
  if (v.done && *v.done) return;
  int* sel = v.sel + (size_t)slot * (2 + kMaxSel);
  const int lane = threadIdx.x;
  const float mx = __uint_as_float(v.stat[4 * slot]);
  if (mse_degenerate(mx)) {
    if (lane == 0) { sel[0] = 1; sel[1] = 0; }   // finalize emits NaN for degenerate mx
    return;
  }
  const int n = ncand;
  if (force_all || n > kMaxStage1) {
    if (lane == 0) { sel[0] = n; sel[1] = -1; }
    return;
  }
  constexpr int PMAX = (kMaxStage1 + 63) / 64;
  const int P = (n + 63) / 64;
  const unsigned long long* g1 = v.h1 + (size_t)slot * (n + 1);
  const unsigned long long* g2 = v.h2 + (size_t)slot * (n + 1);
  // T(c) = sum_{b > c} h[b]: lane-local suffix over its block, then across lanes
  unsigned long long t1[PMAX], t2[PMAX];
  unsigned long long r1 = 0ull, r2 = 0ull;
#pragma unroll
  for (int j = PMAX - 1; j >= 0; --j) {
    t1[j] = r1; t2[j] = r2;                       // exclusive within the lane: b > c
    const int b = lane * P + j;
    if (j < P && b <= n) { r1 += g1[b]; r2 += g2[b]; }
  }
  // candidates above this lane's block contribute sum of later lanes' blocks, plus b = n
  // when it is not inside any block (n == 64 P exactly).
  unsigned long long s1 = r1, s2v = r2;          // inclusive suffix scan over lanes
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long o1 = __shfl_down(s1, off);
    const unsigned long long o2 = __shfl_down(s2v, off);
    if (lane + off < 64) { s1 += o1; s2v += o2; }
  }
  unsigned long long above1 = __shfl_down(s1, 1), above2 = __shfl_down(s2v, 1);
  if (lane == 63) { above1 = 0ull; above2 = 0ull; }
  if (64 * P == n) { above1 += g1[n]; above2 += g2[n]; }   // b = n lies past every block
  const int qmax = 1 << (bits - 1);
  const float denf = (float)(2 * qmax - 1);
  int emx;
  (void)__builtin_frexpf(mx, &emx);
  const long long nterm = (long long)v.nelem * qmax;
  const int clt = 64 - __builtin_clzll((unsigned long long)(nterm > 1 ? nterm - 1 : 1));
  const int K1 = 61 - emx - clt;
  const int K = fixed_exp(mx, v.nq);
  const double S2 = v.s2[slot];
  const double u = 0x1p-24;
  const double fixu = ldexp(1.0, -K1);
  double lo[PMAX], hi[PMAX];
  double mymin = 1e300;
#pragma unroll
  for (int j = 0; j < PMAX; ++j) {
    const int c = lane * P + j;
    lo[j] = 1e300; hi[j] = 1e300;
    if (j < P && c < n) {
      const double s = (double)((2.0f * cand_t(mx, c, n)) / denf);
      const double T1 = (double)(t1[j] + above1) * fixu;
      const double T2 = (double)(t2[j] + above2);
      const double A = S2 - 2.0 * s * T1 + s * s * T2;
      const double mag = S2 + 2.0 * s * T1 + s * s * T2;
      const double slack = 1e-10 * mag;
      const double sh = fmax(A, 0.0) + slack;
      const double B1 = 2.0 * u * (1.0 + u) * (s * sqrt(T2 * sh) + sh) + 2.0 * u * u * (1.0 + u) * (1.0 + u) * (s * s * T2 + sh);
      const double E = B1 + 3.0000002 * u * (sh + B1) + (double)v.nq * ldexp(1.0, -K) +
                       2.0 * s * (double)nterm * fixu + slack + 8.0 * (double)v.nelem * 0x1p-149;
      lo[j] = A - E;
      hi[j] = A + E;
      mymin = fmin(mymin, hi[j]);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mymin = fmin(mymin, __shfl_xor(mymin, off));
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < PMAX; ++j) cnt += (lo[j] <= mymin) ? 1 : 0;
  int pre = cnt;                                   // inclusive prefix over lanes
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(pre, off);
    if (lane >= off) pre += o;
  }
  const int total = __shfl(pre, 63);
  int pos = pre - cnt;
#pragma unroll
  for (int j = 0; j < PMAX; ++j) {
    if (lo[j] <= mymin) {
      if (pos < kMaxSel) sel[2 + pos] = lane * P + j;
      ++pos;
    }
  }
  if (lane == 0) {   // sel = {|S| (n: exhaustive), unused, S ascending...}; |S| == 1 -> c* = sel[2]
    if (total > kMaxSel || total == 0) { sel[0] = n; sel[1] = -1; }
    else { sel[0] = total; sel[1] = 0; }
  }
}

__global__ __launch_bounds__(256) void k_mse_sse(const ProbDesc* __restrict__ d, const QJob* __restrict__ qj,
                                                 const Chunk* __restrict__ chunks, int ncand, int bits, int slot) {
  const Chunk ck = chunks[blockIdx.x];
  const MseView& v = mview(d, qj, ck.job);
  if (v.done && *v.done) return;
  const int* sel = v.sel + (size_t)slot * (2 + kMaxSel);
  const int ns = sel[0];
  if (ns == 1) return;
  const float mx = __uint_as_float(v.stat[4 * slot]);
  if (mse_degenerate(mx)) return;
  __shared__ float4 xs[kSseQuads];
  __shared__ int list[kMaxSel];
  const int nqc = min(kSseQuads, v.nq - ck.start);
  for (int t = threadIdx.x; t < nqc; t += blockDim.x) {
    const int qi = ck.start + t;
    const int row = qi / v.qpr;
    const int qc = qi - row * v.qpr;
    xs[t] = *reinterpret_cast<const float4*>(v.X + (size_t)row * v.ld + 4 * qc);
  }
  const bool all = ns >= ncand;
  if (!all)
    for (int j = threadIdx.x; j < ns; j += blockDim.x) list[j] = sel[2 + j];
  __syncthreads();
  sse_sweep_list(xs, nqc, mx, fixed_exp(mx, v.nq), ncand, bits, all ? nullptr : list, all ? ncand : ns,
                 v.sse + (size_t)slot * ncand);
}

void launch_mse_hist(const ProbDesc* d, const QJob* q, const Chunk* chunks, int nchunks, int ncand, int bits,
                     int slot, hipStream_t s) {
  static const int var = [] {
    const char* e = getenv("ADMMQ_HIST_VARIANT");
    return e ? atoi(e) : 0;
  }();
  if (nchunks <= 0) return;
  if (var == 1) hipLaunchKernelGGL(k_mse_hist<1>, dim3(nchunks), dim3(256), 0, s, d, q, chunks, ncand, bits, slot);
  else if (var == 2) hipLaunchKernelGGL(k_mse_hist<2>, dim3(nchunks), dim3(256), 0, s, d, q, chunks, ncand, bits, slot);
  else if (var == 3) hipLaunchKernelGGL(k_mse_hist<3>, dim3(nchunks), dim3(256), 0, s, d, q, chunks, ncand, bits, slot);
  else hipLaunchKernelGGL(k_mse_hist<0>, dim3(nchunks), dim3(256), 0, s, d, q, chunks, ncand, bits, slot);
}
void launch_mse_select(const ProbDesc* d, const QJob* q, int njobs, int ncand, int bits, int slot, int force_all,
                       hipStream_t s) {
  if (njobs > 0) hipLaunchKernelGGL(k_mse_select, dim3(njobs), dim3(64), 0, s, d, q, ncand, bits, slot, force_all);
}
void launch_mse_sse(const ProbDesc* d, const QJob* q, const Chunk* chunks, int nchunks, int ncand, int bits,
                    int slot, hipStream_t s) {
  if (nchunks > 0) hipLaunchKernelGGL(k_mse_sse, dim3(nchunks), dim3(256), 0, s, d, q, chunks, ncand, bits, slot);
}

}  // namespace admmq

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

// Smallest float32 a >= 0 with rint(fl(a / s)) >= k (IEEE division, half-even ties):
// fl(a/s) is monotone in a, so step from the estimate (k - 1/2) s by ulps.
__device__ __forceinline__ bool reaches(float a, float s, int k) {
  const float y = a / s;
  const float h = (float)k - 0.5f;
  return (y > h) || (y == h && (k & 1) == 0);
}
__device__ float level_threshold(float s, int k) {
  float a = ((float)k - 0.5f) * s;
  if (reaches(a, s, k)) {
    for (int it = 0; it < 64; ++it) {
      const float p = __uint_as_float(__float_as_uint(a) - 1u);
      if (a == 0.f || !reaches(p, s, k)) break;
      a = p;
    }
  } else {
    for (int it = 0; it < 64 && !reaches(a, s, k); ++it) a = __uint_as_float(__float_as_uint(a) + 1u);
  }
  return a;
}

// Per job and iteration: thr[k][c] for k = 1..qmax, c < n into global memory (one
// block per job; every stage-1 block then just copies the table into LDS).
__global__ __launch_bounds__(256) void k_mse_prep(const ProbDesc* __restrict__ d, const QJob* __restrict__ qj,
                                                  int ncand, int bits, int slot) {
  const MseView& v = mview(d, qj, blockIdx.x);
  if (v.done && *v.done) return;
  const float mx = __uint_as_float(v.stat[4 * slot]);
  if (mse_degenerate(mx)) return;
  const int n = ncand;
  const int qmax = 1 << (bits - 1);
  const float den = (float)(2 * qmax - 1);
  for (int e = threadIdx.x; e < qmax * n; e += blockDim.x) {
    const int k = 1 + e / n, c = e - (k - 1) * n;
    const float s = (2.0f * cand_t(mx, c, n)) / den;
    v.thr[k * n + c] = level_threshold(s, k);
  }
}

// Stage 1. thr[k][c] turns every breakpoint probe into one compare:
// |q_c(x)| >= k  <=>  |x| >= thr[k][c]  (thr increasing in c and in k).
// 1024 threads x 4 elements per block; the block's histograms are flushed into one of
// kHistRep replicas of the job's global histograms (replica = block % kHistRep).
__global__ __launch_bounds__(1024) void k_mse_hist(const ProbDesc* __restrict__ d, const QJob* __restrict__ qj,
                                                   const Chunk* __restrict__ chunks, int ncand, int bits, int slot) {
  const Chunk ck = chunks[blockIdx.x];
  const MseView& v = mview(d, qj, ck.job);
  if (v.done && *v.done) return;
  const float mx = __uint_as_float(v.stat[4 * slot]);
  if (mse_degenerate(mx)) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = ncand;
  const int qmax = 1 << (bits - 1);
  unsigned long long* h1 = reinterpret_cast<unsigned long long*>(smem);          // n+1
  unsigned* h2 = reinterpret_cast<unsigned*>(h1 + (n + 1));                       // n+1
  float* thr = reinterpret_cast<float*>(h2 + ((n + 1 + 3) & ~3));                 // [qmax+1][n]
  __shared__ double red[16];
  const float den = (float)(2 * qmax - 1);
  for (int e = n + threadIdx.x; e < (qmax + 1) * n; e += blockDim.x) thr[e] = v.thr[e];
  for (int b = threadIdx.x; b <= n; b += blockDim.x) { h1[b] = 0ull; h2[b] = 0u; }
  __syncthreads();
  const float S0 = (float)(0.2 * (double)mx);
  const float E0 = (float)(1.2 * (double)mx);
  const float inv_step = (n > 1) ? (float)(n - 1) / (E0 - S0) : 0.f;
  int emx;
  (void)__builtin_frexpf(mx, &emx);
  const long long nterm = (long long)v.nelem * qmax;
  const int clt = 64 - __builtin_clzll((unsigned long long)(nterm > 1 ? nterm - 1 : 1));
  const int K1 = 61 - emx - clt;
  const long long total = (long long)v.rows * v.ld;
  double s2 = 0.0;
  // b = n ("level >= k for every candidate") is the most common breakpoint for small
  // k: accumulate it in registers instead of colliding LDS atomics.
  unsigned long long full1 = 0ull;
  unsigned full2 = 0u;
  const long long e = (long long)ck.start + 4LL * threadIdx.x;
  if (e < total) {
    const float4 x4 = *reinterpret_cast<const float4*>(v.X + e);
    const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = xs[j];
      if (x == 0.f) continue;
      s2 += (double)x * (double)x;
      const float a = __builtin_fabsf(x);
      const int cap = (x > 0.f) ? qmax - 1 : qmax;
      int k0 = 0, kfull = 0;
      for (int k = 1; k <= cap; ++k) {
        k0 += (a >= thr[k * n]) ? 1 : 0;
        kfull += (a >= thr[k * n + n - 1]) ? 1 : 0;
      }
      if (k0 <= 0) continue;
      const unsigned long long af = to_fixed(a, K1);
      if (kfull > 0) {
        full1 += af * (unsigned long long)kfull;
        full2 += (unsigned)(kfull * kfull);        // sum_{k<=kfull} (2k-1)
      }
      int bprev = n - 1;
      for (int k = kfull + 1; k <= k0; ++k) {
        // b_k = #{c : a >= thr[k][c]} in [1, n-1]; estimate from t_c ~ S0 + c*step
        const float* tk = thr + k * n;
        const float tau = a * den * __builtin_amdgcn_rcpf((float)(2 * k - 1));   // estimate only
        const float ce = (tau - S0) * inv_step;
        int b = (ce >= (float)n) ? n - 1 : (ce < 0.f ? 1 : (int)ce + 1);
        b = min(max(b, 1), bprev);
        while (b < n - 1 && a >= tk[b]) ++b;
        while (b > 1 && a < tk[b - 1]) --b;
        bprev = b;
        atomicAdd(&h1[b], af);
        atomicAdd(&h2[b], (unsigned)(2 * k - 1));
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
  const int rep = blockIdx.x & (kHistRep - 1);
  unsigned long long* g1 = v.h1 + ((size_t)slot * kHistRep + rep) * (n + 1);
  unsigned long long* g2 = v.h2 + ((size_t)slot * kHistRep + rep) * (n + 1);
  for (int b = threadIdx.x; b <= n; b += blockDim.x) {
    if (h1[b]) atomicAdd(&g1[b], h1[b]);
    if (h2[b]) atomicAdd(&g2[b], (unsigned long long)h2[b]);
  }
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    atomicAdd(&v.s2[slot], t);
  }
}

size_t hist_lds_bytes(int ncand, int bits) {
  const int qmax = 1 << (bits - 1);
  return (size_t)(ncand + 1) * 8 + (size_t)((ncand + 1 + 3) & ~3) * 4 + (size_t)(qmax + 1) * ncand * 4;
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
  const unsigned long long* g1 = v.h1 + (size_t)slot * kHistRep * (n + 1);
  const unsigned long long* g2 = v.h2 + (size_t)slot * kHistRep * (n + 1);
  auto hsum = [&](const unsigned long long* g, int b) {
    unsigned long long t = 0ull;
#pragma unroll
    for (int r = 0; r < kHistRep; ++r) t += g[r * (n + 1) + b];
    return t;
  };
  // T(c) = sum_{b > c} h[b]: lane-local suffix over its block, then across lanes
  unsigned long long t1[PMAX], t2[PMAX];
  unsigned long long r1 = 0ull, r2 = 0ull;
#pragma unroll
  for (int j = PMAX - 1; j >= 0; --j) {
    t1[j] = r1; t2[j] = r2;                       // exclusive within the lane: b > c
    const int b = lane * P + j;
    if (j < P && b <= n) { r1 += hsum(g1, b); r2 += hsum(g2, b); }
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
  if (64 * P == n) { above1 += hsum(g1, n); above2 += hsum(g2, n); }   // b = n lies past every block
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
  if (nchunks <= 0) return;
  hipLaunchKernelGGL(k_mse_hist, dim3(nchunks), dim3(1024), hist_lds_bytes(ncand, bits), s, d, q, chunks, ncand, bits,
                     slot);
}
void launch_mse_prep(const ProbDesc* d, const QJob* q, int njobs, int ncand, int bits, int slot, hipStream_t s) {
  if (njobs > 0) hipLaunchKernelGGL(k_mse_prep, dim3(njobs), dim3(256), 0, s, d, q, ncand, bits, slot);
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

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
#include <algorithm>
#include <mutex>
#include <cstdlib>

#include <hip/hip_ext.h>

#include "quant_device.h"
#include "search_device.h"

namespace admmq {

typedef __attribute__((address_space(1))) unsigned long long gu64;   // global (not flat) sc1 loads

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

// Per-block phase timeline of the last stage-1 launch (diagnostics, admmq_debug_hist_trace):
// s_memrealtime at {start, thresholds ready, elements done, flushed, end}, and the CU id.
constexpr int kHistTraceMax = 8192;
__device__ unsigned long long g_hist_trace[kHistTraceMax][6];
// ... and inside its fused finalize (admm_finalize_block stamps)
__device__ unsigned long long g_fin_trace[kHistTraceMax][5];
// ... and the CU each k_mse_hist3 block ran on: (XCC_ID << 32) | HW_ID (the fused kernel's
// column 5 holds a time stamp, so the CU cannot live there)
__device__ unsigned long long g_hist_cu[kHistTraceMax];
int copy_hist_cu(unsigned long long* host, int n) {
  n = n < kHistTraceMax ? n : kHistTraceMax;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_hist_cu), (size_t)n * sizeof(unsigned long long)) == hipSuccess ? n
                                                                                                                  : -1;
}
int copy_fin_trace(unsigned long long* host, int n) {
  n = n < kHistTraceMax ? n : kHistTraceMax;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fin_trace), (size_t)n * 5 * sizeof(unsigned long long)) == hipSuccess
             ? n : -1;
}

int copy_hist_trace(unsigned long long* host, int n) {
  n = n < kHistTraceMax ? n : kHistTraceMax;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_hist_trace), (size_t)n * 6 * sizeof(unsigned long long)) == hipSuccess
             ? n : -1;
}

// Diagnostics: how often the selection leaves more than one candidate ({|S| == 1,
// 2..kMaxSel, exhaustive} counts since the last reset), for admmq_debug_sel_stats.
__device__ unsigned long long g_sel_stats[3];
__device__ int g_no_stop = 0;   // stop flag of units without one (standalone quantization)
// Diagnostics (admmq_debug_set_sel_widen): every candidate stays in S, so the selection's
// multi-candidate paths (the canonical SSEs; in the fused finalize the record published
// before the ready word) run every time; the exact answer, hence every bit, is the same.
__device__ int g_sel_widen = 0;
int set_sel_widen_search(int on) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_sel_widen), &on, sizeof(int)) == hipSuccess ? 0 : -1;
}
int copy_sel_stats(unsigned long long* host, int reset) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sel_stats), sizeof(g_sel_stats)) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z[3] = {0ull, 0ull, 0ull};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_sel_stats), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 3;
}


// Diagnostics: level_threshold_fast == level_threshold over random (s, k).
__global__ void k_check_thresholds(unsigned seed, int nsamp, unsigned* mismatches) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nsamp; i += gridDim.x * blockDim.x) {
    unsigned x = seed ^ (0x9E3779B9u * (unsigned)(i + 1));
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    const int k = 1 + (int)(x % 40u);
    unsigned y = x * 2654435761u + 12345u;
    y ^= y >> 13; y *= 0x5bd1e995u; y ^= y >> 15;
    const float s = __uint_as_float((y & 0x007FFFFFu) | ((100u + (y >> 24) % 60u) << 23));   // s in [2^-27, 2^33)
    if (level_threshold_fast(s, k) != level_threshold(s, k)) atomicAdd(mismatches, 1u);
  }
}
// Diagnostics: the host's cell lower bound (merged_tables, h3_setup) holds for random mx
// in the range it is used for: every threshold e's actual cell is at most
// floor(z_e (1 + 1e-4)), the cell the host counts it below. Also reports the largest
// deviation of a cell position from its key proportion (in cells x 1e6).
__global__ void k_check_cells(int n, int qmax, unsigned seed, int nsamp, unsigned* bad, unsigned* maxdev) {
  const int M = qmax * n;
  const double kmax = (double)(2 * qmax - 1) * (double)(6LL * (n - 1));
  const float den = (float)(2 * qmax - 1);
  for (long long w = blockIdx.x * (long long)blockDim.x + threadIdx.x; w < (long long)nsamp * M;
       w += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(w / M), e = (int)(w - (long long)i * M);
    unsigned x = seed ^ (0x9E3779B9u * (unsigned)(i + 1));
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    const float mx = __uint_as_float((x & 0x007FFFFFu) | ((27u + (x >> 23) % 201u) << 23));   // [2^-100, 2^101)
    if (!(mx >= 0x1p-100f && mx <= 0x1p100f)) continue;
    const int k = 1 + e / n, c = e - (k - 1) * n;
    const float v = level_threshold_fast((2.0f * cand_t(mx, c, n)) / den, k);
    const float inv = (float)kCells / level_threshold_fast((2.0f * cand_t(mx, n - 1, n)) / den, qmax);
    const int ca = min(kCells - 1, (int)(v * inv));
    const double z = (double)kCells * ((double)(2 * k - 1) * (double)((n - 1) + 5LL * c)) / kmax;
    if ((double)ca > floor(z * (1.0 + 1e-4))) atomicAdd(bad, 1u);
    const double dev = fabs((double)v * (double)inv - z);
    atomicMax(maxdev, (unsigned)fmin(dev * 1e6, 4e9));
  }
}
int check_cells(int n, int bits, unsigned seed, int nsamp, unsigned* maxdev_out) {
  unsigned* d = nullptr;
  if (hipMalloc(&d, 2 * sizeof(unsigned)) != hipSuccess) return -1;
  (void)hipMemset(d, 0, 2 * sizeof(unsigned));
  hipLaunchKernelGGL(k_check_cells, dim3(512), dim3(256), 0, 0, n, 1 << (bits - 1), seed, nsamp, d, d + 1);
  unsigned h[2] = {0u, 0u};
  const bool ok = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipFree(d);
  if (maxdev_out) *maxdev_out = h[1];
  return ok ? (int)h[0] : -1;
}

int check_thresholds(unsigned seed, int nsamp) {
  unsigned* d = nullptr;
  if (hipMalloc(&d, sizeof(unsigned)) != hipSuccess) return -1;
  (void)hipMemset(d, 0, sizeof(unsigned));
  hipLaunchKernelGGL(k_check_thresholds, dim3(256), dim3(256), 0, 0, seed, nsamp, d);
  unsigned h = 0;
  const bool ok = hipMemcpy(&h, d, sizeof(unsigned), hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipFree(d);
  return ok ? (int)h : -1;
}



// Candidate selection for one job from the summed stage-1 histograms H1/H2 (LDS,
// n+1 bins) and S2, by one wave. Lane l owns candidates [l P, l P + P), P = ceil(n/64);
// T(c) = sum_{b>c} H[b] = (later lanes' blocks, wave suffix scan) + (rest of the lane's
// block, walked downwards). A(c) = S2 - 2 s T1 + s^2 T2 with E(c) its rigorous error
// bound (oracle/stage1_model.py); pass 1 finds min(A + E), pass 2 writes
// S = {c : A - E <= min(A + E)} in ascending order (prefix count over lanes).
__device__ void select_wave(const MseView& v, int* sel, int* lsel, const unsigned long long* H1,
                            const unsigned long long* H2, double S2, float mx, int n, int qmax) {
  const int lane = threadIdx.x & 63;
  const int P = (n + 63) / 64;
  const int c0 = lane * P, c1 = min(c0 + P, n);   // this lane's candidates [c0, c1)
  unsigned long long r1 = 0ull, r2 = 0ull;
  for (int b = c0; b < c1; ++b) { r1 += H1[b]; r2 += H2[b]; }
  unsigned long long s1 = r1, s2v = r2;          // inclusive suffix scan over lanes
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long o1 = __shfl_down(s1, off);
    const unsigned long long o2 = __shfl_down(s2v, off);
    if (lane + off < 64) { s1 += o1; s2v += o2; }
  }
  unsigned long long above1 = __shfl_down(s1, 1), above2 = __shfl_down(s2v, 1);
  if (lane == 63) { above1 = 0ull; above2 = 0ull; }
  above1 += H1[n]; above2 += H2[n];               // b = n lies past every candidate
  SelCtx cx;
  cx.S2 = S2; cx.mx = mx; cx.n = n; cx.denf = (float)(2 * qmax - 1);
  cx.u = 0x1p-24;
  cx.fixu = ldexp(1.0, -hist_fixed_exp(mx, v.nelem, qmax));
  cx.Kterm = (double)v.nq * ldexp(1.0, -fixed_exp(mx, v.nq));
  cx.Nterm = (double)((long long)v.nelem * qmax);
  cx.tiny = 8.0 * (double)v.nelem * 0x1p-149;
  double mymin = 1e300;
  {
    unsigned long long t1 = above1, t2 = above2;
    for (int c = c1 - 1; c >= c0; --c) {
      double lo, hi;
      cx.bounds(c, t1, t2, lo, hi);
      mymin = fmin(mymin, hi);
      t1 += H1[c]; t2 += H2[c];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mymin = fmin(mymin, __shfl_xor(mymin, off));
  unsigned long long keep = 0ull;                  // bit (c - c0) set: c in S (P <= 16)
  int cnt = 0;
  {
    unsigned long long t1 = above1, t2 = above2;
    for (int c = c1 - 1; c >= c0; --c) {
      double lo, hi;
      cx.bounds(c, t1, t2, lo, hi);
      if (lo <= mymin || g_sel_widen != 0) { keep |= 1ull << (c - c0); ++cnt; }
      t1 += H1[c]; t2 += H2[c];
    }
  }
  int pre = cnt;                                   // inclusive prefix over lanes
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(pre, off);
    if (lane >= off) pre += o;
  }
  const int total = __shfl(pre, 63);
  int pos = pre - cnt;
  for (int c = c0; c < c1; ++c) {
    if ((keep >> (c - c0)) & 1ull) {
      if (pos < kMaxSel) { sel[2 + pos] = c; lsel[2 + pos] = c; }
      ++pos;
    }
  }
  if (lane == 0) {   // sel = {|S| (n: exhaustive), unused, S ascending...}; |S| == 1 -> c* = sel[2]
    if (total > kMaxSel || total == 0) { sel[0] = n; sel[1] = -1; }
    else { sel[0] = total; sel[1] = 0; }
    lsel[0] = sel[0]; lsel[1] = sel[1];
    if (ADMMQ_TRACE) atomicAdd(&g_sel_stats[(total == 1) ? 0 : ((total > kMaxSel || total == 0) ? 2 : 1)], 1ull);
  }
}

// Stage 2 inside the last stage-1 block of a job (|S| > 1 is rare: ~0.1 % of the
// selections on the benchmark workload): the canonical SSE of every candidate in S
// (or of all of them) over the job's quads, 512-quad tiles staged in LDS, into v.sse.
// Removes a separate stage-2 launch from every iteration.
__device__ void sse_in_block(const MseView& v, const int* lsel, int ncand, int bits, int slot, float mx, float4* xs) {
  const int ns = lsel[0];
  if (ns == 1) return;
  const bool all = ns >= ncand;
  const int K = fixed_exp(mx, v.nq);
  for (int q0 = 0; q0 < v.nq; q0 += kSseQuads) {
    const int nqc = min(kSseQuads, v.nq - q0);
    for (int t = threadIdx.x; t < nqc; t += blockDim.x) {
      const int qi = q0 + t;
      const int row = qi / v.qpr;
      const int qc = qi - row * v.qpr;
      xs[t] = load_x4(v.X, v.U, (long long)row * v.ld + 4 * qc);
    }
    __syncthreads();
    sse_sweep_list(xs, nqc, mx, K, ncand, bits, all ? nullptr : lsel + 2, all ? ncand : ns,
                   v.sse + (size_t)slot * ncand);
    __syncthreads();
  }
}

// Stage 1. Each element x (a = |x|) has level k reached by candidate c iff
// a >= thr[k][c]; levels k <= kfull are reached by every candidate (b_k = n, summed
// in registers), levels kfull < k <= k0 have a breakpoint b_k in [1, n-1]: a linear
// estimate from t_c ~ S0 + c step (off by at most one) checked against the two
// neighbouring thresholds (one ds_read2), corrected, and re-verified in a rare slow
// path. QMAX = 2^(bits-1) is a template argument so the level loop unrolls and the
// LDS reads of all levels of an element are in flight together.
// 1024 threads x 4 elements per block; the block's histograms are flushed into one of
// kHistRep replicas of the job's global histograms; the last block of the job to
// finish (ticket) sums the replicas and runs the candidate selection.
template <int QMAX, int NV>
__global__ __launch_bounds__(1024, 8) void k_mse_hist(const ProbDesc* __restrict__ d, const QJob* __restrict__ qj,
                                                   const Chunk* __restrict__ chunks, int ncand, int slot, int abl) {
  const unsigned long long T0 = ADMMQ_NOW();
  const Chunk ck = chunks[blockIdx.x];
  const MseView& v = mview(d, qj, ck.job);
  if (v.done && *v.done) return;
  int* sel = v.sel + (size_t)slot * (2 + kMaxSel);
  const float mx = __uint_as_float(v.stat[4 * slot]);
  if (mse_degenerate(mx)) {     // finalize emits NaN for degenerate mx
    if (ck.start == 0 && threadIdx.x == 0) { sel[0] = 1; sel[1] = 0; }
    return;
  }
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = ncand;
  const int nb = n + 1 + 64;   // bins 0..n, then one private dummy bin per lane (branch-free atomics)
  unsigned long long* h1 = reinterpret_cast<unsigned long long*>(smem);          // nb
  unsigned* h2 = reinterpret_cast<unsigned*>(h1 + nb);                            // nb
  float* thr = reinterpret_cast<float*>(h2 + ((nb + 3) & ~3));                    // [QMAX][n]
  __shared__ double red[16];
  __shared__ int last;
  // this thread's 4 elements: issued first, so the load overlaps the table setup
  const long long total = ck.total;   // the unit's end (ADMM units are whole rows; standalone: the job's end)
  float4 x4v[NV];   // NV float4 per thread: start + 4 tid + 4096 g
#pragma unroll
  for (int g = 0; g < NV; ++g) {
    const long long e = (long long)ck.start + 4LL * threadIdx.x + 4096LL * g;
    x4v[g] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < total) x4v[g] = load_x4(v.X, v.U, e);
  }
  fill_thresholds(thr, mx, n, QMAX, blockDim.x);
  if (abl & 32) { __syncthreads(); fill_thresholds(thr, mx, n, QMAX, blockDim.x); }
  for (int b = threadIdx.x; b < nb; b += blockDim.x) { h1[b] = 0ull; h2[b] = 0u; }
  __syncthreads();
  const unsigned long long T1 = ADMMQ_NOW();
  const float S0 = (float)(0.2 * (double)mx);
  const float E0 = (float)(1.2 * (double)mx);
  const float inv_step = (n > 1) ? (float)(n - 1) / (E0 - S0) : 0.f;
  const int K1 = hist_fixed_exp(mx, v.nelem, QMAX);
  const int dummy = n + 1 + (threadIdx.x & 63);
  float tlo0[QMAX], thin[QMAX];   // per level: thresholds of the first and the last candidate
#pragma unroll
  for (int k = 0; k < QMAX; ++k) { tlo0[k] = thr[k * n]; thin[k] = thr[k * n + n - 1]; }
  double s2 = 0.0;
  unsigned long long full1 = 0ull;
  unsigned full2 = 0u;
#pragma unroll
  for (int j = 0; j < 4 * NV; ++j) {
    const float4 q4 = x4v[j >> 2];
    const float x = (j & 3) == 0 ? q4.x : ((j & 3) == 1 ? q4.y : ((j & 3) == 2 ? q4.z : q4.w));
    hist_insert_elem<QMAX>(x, thr, n, S0, inv_step, K1, dummy, tlo0, thin, h1, h2, s2, full1, full2);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s2 += __shfl_xor(s2, off);
    full1 += __shfl_xor(full1, off);
    full2 += (unsigned)__shfl_xor((int)full2, off);
  }
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = s2;
    if (full1) atomicAdd(&h1[n], full1);
    if (full2) atomicAdd(&h2[n], full2);
  }
  __syncthreads();
  const unsigned long long T2 = ADMMQ_NOW();
  const int rep = blockIdx.x & (kHistRep - 1);
  unsigned long long* g1 = v.h1 + (size_t)slot * kHistRep * (n + 1);
  unsigned long long* g2 = v.h2 + (size_t)slot * kHistRep * (n + 1);
  for (int b = threadIdx.x; b <= n; b += blockDim.x) {
    if (h1[b]) atomicAdd(&g1[rep * (n + 1) + b], h1[b]);
    if (h2[b]) atomicAdd(&g2[rep * (n + 1) + b], (unsigned long long)h2[b]);
  }
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    atomicAdd(&v.s2[slot], t);
  }
  // ticket: the last block of this job to arrive selects the candidate set. Everything
  // it reads was written by device-scope atomics (performed at the coherence point), so
  // draining this block's outstanding atomics (vmcnt(0)) orders them before the ticket;
  // no L2 writeback (a release fence per block costs ~100+ us over the grid).
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0)
    last = (__hip_atomic_fetch_add(&v.ticket[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (unsigned)(v.nhist - 1)) ? 1 : 0;
  __syncthreads();
  const unsigned long long T3 = ADMMQ_NOW();
  auto trace = [&](unsigned long long T4) {
    if (ADMMQ_TRACE && threadIdx.x == 0 && blockIdx.x < kHistTraceMax) {
      g_hist_trace[blockIdx.x][0] = T0; g_hist_trace[blockIdx.x][1] = T1; g_hist_trace[blockIdx.x][2] = T2;
      g_hist_trace[blockIdx.x][3] = T3; g_hist_trace[blockIdx.x][4] = T4;
      g_hist_trace[blockIdx.x][5] = ((unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) << 32) |
                                    __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    }
  };
  if (!last) { trace(T3); return; }
  // every byte handed over by the other blocks (h1/h2 replicas, s2) was written by
  // memory-side atomics drained before the ticket and is read below by agent-scope
  // (sc1) atomic loads only, so no L1 invalidate is needed (cdna_hip_programming.md
  // Guideline 16, sc1 consumer); the wavefront fence only keeps the loads after the ticket
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  unsigned long long* H1 = h1;                                            // reuse LDS: n+1 each
  unsigned long long* H2 = reinterpret_cast<unsigned long long*>(thr);
  for (int b = threadIdx.x; b <= n; b += blockDim.x) {
    unsigned long long t1 = 0ull, t2 = 0ull;
#pragma unroll
    for (int r = 0; r < kHistRep; ++r) {
      t1 += __hip_atomic_load((gu64*)&g1[r * (n + 1) + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t2 += __hip_atomic_load((gu64*)&g2[r * (n + 1) + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    H1[b] = t1; H2[b] = t2;
  }
  __syncthreads();
  __shared__ int lsel[2 + kMaxSel];
  if (threadIdx.x < 64) {
    const double S2 = __hip_atomic_load((__attribute__((address_space(1))) double*)&v.s2[slot], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    select_wave(v, sel, lsel, H1, H2, S2, mx, n, QMAX);
  }
  __syncthreads();
  sse_in_block(v, lsel, n, QMAX == 1 ? 1 : 31 - __builtin_clz(QMAX) + 1, slot, mx, reinterpret_cast<float4*>(smem));
  trace(ADMMQ_NOW());
}

// ---------------------------------------------------------------------------
// Stage 1, merged-threshold form (k_mse_hist3; qmax * ncand <= kMaxMerged).
//
// With B(a) = #{(k, c) : thr[k][c] <= a} over ALL levels and candidates and
// L(k, c) = #{(k', c') : thr[k'][c'] <= thr[k][c]} (ties counted), for every a >= 0:
//     a >= thr[k][c]  <=>  B(a) >= L(k, c).
// So each element is placed once, in bucket B(|x|), and per candidate
//     T1(c) = sum_k sum{ af : B >= L(k, c) },   T2(c) = sum_k (2k-1) #{ B >= L(k, c) }
// over the elements allowed level k (x > 0 reaches at most qmax - 1, so the top level
// reads the negatives' buckets only): the same integers as the per-level breakpoint
// sums of k_mse_hist (each (element, level) pair contributes af once).
//
// The sorted order of the thresholds does not depend on mx: thr[k][c] is within a few
// ulps of (2k-1) ((n-1) + 5c) * mx / (5 (n-1) den), an integer key whose distinct
// values differ by >= 1.5e-5 relative for every supported (n, qmax). The host
// computes that order once (rank0) with the groups of exactly equal keys; each block
// scatters its thresholds by it, orders the tie groups by their actual values,
// checks the result is non-decreasing (else ranks them by counting) and derives L.
// A coarse index cnt[g] = #{thresholds in cells < g} over kCells equal cells of
// [0, max threshold] then turns B(a) into two independent LDS reads and a walk of
// the few thresholds of a's cell.
constexpr int kH3Threads = 512;       // k_mse_hist3 block (its helpers take the size as a constant:
constexpr int kSmallThreads = 1024;   // k_mse_small_admm block  reading blockDim is a global load)

// Candidate selection from per-candidate totals T1/T2 (LDS) and S2, by one wave:
// as select_wave, without the suffix scan.
__device__ void select_wave2(const MseView& v, int* sel, int* lsel, const unsigned long long* T1v,
                             const unsigned long long* T2v, double S2, float mx, int n, int qmax) {
  const int lane = threadIdx.x & 63;
  const int P = (n + 63) / 64;
  const int c0 = lane * P, c1 = min(c0 + P, n);
  SelCtx cx;
  cx.S2 = S2; cx.mx = mx; cx.n = n; cx.denf = (float)(2 * qmax - 1);
  cx.u = 0x1p-24;
  cx.fixu = ldexp(1.0, -hist_fixed_exp(mx, v.nelem, qmax));
  cx.Kterm = (double)v.nq * ldexp(1.0, -fixed_exp(mx, v.nq));
  cx.Nterm = (double)((long long)v.nelem * qmax);
  cx.tiny = 8.0 * (double)v.nelem * 0x1p-149;
  double mymin = 1e300;
  for (int c = c0; c < c1; ++c) {
    double lo, hi;
    cx.bounds(c, T1v[c], T2v[c], lo, hi);
    mymin = fmin(mymin, hi);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mymin = fmin(mymin, __shfl_xor(mymin, off));
  unsigned long long keep = 0ull;                  // bit (c - c0) set: c in S (P <= 16)
  int cnt = 0;
  for (int c = c0; c < c1; ++c) {
    double lo, hi;
    cx.bounds(c, T1v[c], T2v[c], lo, hi);
    if (lo <= mymin || g_sel_widen != 0) { keep |= 1ull << (c - c0); ++cnt; }
  }
  int pre = cnt;                                   // inclusive prefix over lanes
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(pre, off);
    if (lane >= off) pre += o;
  }
  const int total = __shfl(pre, 63);
  int pos = pre - cnt;
  for (int c = c0; c < c1; ++c) {
    if ((keep >> (c - c0)) & 1ull) {
      if (pos < kMaxSel) { sel[2 + pos] = c; lsel[2 + pos] = c; }
      ++pos;
    }
  }
  if (lane == 0) {
    if (total > kMaxSel || total == 0) { sel[0] = n; sel[1] = -1; }
    else { sel[0] = total; sel[1] = 0; }
    lsel[0] = sel[0]; lsel[1] = sel[1];
    if (ADMMQ_TRACE) atomicAdd(&g_sel_stats[(total == 1) ? 0 : ((total > kMaxSel || total == 0) ? 2 : 1)], 1ull);
  }
}

// The same selection by the whole block, one candidate per thread (n <= blockDim.x):
// thread c holds T1(c), T2(c) in registers; the bounds are computed once per candidate
// (the one-wave form walks ceil(n/64) candidates per lane twice, a serial fp64 chain of
// ~4 us); min(A + E) and the ascending list of S come from block reductions. Ends with
// a block barrier (lsel visible to every thread).
__device__ void select_block(const MseView& v, int* sel, int* lsel, unsigned long long t1, unsigned long long t2,
                             double S2, float mx, int n, int qmax) {
  __shared__ double wmin[16];
  __shared__ int wcnt[16];
  const int c = threadIdx.x, lane = c & 63, w = c >> 6, nw = (int)(blockDim.x >> 6);
  SelCtx cx;
  cx.S2 = S2; cx.mx = mx; cx.n = n; cx.denf = (float)(2 * qmax - 1);
  cx.u = 0x1p-24;
  cx.fixu = ldexp(1.0, -hist_fixed_exp(mx, v.nelem, qmax));
  cx.Kterm = (double)v.nq * ldexp(1.0, -fixed_exp(mx, v.nq));
  cx.Nterm = (double)((long long)v.nelem * qmax);
  cx.tiny = 8.0 * (double)v.nelem * 0x1p-149;
  double lo = 1e300, hi = 1e300;
  if (c < n) cx.bounds(c, t1, t2, lo, hi);
  const double m = wave_min_f64(hi);
  if (lane == 0) wmin[w] = m;
  __syncthreads();
  double mn = wmin[0];
  for (int k = 1; k < nw; ++k) mn = fmin(mn, wmin[k]);
  const bool keep = c < n && (lo <= mn || g_sel_widen != 0);
  const unsigned long long bal = __ballot(keep);
  if (lane == 0) wcnt[w] = __popcll(bal);
  __syncthreads();
  int pos = __popcll(bal & ((1ull << lane) - 1ull)), total = 0;
  for (int k = 0; k < nw; ++k) { pos += k < w ? wcnt[k] : 0; total += wcnt[k]; }
  if (keep && pos < kMaxSel) { sel[2 + pos] = c; lsel[2 + pos] = c; }
  if (c == 0) {
    if (total > kMaxSel || total == 0) { sel[0] = n; sel[1] = -1; }
    else { sel[0] = total; sel[1] = 0; }
    lsel[0] = sel[0]; lsel[1] = sel[1];
    if (ADMMQ_TRACE) atomicAdd(&g_sel_stats[(total == 1) ? 0 : ((total > kMaxSel || total == 0) ? 2 : 1)], 1ull);
  }
  __syncthreads();
}


// Rank-by-counting of the thresholds (fallback when the host order does not hold):
// rows thr[j][.] are non-decreasing; with the order (value, level, candidate)
// rank(k, c) = sum_{j<k} #{row j <= T} + c + sum_{j>k} #{row j < T}, L = sum_j #{row j <= T}.
__device__ void rank_by_counting(const float* thr, float* tsort, unsigned short* L_out, float mx, int n, int qmax) {
  const int M = qmax * n;
  const float S0 = (float)(0.2 * (double)mx);
  const float E0 = (float)(1.2 * (double)mx);
  const float inv_step = (n > 1) ? (float)(n - 1) / (E0 - S0) : 0.f;
  const float den = (float)(2 * qmax - 1);
  for (int e = threadIdx.x; e < M; e += blockDim.x) {
    const int k = e / n, c = e - k * n;
    const float T = thr[e];
    int rank = c, L = 0;
    for (int j = 0; j < qmax; ++j) {
      const float* row = thr + j * n;
      int le;
      if (j == k) {
        le = c + 1;
        while (le < n && row[le] <= T) ++le;
      } else {
        const float ce = (T * den / (float)(2 * j + 1) - S0) * inv_step;
        le = (ce < 0.f) ? 0 : (ce >= (float)n ? n : (int)ce + 1);
        while (le < n && row[le] <= T) ++le;
        while (le > 0 && row[le - 1] > T) --le;
      }
      L += le;
      if (j < k) rank += le;
      if (j > k) {
        int lt = le;
        while (lt > 0 && row[lt - 1] == T) --lt;
        rank += lt;
      }
    }
    L_out[e] = (unsigned short)L;
    tsort[rank] = T;
  }
}

// Diagnostics: s_memrealtime stamps inside the stage-1 table setup of the last launch, per
// block {start, thresholds + host order in LDS, ties ordered, L, cells} (admmq_debug_setup_trace).
constexpr int kSetupTraceMax = 4096;
__device__ unsigned long long g_setup_trace[kSetupTraceMax][5];
int copy_setup_trace(unsigned long long* host, int n) {
  n = n < kSetupTraceMax ? n : kSetupTraceMax;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_setup_trace), (size_t)n * 5 * sizeof(unsigned long long)) == hipSuccess
             ? n : -1;
}
// Phase stamps of k_mse_small_admm's blocks (last launch): {start, loads+flag, setup,
// insert, suffix, select, stage 2, end} and the selected-list length (admmq_debug_small_trace).
constexpr int kSmallTraceMax = 64;
__device__ unsigned long long g_small_trace[kSmallTraceMax][9];
int copy_small_trace(unsigned long long* host, int n) {
  n = n < kSmallTraceMax ? n : kSmallTraceMax;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_small_trace), (size_t)n * 9 * sizeof(unsigned long long)) == hipSuccess
             ? n : -1;
}
#define ADMMQ_SMALL_STAMP(k) \
  if (ADMMQ_TRACE && threadIdx.x == 0 && blockIdx.x < kSmallTraceMax) g_small_trace[blockIdx.x][k] = ADMMQ_NOW()
#define ADMMQ_SETUP_STAMP(k) \
  if (ADMMQ_TRACE && threadIdx.x == 0 && blockIdx.x < kSetupTraceMax) g_setup_trace[blockIdx.x][k] = ADMMQ_NOW()

// The global inputs of the stage-1 table setup that do not depend on max|x|: this
// thread's entries of the host order of the thresholds (blocks of >= 512 threads) and
// its tie group (packed 6 x u16). The kernels issue these loads before their element
// loads: vector loads complete in issue order, so issued after the elements any wait for
// them would wait for all of the elements too.
constexpr int kR0 = (kMaxMerged + 511) / 512;
struct H3Pre {
  unsigned short r0v[kR0];
  unsigned gw[3];
};
__device__ __forceinline__ void h3_load_order(const unsigned short* __restrict__ rank0, int M,
                                              const unsigned short* __restrict__ groups, int ngroups, H3Pre& pre, int nt) {
  // unconditional loads (clamped index; entries past M / ngroups are ignored), so the
  // compiler's wait counts stay exact: rank0 holds kMaxMerged entries and groups
  // kMaxMerged / 2 groups of 12 B (4-byte aligned), whatever M and ngroups are
#pragma unroll
  for (int j = 0; j < kR0; ++j) {
    const int i = threadIdx.x + j * nt;
    pre.r0v[j] = rank0[min(i, M - 1)];
  }
  const unsigned* g32 = reinterpret_cast<const unsigned*>(groups + 6 * min((int)threadIdx.x, kMaxMerged / 2 - 1));
  pre.gw[0] = g32[0]; pre.gw[1] = g32[1]; pre.gw[2] = g32[2];
  (void)ngroups;
}

// Stage-1 table of one job in LDS (the setup of k_mse_hist3 and k_mse_small_admm): the
// thresholds in the host's merged order with the tie groups ordered by value, L per
// (level, candidate), the coarse cell index; the buckets zeroed. Returns the cell scale.
//
// L and the cell index come almost entirely from the host (they do not depend on mx):
// distinct keys give distinct thresholds, so L = rank + 1 outside the tie groups, and
// cells_g[g] (after the kMaxMerged rank entries of the host order) is a LOWER bound of
// #{thresholds in cells < g} valid for every mx: the host counts the thresholds whose
// key puts them below cell g with a 1e-4 relative margin (the thresholds are within a
// few ulps of their key's proportion of the largest one). h3_insert_n starts each
// element's search there and walks up to the exact count. If the host order does not
// hold for this mx (never observed), everything is derived in the block instead.
template <int QMAX>
__device__ __forceinline__ float h3_setup(float mx, int n, const H3Pre& pre,
                                         const unsigned short* __restrict__ groups, int ngroups,
                                         const unsigned short* __restrict__ cells_g,
                                         unsigned long long* sumA, unsigned long long* sumN, unsigned* cntA,
                                         unsigned* cntN, float* thr, float* tsort, unsigned short* rnk,
                                         unsigned short* cell, int nt) {
  const int M = QMAX * n;
  const int nb = M + 1 + 64;
  ADMMQ_SETUP_STAMP(0);
  // the host cell index (kCells + 1 entries as u32 pairs), issued first: used only at
  // the end of the setup
  constexpr int kCellWords = (kCells + 2) / 2;
  const unsigned* cw = reinterpret_cast<const unsigned*>(cells_g);
  unsigned cv[(kCellWords + 511) / 512];
  const int ncw = (kCellWords + nt - 1) / nt;
#pragma unroll
  for (int j = 0; j < (kCellWords + 511) / 512; ++j)
    if (j < ncw) cv[j] = gld_u32(cw + min((int)threadIdx.x + j * nt, kCellWords - 1));
  // the candidates' scales s_c = fl(2 t_c / den), one division each (not one per level and
  // candidate), in LDS after the cell index (hist3_lds_bytes)
  const float den = (float)(2 * QMAX - 1);
  float* scand = reinterpret_cast<float*>(cell + kCells + 2);   // 4-B aligned: cell is, kCells + 2 is even
  for (int c = threadIdx.x; c < n; c += nt) scand[c] = (2.0f * cand_t(mx, c, n)) / den;
  __syncthreads();
  // thresholds, each also scattered to its host-order rank (kR0 * nt >= kMaxMerged >= M);
  // L = rank + 1 (tie groups below)
#pragma unroll
  for (int j = 0; j < kR0; ++j) {
    const int e = threadIdx.x + j * nt;
    if (e < M) {
      const int k = 1 + e / n, c = e - (k - 1) * n;
      const float v = level_threshold_fast(scand[c], k);
      thr[e] = v;
      tsort[pre.r0v[j]] = v;
      rnk[e] = (unsigned short)(pre.r0v[j] + 1);
    }
  }
  for (int i = threadIdx.x; i < nb; i += nt) { sumA[i] = 0ull; sumN[i] = 0ull; cntA[i] = 0u; cntN[i] = 0u; }
  __syncthreads();
  ADMMQ_SETUP_STAMP(1);
  // exact-key ties: order by actual value, L = 1 + index of the last equal value (the
  // thread's first group was prefetched; a load in the same loop would, after the join,
  // make the compiler wait for every outstanding load, the elements included)
  auto tie_group = [&](const unsigned short* gr) {
    const int r0 = gr[0], m = gr[1];
    int es[4];
    float vs[4];
    for (int j = 0; j < m; ++j) { es[j] = gr[2 + j]; vs[j] = thr[es[j]]; }
    for (int i = 1; i < m; ++i)                                 // insertion sort, stable
      for (int j = i; j > 0 && vs[j - 1] > vs[j]; --j) {
        const float tv = vs[j]; vs[j] = vs[j - 1]; vs[j - 1] = tv;
        const int te = es[j]; es[j] = es[j - 1]; es[j - 1] = te;
      }
    for (int j = 0; j < m; ++j) {
      int l = j;
      while (l + 1 < m && vs[l + 1] == vs[j]) ++l;
      tsort[r0 + j] = vs[j];
      rnk[es[j]] = (unsigned short)(r0 + l + 1);
    }
  };
  if ((int)threadIdx.x < ngroups) {
    const unsigned short gr[6] = {(unsigned short)(pre.gw[0] & 0xFFFFu), (unsigned short)(pre.gw[0] >> 16),
                                  (unsigned short)(pre.gw[1] & 0xFFFFu), (unsigned short)(pre.gw[1] >> 16),
                                  (unsigned short)(pre.gw[2] & 0xFFFFu), (unsigned short)(pre.gw[2] >> 16)};
    tie_group(gr);
  }
  if (ngroups > nt)
    for (int g = threadIdx.x + nt; g < ngroups; g += nt) tie_group(groups + 6 * g);
  // the host cell index into LDS
  unsigned* cell32 = reinterpret_cast<unsigned*>(cell);
#pragma unroll
  for (int j = 0; j < (kCellWords + 511) / 512; ++j) {
    const int i = threadIdx.x + j * nt;
    if (j < ncw && i < kCellWords) cell32[i] = cv[j];
  }
  __syncthreads();
  ADMMQ_SETUP_STAMP(2);
  // the order check (sorted thresholds non-decreasing); the cell scale from the largest
  // threshold (level QMAX of the last candidate), computed directly
  int bad = 0;
  for (int r = threadIdx.x; r + 1 < M; r += nt) bad |= (tsort[r] > tsort[r + 1]) ? 1 : 0;
  const float inv = (float)kCells / level_threshold_fast((2.0f * cand_t(mx, n - 1, n)) / den, QMAX);
  // the host bound assumes normal-range thresholds (relative rounding): elsewhere, exact cells
  bad |= (mx >= 0x1p-100f && mx <= 0x1p100f) ? 0 : 1;
  if (__syncthreads_or(bad)) {   // never expected: rank by counting, exact cells (exact either way)
    rank_by_counting(thr, tsort, rnk, mx, n, QMAX);
    __syncthreads();
    const float inv2 = (float)kCells / tsort[M - 1];
    for (int r = threadIdx.x; r < M; r += nt) {
      const int cr = min(kCells - 1, (int)(tsort[r] * inv2));
      const int cp = r == 0 ? -1 : min(kCells - 1, (int)(tsort[r - 1] * inv2));
      for (int g = cp + 1; g <= cr; ++g) cell[g] = (unsigned short)r;
      if (r == M - 1)
        for (int g = cr + 1; g <= kCells; ++g) cell[g] = (unsigned short)M;
    }
    __syncthreads();
    ADMMQ_SETUP_STAMP(3);
    ADMMQ_SETUP_STAMP(4);
    return inv2;
  }
  ADMMQ_SETUP_STAMP(3);
  ADMMQ_SETUP_STAMP(4);
  return inv;
}

// Buckets B = #{thresholds <= |x|} of N elements and their LDS histogram adds, in phases whose LDS reads are independent across the
// elements (so their latencies overlap instead of chaining element after element): the
// cell's lower bound, then three threshold probes, then the walk for an element whose cell
// still holds more thresholds <= |x| (rare), then the histogram adds.
template <int N>
__device__ __forceinline__ void h3_insert_n(const float* xs, float inv, const float* tsort, const unsigned short* cell,
                                            int M, int K1, int dummy, unsigned long long* sumA,
                                            unsigned long long* sumN, unsigned* cntA, unsigned* cntN) {
  float a[N];
  int B[N], hi[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {   // start at the cell's lower bound (h3_setup); the upper bound is M
    a[j] = __builtin_fabsf(xs[j]);
    const int g = min(kCells - 1, (int)(a[j] * inv));
    B[j] = cell[g];
    hi[j] = M;
  }
  bool more[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int b0 = B[j];
    const float p0 = tsort[min(b0, M - 1)], p1 = tsort[min(b0 + 1, M - 1)], p2 = tsort[min(b0 + 2, M - 1)];
    const int cnt = (b0 < hi[j] && p0 <= a[j] ? 1 : 0) + (b0 + 1 < hi[j] && p1 <= a[j] ? 1 : 0) +
                    (b0 + 2 < hi[j] && p2 <= a[j] ? 1 : 0);   // sorted: the prefix of <= a
    B[j] = b0 + cnt;
    more[j] = cnt == 3;
  }
#pragma unroll
  for (int j = 0; j < N; ++j)
    if (more[j])
      while (B[j] < hi[j] && tsort[B[j]] <= a[j]) ++B[j];   // B = #{thresholds <= a}
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const bool live = B[j] > 0;
    const int b = live ? B[j] : dummy;
    const bool neg = xs[j] < 0.f;
    const unsigned long long af = live ? to_fixed(a[j], K1) : 0ull;
    atomicAdd(neg ? &sumN[b] : &sumA[b], af);
    atomicAdd(neg ? &cntN[b] : &cntA[b], live ? 1u : 0u);
  }
}

// all = positives + negatives, then suffix sums S[i] = sum over buckets >= i of the four
// bucket arrays in one block pass: contiguous per-thread runs, then a scan of the run
// totals over the block (in thread order; the wave totals are summed by an unrolled,
// predicated loop, so their reads are issued together). Runs of up to PMAX buckets are
// held in registers (one round of independent LDS reads, one of writes); longer ones
// are walked in LDS. PMAX = 0: the walk in LDS and a plain loop over the wave totals
// (fewest registers). Ends with a block barrier.
template <int NT, int PMAX>
__device__ __forceinline__ void h3_suffix(int M, unsigned long long* sumA, unsigned long long* sumN, unsigned* cntA,
                                          unsigned* cntN, unsigned long long* wtot, unsigned long long* wtot2,
                                          unsigned* wtot32, unsigned* wtot32b) {
  constexpr int NW = NT / 64;
  const int len = M + 1;
  const int per = (len + NT - 1) / NT;
  const int b0 = threadIdx.x * per, b1 = min(b0 + per, len);
  if constexpr (PMAX == 0) {   // fewest registers (the 1024-thread kernel holds its elements across this)
    unsigned long long r1 = 0ull, r2 = 0ull;
    unsigned r3 = 0u, r4 = 0u;
    for (int i = b1 - 1; i >= b0; --i) {
      const unsigned long long sn = sumN[i];
      const unsigned c = cntN[i];
      r1 += sumA[i] + sn; sumA[i] = r1;
      r2 += sn; sumN[i] = r2;
      r3 += cntA[i] + c; cntA[i] = r3;
      r4 += c; cntN[i] = r4;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // wave suffix sums (DPP); the lanes above this one hold q - r
    const unsigned long long q1 = wave_suffix_u64(r1), q2 = wave_suffix_u64(r2);
    const unsigned q3 = wave_suffix_u32(r3), q4 = wave_suffix_u32(r4);
    if (lane == 0) { wtot[w] = q1; wtot2[w] = q2; wtot32[w] = q3; wtot32b[w] = q4; }
    __syncthreads();
    unsigned long long a1 = q1 - r1, a2 = q2 - r2;
    unsigned a3 = q3 - r3, a4 = q4 - r4;
    for (int j = w + 1; j < NW; ++j) { a1 += wtot[j]; a2 += wtot2[j]; a3 += wtot32[j]; a4 += wtot32b[j]; }
    for (int i = b0; i < b1; ++i) { sumA[i] += a1; sumN[i] += a2; cntA[i] += a3; cntN[i] += a4; }
    __syncthreads();
    return;
  }
  constexpr int PM = PMAX > 0 ? PMAX : 1;
  const bool inreg = per <= PMAX;   // block-uniform
  unsigned long long ra[PM], rn[PM];
  unsigned ca[PM], cn[PM];
  unsigned long long r1 = 0ull, r2 = 0ull;
  unsigned r3 = 0u, r4 = 0u;
  if (inreg) {
#pragma unroll
    for (int i = 0; i < PM; ++i) {
      const int idx = b0 + i;
      const bool ok = idx < b1;
      ra[i] = ok ? sumA[idx] : 0ull; rn[i] = ok ? sumN[idx] : 0ull;
      ca[i] = ok ? cntA[idx] : 0u;   cn[i] = ok ? cntN[idx] : 0u;
    }
#pragma unroll
    for (int i = PM - 1; i >= 0; --i) {   // entries past the run are zero
      r1 += ra[i] + rn[i]; r2 += rn[i]; r3 += ca[i] + cn[i]; r4 += cn[i];
      ra[i] = r1; rn[i] = r2; ca[i] = r3; cn[i] = r4;
    }
  } else {
    for (int i = b1 - 1; i >= b0; --i) {
      const unsigned long long sn = sumN[i];
      const unsigned c = cntN[i];
      r1 += sumA[i] + sn; sumA[i] = r1;
      r2 += sn; sumN[i] = r2;
      r3 += cntA[i] + c; cntA[i] = r3;
      r4 += c; cntN[i] = r4;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // wave suffix sums (DPP); the lanes above this one hold q - r
  const unsigned long long q1 = wave_suffix_u64(r1), q2 = wave_suffix_u64(r2);
  const unsigned q3 = wave_suffix_u32(r3), q4 = wave_suffix_u32(r4);
  if (lane == 0) { wtot[w] = q1; wtot2[w] = q2; wtot32[w] = q3; wtot32b[w] = q4; }
  __syncthreads();
  unsigned long long a1 = q1 - r1, a2 = q2 - r2;
  unsigned a3 = q3 - r3, a4 = q4 - r4;
#pragma unroll
  for (int j = 1; j < NW; ++j)
    if (j > w) { a1 += wtot[j]; a2 += wtot2[j]; a3 += wtot32[j]; a4 += wtot32b[j]; }
  if (inreg) {
#pragma unroll
    for (int i = 0; i < PM; ++i) {
      const int idx = b0 + i;
      if (idx < b1) { sumA[idx] = ra[i] + a1; sumN[idx] = rn[i] + a2; cntA[idx] = ca[i] + a3; cntN[idx] = cn[i] + a4; }
    }
  } else {
    for (int i = b0; i < b1; ++i) { sumA[i] += a1; sumN[i] += a2; cntA[i] += a3; cntN[i] += a4; }
  }
  __syncthreads();
}

// Per-candidate level sums T1(c), T2(c) from the suffix-summed buckets (x > 0 reaches at
// most qmax - 1 levels, so the top level reads the negatives' buckets only).
template <int QMAX>
__device__ __forceinline__ void h3_totals(int c, int n, const unsigned short* rnk, const unsigned long long* sumA,
                                          const unsigned long long* sumN, const unsigned* cntA, const unsigned* cntN,
                                          unsigned long long& t1, unsigned long long& t2) {
  t1 = 0ull; t2 = 0ull;
#pragma unroll
  for (int k = 1; k < QMAX; ++k) {
    const int L = rnk[(k - 1) * n + c];
    t1 += sumA[L];
    t2 += (unsigned long long)(2 * k - 1) * cntA[L];
  }
  const int L = rnk[(QMAX - 1) * n + c];
  t1 += sumN[L];
  t2 += (unsigned long long)(2 * QMAX - 1) * cntN[L];
}

// FIN (ADMM jobs only): the search launch also runs the finalize step (k_finalize_admm's
// projection + dual update + next right-hand side) on the block's own elements, which
// it already holds: units are whole rows, every block of the launch is resident at once
// (the host checks the occupancy), and after its ticket each block waits for its job's
// selection. The last block of a job publishes the selection record with write-through
// (sc1) stores, then the job's ready word = iter + 1; the others poll that word (one
// wave, relaxed agent-scope loads with s_sleep) and read the record with sc1 loads. The
// wait is bounded (`wait_polls`, ~10 ms by default): past it the block sets flags[3]
// (reported as an internal fault in admmq_admm_run's info) and ends WITHOUT finalizing
// its elements, so a broken residency assumption can neither hang the GPU nor finalize
// with a stale selection record; the caller re-runs the call with the separate finalize
// launch (the PyTorch op does). Saves the finalize launch, its dependent parameter chain
// and its re-read of H_T and U.
#ifndef ADMMQ_FIN_STREAM
#define ADMMQ_FIN_STREAM 1
#endif
constexpr bool kFinStream = ADMMQ_FIN_STREAM != 0;   // the fused finalize stores each group at once
// NV = 3 (FIN: the launches whose units would not all be resident at 2 groups per thread,
// e.g. C4): U is re-read with H and F for the finalize instead of held across the search
// (its registers are what would spill), an L2 hit written by the solve's epilogue.
template <int QMAX, int NV, bool FIN>
__global__ __launch_bounds__(kH3Threads, 4) void k_mse_hist3(
    const ProbDesc* __restrict__ d, const QJob* __restrict__ qj, const Chunk* __restrict__ chunks, int ncand, int slot,
    const unsigned short* __restrict__ rank0, const unsigned short* __restrict__ groups, int ngroups, int bits,
    int iter, unsigned wait_polls) {
  const unsigned long long T0 = ADMMQ_NOW();
  const Chunk ck = chunks[blockIdx.x];
  // first-needed inputs straight from the unit (one dependent level): stop flag, max|x|,
  // the threshold order, this thread's elements - all issued before any is used
  // (straight-line global loads; past the end a clamped address, zeroed below)
  const int stopped = gld_i32(ck.done ? ck.done : &g_no_stop);
  const float mx = __uint_as_float(gld_u32(ck.stat + 4 * slot));
  const long long total = ck.total;
  H3Pre pre;
  h3_load_order(rank0, QMAX * ncand, groups, ngroups, pre, kH3Threads);
  asm volatile("" ::: "memory");   // issue order: the loads above before the element loads
  constexpr bool kReloadU = FIN && NV >= 3;
  float4 x4[2 * NV], u4[2 * NV], h4[FIN ? 2 * NV : 1], f4[FIN ? 2 * NV : 1];
#pragma unroll
  for (int hh = 0; hh < 2 * NV; ++hh) {   // 8 NV elements: float4 hh at start + 4 tid + 2048 hh
    const long long e = (long long)ck.start + 4LL * threadIdx.x + 2048LL * hh;
    x4[hh] = gld4(ck.X + (e < total ? e : 0));
  }
  if (ck.U) {
#pragma unroll
    for (int hh = 0; hh < 2 * NV; ++hh) {
      const long long e = (long long)ck.start + 4LL * threadIdx.x + 2048LL * hh;
      u4[hh] = gld4(ck.U + (e < total ? e : 0));
    }
  }
  const MseView& v = mview(d, qj, ck.job);
  if (stopped) return;
  int* sel = v.sel + (size_t)slot * (2 + kMaxSel);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ double red[8];
  __shared__ unsigned long long wtot[8], wtot2[8];
  __shared__ unsigned wtot32[8], wtot32b[8];
  __shared__ int last;
  __shared__ int timed_out;
  __shared__ int lsel[2 + kMaxSel];
  const int n = ncand;
  // the finalize step's other inputs (current H, padded F): issued after the search
  // (FIN: before the wait for the selection), so they hold no registers during the search
  auto load_hf = [&]() {
#pragma unroll
    for (int hh = 0; hh < 2 * NV; ++hh) {
      const long long ec = (long long)ck.start + 4LL * threadIdx.x + 2048LL * hh;
      if constexpr (kReloadU) u4[hh] = gld4(ck.U + (ec < total ? ec : 0));
      h4[hh] = gld4(ck.H + (ec < total ? ec : 0));
      f4[hh] = gld4(ck.F + (ec < total ? ec : 0));
    }
  };
  if (mse_degenerate(mx)) {     // the projection emits NaN for degenerate mx (no search)
    if (ck.start == 0 && threadIdx.x == 0) { sel[0] = 1; sel[1] = 0; }
    if constexpr (FIN) {   // (one unit per block)
      const ProbDesc& p = d[ck.job];
#pragma unroll
      for (int hh = 0; hh < 2 * NV; ++hh) {
        const long long e = (long long)ck.start + 4LL * threadIdx.x + 2048LL * hh;
        const long long ec = e < total ? e : 0;
        h4[hh] = gld4(ck.H + ec);
        f4[hh] = gld4(ck.F + ec);
      }
      admm_finalize_block<kH3Threads, 2 * NV, kFinStream>(p, ck.start, total, x4, u4, h4, f4,
                                                    qparams_mse(bits, __builtin_nanf("")), slot, iter,
                                                    blockIdx.x & (kResRep - 1), reinterpret_cast<unsigned*>(smem));
    }
    return;
  }
  const int M = QMAX * n;
  const int nb = M + 1 + 64;                  // buckets 0..M, then one private dummy per lane
  unsigned long long* sumA = reinterpret_cast<unsigned long long*>(smem);   // positives, then all
  unsigned long long* sumN = sumA + nb;
  unsigned* cntA = reinterpret_cast<unsigned*>(sumN + nb);
  unsigned* cntN = cntA + nb;
  float* thr = reinterpret_cast<float*>(cntN + nb);                          // M
  float* tsort = thr + M;                                                    // M
  unsigned short* rnk = reinterpret_cast<unsigned short*>(tsort + M);        // M: rank, then L
  unsigned short* cell = rnk + ((M + 1) & ~1);                               // kCells + 1
  const float inv = h3_setup<QMAX>(mx, n, pre, groups, ngroups, rank0 + kMaxMerged, sumA, sumN, cntA, cntN, thr, tsort,
                                   rnk, cell, kH3Threads);
  const unsigned long long T1 = ADMMQ_NOW();
  const int K1 = hist_fixed_exp(mx, v.nelem, QMAX);
  const int dummy = M + 1 + (threadIdx.x & 63);
  double s2 = 0.0;
  // a block may take several consecutive units of its job (ck.reps, `step` elements each):
  // one table setup and one flush for all of them (not FIN: the fused finalize's launch
  // has one unit per block, all resident)
  const int reps = FIN ? 1 : max(ck.reps, 1);
  if constexpr (!FIN) {
    // several units per block: X - U of unit r is formed first (its x4 / u4 registers are
    // then free), the loads of unit r + 1 are issued into them, and unit r's inserts run
    // while those loads are in flight (the same elements, sums and order as one unit at a
    // time; 16 NV more VGPRs, not 32 NV)
    for (int r = 0; r < reps; ++r) {
      const long long ub = (long long)ck.start + (long long)r * ck.step;
      const long long ue = reps > 1 ? min(ub + ck.step, total) : total;
      float4 xv[2 * NV];
#pragma unroll
      for (int hh = 0; hh < 2 * NV; ++hh) {   // X - U (ADMM: H_T - U); zero past the end
        float4 xa = x4[hh];
        if (ck.U) xa = sub4(xa, u4[hh]);
        const long long e = ub + 4LL * threadIdx.x + 2048LL * hh;
        xv[hh] = e >= ue ? make_float4(0.f, 0.f, 0.f, 0.f) : xa;
      }
      if (r + 1 < reps) {
        const long long nb = ub + ck.step, ne = min(nb + ck.step, total);
#pragma unroll
        for (int hh = 0; hh < 2 * NV; ++hh) {
          const long long e = nb + 4LL * threadIdx.x + 2048LL * hh;
          x4[hh] = gld4(ck.X + (e < ne ? e : 0));
          if (ck.U) u4[hh] = gld4(ck.U + (e < ne ? e : 0));
        }
      }
#pragma unroll
      for (int hb = 0; hb < 2 * NV; hb += 2) {
        const float4 xa = xv[hb], xb = xv[hb + 1];
        const float xs[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) s2 += (double)xs[j] * (double)xs[j];
        h3_insert_n<8>(xs, inv, tsort, cell, M, K1, dummy, sumA, sumN, cntA, cntN);
      }
    }
  }
  for (int r = 0; FIN && r < reps; ++r) {
    const long long ub = (long long)ck.start + (long long)r * ck.step;   // unit r (r > 0: reps > 1 only)
    const long long ue = reps > 1 ? min(ub + ck.step, total) : total;
    if (r > 0) {   // this unit's elements (unit 0's were issued before the table setup)
#pragma unroll
      for (int hh = 0; hh < 2 * NV; ++hh) {
        const long long e = ub + 4LL * threadIdx.x + 2048LL * hh;
        x4[hh] = gld4(ck.X + (e < ue ? e : 0));
        if (ck.U) u4[hh] = gld4(ck.U + (e < ue ? e : 0));
      }
    }
#pragma unroll
    for (int hb = 0; hb < 2 * NV; hb += 2) {   // X - U (ADMM: H_T - U); zero past the end
      float4 xa = x4[hb], xb = x4[hb + 1];
      if (ck.U) { xa = sub4(xa, u4[hb]); xb = sub4(xb, u4[hb + 1]); }
      const long long e = ub + 4LL * threadIdx.x + 2048LL * hb;
      if (e >= ue) xa = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e + 2048 >= ue) xb = make_float4(0.f, 0.f, 0.f, 0.f);
      const float xs[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) s2 += (double)xs[j] * (double)xs[j];
      h3_insert_n<8>(xs, inv, tsort, cell, M, K1, dummy, sumA, sumN, cntA, cntN);
    }
  }
  __syncthreads();
  const unsigned long long T2 = ADMMQ_NOW();
  h3_suffix<kH3Threads, 4>(M, sumA, sumN, cntA, cntN, wtot, wtot2, wtot32, wtot32b);
  // per-candidate totals of this block into one of kHistRep replicas
  const int rep = blockIdx.x & (kHistRep - 1);
  unsigned long long* g1 = v.h1 + ((size_t)slot * kHistRep + rep) * (n + 1);
  unsigned long long* g2 = v.h2 + ((size_t)slot * kHistRep + rep) * (n + 1);
  for (int c = threadIdx.x; c < n; c += blockDim.x) {
    unsigned long long t1, t2;
    h3_totals<QMAX>(c, n, rnk, sumA, sumN, cntA, cntN, t1, t2);
    if (t1) atomicAdd(&g1[c], t1);
    if (t2) atomicAdd(&g2[c], t2);
  }
  s2 = wave_sum_f64(s2);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s2;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    atomicAdd(&v.s2[slot], t);
  }
  // ticket: the last block of this job selects the candidate set (all its inputs were
  // written by device-scope atomics: drain them, no L2 writeback needed)
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0)
    last = (__hip_atomic_fetch_add(&v.ticket[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (unsigned)((ck.nblk > 0 ? ck.nblk : v.nhist) - 1)) ? 1 : 0;
  __syncthreads();
  const unsigned long long T3 = ADMMQ_NOW();
  auto trace = [&](unsigned long long T4) {
    if (ADMMQ_TRACE && threadIdx.x == 0 && blockIdx.x < kHistTraceMax) {
      g_hist_trace[blockIdx.x][0] = T0; g_hist_trace[blockIdx.x][1] = T1; g_hist_trace[blockIdx.x][2] = T2;
      g_hist_trace[blockIdx.x][3] = T3; g_hist_trace[blockIdx.x][4] = T4; g_hist_trace[blockIdx.x][5] = 0;
      g_hist_cu[blockIdx.x] = ((unsigned long long)(__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xFF) << 32) |
                              __builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
  };
  if (last) {
    // every byte handed over by the other blocks (h1/h2 replicas, s2) was written by
    // memory-side atomics drained before the ticket and is read below by agent-scope
    // (sc1) atomic loads only, so no L1 invalidate is needed (cdna_hip_programming.md
    // Guideline 16, sc1 consumer); the wavefront fence only keeps the loads after the ticket
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const unsigned long long* G1 = v.h1 + (size_t)slot * kHistRep * (n + 1);
    const unsigned long long* G2 = v.h2 + (size_t)slot * kHistRep * (n + 1);
    // (a one-wave form - lane l summing candidates 4l .. 4l + 3 over the kHistRep replicas
    // itself - made the other blocks' wait for this selection 8.0 -> 16.8 us at C3: 64
    // dependent sc1 loads per lane against 16 per thread here)
    if (n <= (int)blockDim.x) {
      const int c = threadIdx.x;
      unsigned long long t1 = 0ull, t2 = 0ull;
      if (c < n) {
#pragma unroll
        for (int r = 0; r < kHistRep; ++r) {
          t1 += __hip_atomic_load((gu64*)&G1[r * (n + 1) + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          t2 += __hip_atomic_load((gu64*)&G2[r * (n + 1) + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      const double S2 = __hip_atomic_load((__attribute__((address_space(1))) double*)&v.s2[slot], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
      select_block(v, sel, lsel, t1, t2, S2, mx, n, QMAX);
    } else {
      unsigned long long* T1v = sumA;                 // reuse LDS: n each
      unsigned long long* T2v = sumN;
      for (int c = threadIdx.x; c < n; c += blockDim.x) {
        unsigned long long t1 = 0ull, t2 = 0ull;
#pragma unroll
        for (int r = 0; r < kHistRep; ++r) {
          t1 += __hip_atomic_load((gu64*)&G1[r * (n + 1) + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          t2 += __hip_atomic_load((gu64*)&G2[r * (n + 1) + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        T1v[c] = t1; T2v[c] = t2;
      }
      __syncthreads();
      if (threadIdx.x < 64) {
        const double S2 = __hip_atomic_load((__attribute__((address_space(1))) double*)&v.s2[slot], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        select_wave2(v, sel, lsel, T1v, T2v, S2, mx, n, QMAX);
      }
      __syncthreads();
    }
    sse_in_block(v, lsel, n, QMAX == 1 ? 1 : 31 - __builtin_clz(QMAX) + 1, slot, mx, reinterpret_cast<float4*>(smem));
    trace(ADMMQ_NOW());
    if constexpr (FIN) {
      // publish. A single candidate c* (nearly always) travels in the ready word itself,
      // (iter + 1) << 32 | 1 << 31 | c*: the waiting blocks need nothing else, so neither the
      // record's write-through stores nor their drain sit before it (the record keeps the
      // plain stores of select_block for the later launches). Otherwise the record
      // write-through, drained, then the ready word.
      const unsigned long long tag = (unsigned long long)(unsigned)(iter + 1) << 32;
      if (lsel[0] == 1) {
        if (threadIdx.x == 0)
          __hip_atomic_store(v.ready + slot, tag | 0x80000000ull | (unsigned)lsel[2], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      } else {
        const int nrec = 2 + min(lsel[0], kMaxSel);
        for (int j = threadIdx.x; j < nrec; j += blockDim.x)
          __hip_atomic_store(sel + j, lsel[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(v.ready + slot, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else {
    trace(T3);
  }
  if constexpr (FIN) {
    const ProbDesc& p = d[ck.job];
    load_hf();
    if (!last) {   // wait for the job's selection (bounded)
      if (threadIdx.x == 0) {
        unsigned polls = 0;
        int to = 0;
        unsigned long long w;
        while (((w = __hip_atomic_load(v.ready + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) !=
               (unsigned long long)(unsigned)(iter + 1)) {
          __builtin_amdgcn_s_sleep(2);
          if (++polls >= wait_polls) {
            __hip_atomic_store(p.flags + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            to = 1;
            break;
          }
        }
        timed_out = to;
        if (!to && (w & 0x80000000ull)) {   // the single candidate, from the ready word
          lsel[0] = 1;
          lsel[2] = (int)(w & 0x7FFFFFFFull);
        } else {
          lsel[0] = __hip_atomic_load(sel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          lsel[2] = __hip_atomic_load(sel + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      __syncthreads();
      if (timed_out) {   // internal fault: leave the elements unfinalized (the caller re-runs)
        __builtin_amdgcn_s_waitcnt(0);
        return;
      }
    }
    QParams qp;
    if (lsel[0] == 1) {
      qp = qparams_mse(bits, cand_t(mx, lsel[2], n));
    } else {   // |S| > 1: the canonical SSEs decide (written by the last block's atomics)
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      qp = block_qparams(kMse, bits, v, slot, n, 0, 0.f, 0.f);
    }
    __syncthreads();   // the search tables' LDS is reused as rmax
    if (ADMMQ_TRACE && threadIdx.x == 0 && blockIdx.x < kHistTraceMax) g_hist_trace[blockIdx.x][5] = ADMMQ_NOW();
    admm_finalize_block<kH3Threads, 2 * NV, kFinStream>(p, ck.start, total, x4, u4, h4, f4, qp, slot, iter,
                                                  blockIdx.x & (kResRep - 1), reinterpret_cast<unsigned*>(smem),
                                                  ADMMQ_TRACE && blockIdx.x < kHistTraceMax ? g_fin_trace[blockIdx.x] : nullptr);
    if (ADMMQ_TRACE && threadIdx.x == 0 && blockIdx.x < kHistTraceMax) {
      // columns 4, 5: {wait for the selection done, finalize done} (the search ended at 3 / 4)
      const unsigned long long tw = g_hist_trace[blockIdx.x][5];
      g_hist_trace[blockIdx.x][4] = tw;
      g_hist_trace[blockIdx.x][5] = ADMMQ_NOW();
    }
  }
}

// Small ADMM jobs (thin factors, I <= kThinRows: the 9-row spatial mode of a 3x3 conv,
// at most 24 k elements): one 1024-thread block per job runs stage 1 over all of the job's
// elements with the histograms kept in LDS, the candidate selection, stage 2 when
// |S| > 1, and then k_finalize_admm's step for the same elements - no cross-block
// flush, ticket, or separate finalize launch (the three were ~30 us of latency per
// iteration for ~10 k elements). Same integers and the same float32 operations as the
// multi-block path (the histograms are exact sums; S2 only sets the rigorous bounds).
template <int QMAX, int G>   // G: float4 groups per thread (1024 threads x 4 G elements cover the job)
__global__ __launch_bounds__(kSmallThreads) void k_mse_small_admm(const ProbDesc* __restrict__ d, const int* __restrict__ jobs,
                                                         int ncand, int bits, int slot, int iter,
                                                         const unsigned short* __restrict__ rank0,
                                                         const unsigned short* __restrict__ groups, int ngroups) {
  ADMMQ_SMALL_STAMP(0);
  // the job index through a scalar register: the descriptor fields are then scalar loads
  const ProbDesc& p = d[__builtin_amdgcn_readfirstlane(jobs[blockIdx.x])];
  const long long total = (long long)p.I * p.ld;
  // the stop flag and max|x| first (the table setup needs only them), then every element
  // of the job (H_T, U for the search; H, F too for the finalize step), straight-line
  // (past the end a clamped address, zeroed below): the element loads stay in flight
  // through the threshold-table setup
  const int stopped = gld_i32(p.flags);
  const float mx = __uint_as_float(gld_u32(p.mv.stat + 4 * slot));
  H3Pre pre;
  h3_load_order(rank0, QMAX * ncand, groups, ngroups, pre, kSmallThreads);
  asm volatile("" ::: "memory");   // issue order: the loads above before the element loads
  const float *HTp = p.HT, *Up = p.U, *Hp = p.H, *Fpp = p.Fp;
  float4 t4[G], u4[G], h4[G], f4[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const long long e = 4LL * threadIdx.x + 4096LL * g;
    const long long ec = e < total ? e : 0;
    t4[g] = gld4(HTp + ec);
    u4[g] = gld4(Up + ec);
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const long long e = 4LL * threadIdx.x + 4096LL * g;
    const long long ec = e < total ? e : 0;
    h4[g] = gld4(Hp + ec);
    f4[g] = gld4(Fpp + ec);
  }
  const MseView& v = p.mv;
  ADMMQ_SMALL_STAMP(1);
  int* sel = v.sel + (size_t)slot * (2 + kMaxSel);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ unsigned long long wtot[16], wtot2[16];
  __shared__ unsigned wtot32[16], wtot32b[16];
  __shared__ double red[16];
  __shared__ int lsel[2 + kMaxSel];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (int)(blockDim.x >> 6);
  if (!mse_degenerate(mx)) {
    const int n = ncand;
    const int M = QMAX * n;
    const int nb = M + 1 + 64;
    unsigned long long* sumA = reinterpret_cast<unsigned long long*>(smem);
    unsigned long long* sumN = sumA + nb;
    unsigned* cntA = reinterpret_cast<unsigned*>(sumN + nb);
    unsigned* cntN = cntA + nb;
    float* thr = reinterpret_cast<float*>(cntN + nb);
    float* tsort = thr + M;
    unsigned short* rnk = reinterpret_cast<unsigned short*>(tsort + M);
    unsigned short* cell = rnk + ((M + 1) & ~1);
    const float inv = h3_setup<QMAX>(mx, n, pre, groups, ngroups, rank0 + kMaxMerged, sumA, sumN, cntA, cntN, thr,
                                     tsort, rnk, cell, kSmallThreads);
    // the stop test after the (LDS-only) setup: tested earlier, the compiler would sink
    // the element loads below it and their latency would no longer overlap the setup
    if (stopped) return;   // converged earlier (sticky break)
    ADMMQ_SMALL_STAMP(2);
    const int K1 = hist_fixed_exp(mx, v.nelem, QMAX);
    const int dummy = M + 1 + lane;
#pragma unroll
    for (int g = 0; g < G; ++g)   // past the end: zeros (the clamped loads read element 0)
      if (4LL * threadIdx.x + 4096LL * g >= total) { t4[g] = make_float4(0.f, 0.f, 0.f, 0.f); u4[g] = t4[g]; }
    double s2 = 0.0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float xs[4] = {t4[g].x - u4[g].x, t4[g].y - u4[g].y, t4[g].z - u4[g].z, t4[g].w - u4[g].w};   // H_T - U
#pragma unroll
      for (int k = 0; k < 4; ++k) s2 += (double)xs[k] * (double)xs[k];
      h3_insert_n<4>(xs, inv, tsort, cell, M, K1, dummy, sumA, sumN, cntA, cntN);
    }
    __syncthreads();
    ADMMQ_SMALL_STAMP(3);
    h3_suffix<kSmallThreads, 0>(M, sumA, sumN, cntA, cntN, wtot, wtot2, wtot32, wtot32b);
    ADMMQ_SMALL_STAMP(4);
    unsigned long long t1 = 0ull, t2 = 0ull;   // candidate tid (n <= 1024)
    if ((int)threadIdx.x < n) h3_totals<QMAX>(threadIdx.x, n, rnk, sumA, sumN, cntA, cntN, t1, t2);
    s2 = wave_sum_f64(s2);
    if (lane == 0) red[w] = s2;
    __syncthreads();
    double S2 = 0.0;
    for (int k = 0; k < nw; ++k) S2 += red[k];
    select_block(v, sel, lsel, t1, t2, S2, mx, n, QMAX);
    ADMMQ_SMALL_STAMP(5);
    if (ADMMQ_TRACE && threadIdx.x == 0 && blockIdx.x < kSmallTraceMax) g_small_trace[blockIdx.x][8] = (unsigned)lsel[0];
    sse_in_block(v, lsel, n, bits, slot, mx, reinterpret_cast<float4*>(smem));
    __syncthreads();
    ADMMQ_SMALL_STAMP(6);
  }
  if (stopped) return;   // (degenerate max|x|: no setup above)
  // k_finalize_admm's step (source/admm.py:59-65) with the chosen scale: straight from
  // this block's own selection (LDS) when |S| = 1, else from the canonical SSEs its
  // stage 2 wrote (no dependent global reads of the record on the common path)
  const QParams qp = mse_degenerate(mx) ? qparams_mse(bits, __builtin_nanf(""))
                     : (lsel[0] == 1 ? qparams_mse(bits, cand_t(mx, lsel[2], ncand))
                                     : block_qparams(kMse, bits, v, slot, ncand, 0, 0.f, 0.f));
  admm_finalize_block<kSmallThreads, G>(p, 0, total, t4, u4, h4, f4, qp, slot, iter, 0, nullptr);   // thin: no split
  ADMMQ_SMALL_STAMP(7);
}

// maxtotal: the largest I * ld among the jobs (picks G); 0 when the path cannot run
int small_admm_groups(long long maxtotal) {
  const long long g = (maxtotal + 4095) / 4096;
  return g <= 1 ? 1 : (g <= 2 ? 2 : (g <= 3 ? 3 : (g <= 4 ? 4 : (g <= 6 ? 6 : 0))));
}

void launch_mse_small_admm(const ProbDesc* d, const int* jobs, int njobs, int ngr, int ncand, int bits, int slot,
                           int iter, const unsigned short* rank0, const unsigned short* groups, int ngroups,
                           hipStream_t s) {
  if (njobs <= 0) return;
  const size_t lds = hist3_lds_bytes(ncand, bits);
#define ADMMQ_SMG(Q, GG) \
  hipLaunchKernelGGL((k_mse_small_admm<Q, GG>), dim3(njobs), dim3(kSmallThreads), lds, s, d, jobs, ncand, bits, slot, iter, \
                     rank0, groups, ngroups)
#define ADMMQ_SM(Q)                        \
  switch (ngr) {                           \
    case 1: ADMMQ_SMG(Q, 1); break;        \
    case 2: ADMMQ_SMG(Q, 2); break;        \
    case 3: ADMMQ_SMG(Q, 3); break;        \
    case 4: ADMMQ_SMG(Q, 4); break;        \
    default: ADMMQ_SMG(Q, 6); break;       \
  }
  switch (bits) {
    case 1: ADMMQ_SM(1); break;
    case 2: ADMMQ_SM(2); break;
    case 3: ADMMQ_SM(4); break;
    case 4: ADMMQ_SM(8); break;
    default: ADMMQ_SM(16); break;
  }
#undef ADMMQ_SM
#undef ADMMQ_SMG
}

size_t hist3_lds_bytes(int ncand, int bits) {
  const size_t M = (size_t)ncand << (bits - 1);
  const size_t nb = M + 1 + 64;
  const size_t bytes = nb * (8 + 8 + 4 + 4) + M * 8 + (((M + 1) & ~(size_t)1) + kCells + 2) * 2 + (size_t)ncand * 4;
  return std::max((bytes + 15) & ~(size_t)15, (size_t)kSseQuads * 16);
}

size_t hist_lds_bytes(int ncand, int bits) {
  const int qmax = 1 << (bits - 1);
  const size_t nb = (size_t)ncand + 1 + 64;
  const size_t thr = std::max((size_t)qmax * ncand * 4, (size_t)(ncand + 1) * 8);   // also holds H2 sums
  return std::max(nb * 8 + ((nb + 3) & ~(size_t)3) * 4 + thr, (size_t)kSseQuads * 16);   // >= stage-2 tile
}

// Exhaustive / degenerate path only (stage 1 not run): sel = {n, -1} or {1, 0}.
__global__ __launch_bounds__(64) void k_mse_select_all(const ProbDesc* __restrict__ d, const QJob* __restrict__ qj,
                                                       int ncand, int slot) {
  const MseView& v = mview(d, qj, blockIdx.x);
  if (v.done && *v.done) return;
  int* sel = v.sel + (size_t)slot * (2 + kMaxSel);
  const float mx = __uint_as_float(v.stat[4 * slot]);
  if (threadIdx.x == 0) {
    if (mse_degenerate(mx)) { sel[0] = 1; sel[1] = 0; }
    else { sel[0] = ncand; sel[1] = -1; }
  }
}

// Stage 2: canonical SSE of the candidates in S (or all) over 512-quad chunks. Only
// jobs with |S| > 1 have work, so a small grid strides over the chunk list.
__global__ __launch_bounds__(256) void k_mse_sse(const ProbDesc* __restrict__ d, const QJob* __restrict__ qj,
                                                 const Chunk* __restrict__ chunks, int nchunks, int ncand, int bits,
                                                 int slot) {
  __shared__ float4 xs[kSseQuads];
  __shared__ int list[kMaxSel];
  __shared__ int todo[256];
  __shared__ int ntodo;
  // one pass of parallel checks (chunk -> job -> done / |S|): almost always nothing to do
  if (threadIdx.x == 0) ntodo = 0;
  __syncthreads();
  for (int base = blockIdx.x; base < nchunks; base += gridDim.x * (int)blockDim.x) {
    const int ci = base + threadIdx.x * gridDim.x;
    if (ci < nchunks) {
      const Chunk ck = chunks[ci];
      const MseView& v = mview(d, qj, ck.job);
      const bool live = !(v.done && *v.done) && v.sel[(size_t)slot * (2 + kMaxSel)] != 1 &&
                        !mse_degenerate(__uint_as_float(v.stat[4 * slot]));
      if (live) todo[atomicAdd(&ntodo, 1)] = ci;
    }
    __syncthreads();
    for (int w = 0; w < ntodo; ++w) {
      const Chunk ck = chunks[todo[w]];
      const MseView& v = mview(d, qj, ck.job);
      const int* sel = v.sel + (size_t)slot * (2 + kMaxSel);
      const int ns = sel[0];
      const float mx = __uint_as_float(v.stat[4 * slot]);
      const int nqc = min(kSseQuads, v.nq - ck.start);
      for (int t = threadIdx.x; t < nqc; t += blockDim.x) {
        const int qi = ck.start + t;
        const int row = qi / v.qpr;
        const int qc = qi - row * v.qpr;
        xs[t] = load_x4(v.X, v.U, (long long)row * v.ld + 4 * qc);
      }
      const bool all = ns >= ncand;
      if (!all)
        for (int j = threadIdx.x; j < ns; j += blockDim.x) list[j] = sel[2 + j];
      __syncthreads();
      sse_sweep_list(xs, nqc, mx, fixed_exp(mx, v.nq), ncand, bits, all ? nullptr : list, all ? ncand : ns,
                     v.sse + (size_t)slot * ncand);
      __syncthreads();   // xs / list reused by the next chunk
    }
    if (threadIdx.x == 0) ntodo = 0;
    __syncthreads();
  }
}

void launch_mse_hist(const ProbDesc* d, const QJob* q, const Chunk* chunks, int nchunks, int ncand, int bits,
                     int slot, int nv, hipStream_t s) {
  if (nchunks <= 0) return;
  const size_t lds = hist_lds_bytes(ncand, bits);
  const int abl = 0;
#define ADMMQ_H1(Q, V) \
  hipLaunchKernelGGL((k_mse_hist<Q, V>), dim3(nchunks), dim3(1024), lds, s, d, q, chunks, ncand, slot, abl)
#define ADMMQ_H1N(Q) if (nv == 3) ADMMQ_H1(Q, 3); else if (nv == 2) ADMMQ_H1(Q, 2); else ADMMQ_H1(Q, 1)
  switch (bits) {
    case 1: ADMMQ_H1N(1); break;
    case 2: ADMMQ_H1N(2); break;
    case 3: ADMMQ_H1N(4); break;
    case 4: ADMMQ_H1N(8); break;
    case 5: ADMMQ_H1N(16); break;
    default: ADMMQ_H1N(32); break;
  }
#undef ADMMQ_H1N
#undef ADMMQ_H1
}
bool merged_ok(int ncand, int bits) {
  return ncand >= 2 && ((size_t)ncand << (bits - 1)) <= (size_t)kMaxMerged && hist3_lds_bytes(ncand, bits) <= 150 * 1024;
}
void launch_mse_hist3(const ProbDesc* d, const QJob* q, const Chunk* chunks, int nchunks, int ncand, int bits, int slot,
                      const unsigned short* rank0, const unsigned short* groups, int ngroups, int nv, bool fin, int iter,
                      unsigned wait_polls, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  if (nchunks <= 0) return;
  const size_t lds = hist3_lds_bytes(ncand, bits);
  // ev0 / ev1 (profiling, may be null): recorded by the dispatch itself at the kernel's start / end
#define ADMMQ_H3(Q, V, F)                                                                                         \
  hipExtLaunchKernelGGL((k_mse_hist3<Q, V, F>), dim3(nchunks), dim3(kH3Threads), lds, s, ev0, ev1, 0u, d, q, chunks, \
                        ncand, slot, rank0, groups, ngroups, bits, iter, wait_polls)
#define ADMMQ_H3N(Q)                               \
  if (fin) {                                       \
    if (nv == 3) ADMMQ_H3(Q, 3, true);             \
    else if (nv == 2) ADMMQ_H3(Q, 2, true);        \
    else ADMMQ_H3(Q, 1, true);                     \
  } else {                                         \
    if (nv == 3) ADMMQ_H3(Q, 3, false);            \
    else if (nv == 2) ADMMQ_H3(Q, 2, false);       \
    else ADMMQ_H3(Q, 1, false);                    \
  }
  switch (bits) {
    case 1: ADMMQ_H3N(1); break;
    case 2: ADMMQ_H3N(2); break;
    case 3: ADMMQ_H3N(4); break;
    case 4: ADMMQ_H3N(8); break;
    default: ADMMQ_H3N(16); break;
  }
#undef ADMMQ_H3N
#undef ADMMQ_H3
}

// Resident blocks of the fused (FIN) search kernel on the CURRENT device (all of a
// launch's blocks must be resident at once for its in-kernel wait): occupancy x CUs.
// The occupancy API cannot see other work on the device (a kernel of another stream,
// RCCL): a wait that times out because of it is reported as an internal fault and its
// elements are left unfinalized (k_mse_hist3), and the caller re-runs the call with the
// separate finalize launch. (A one-block-per-CU margin would disable the fused form at
// C3: 371 units against 2 x 256 resident blocks, 63 KB of LDS each.) The CU count is
// looked up once per device.
int hist3_fin_capacity(int ncand, int bits, int nv) {
  constexpr int kMaxDev = 64;
  static std::once_flag once[kMaxDev];
  static int cus[kMaxDev];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 0;
  std::call_once(once[dev], [dev]() {
    int n = 0;
    cus[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess ? n : 0;
  });
  const size_t lds = hist3_lds_bytes(ncand, bits);
  int per = 0;
  hipError_t e = hipErrorInvalidValue;
#define ADMMQ_OCC(Q) \
  e = nv == 3   ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_mse_hist3<Q, 3, true>, kH3Threads, lds) \
      : nv == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_mse_hist3<Q, 2, true>, kH3Threads, lds) \
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_mse_hist3<Q, 1, true>, kH3Threads, lds)
  switch (bits) {
    case 1: ADMMQ_OCC(1); break;
    case 2: ADMMQ_OCC(2); break;
    case 3: ADMMQ_OCC(4); break;
    case 4: ADMMQ_OCC(8); break;
    default: ADMMQ_OCC(16); break;
  }
#undef ADMMQ_OCC
  return e == hipSuccess ? per * cus[dev] : 0;
}
void launch_mse_select_all(const ProbDesc* d, const QJob* q, int njobs, int ncand, int slot, hipStream_t s) {
  if (njobs > 0) hipLaunchKernelGGL(k_mse_select_all, dim3(njobs), dim3(64), 0, s, d, q, ncand, slot);
}
void launch_mse_sse(const ProbDesc* d, const QJob* q, const Chunk* chunks, int nchunks, int ncand, int bits,
                    int slot, hipStream_t s) {
  if (nchunks > 0)
    hipLaunchKernelGGL(k_mse_sse, dim3(std::min((nchunks + 255) / 256 * 4, 1024)), dim3(256), 0, s, d, q, chunks, nchunks,
                       ncand, bits, slot);
}

}  // namespace admmq

// The thin factors (I <= kThinRows: the 9-row spatial mode of a 3x3 conv): their solve
// in one canonical summation order, per iteration (k_thin_solve) or inside a persistent
// launch that runs every iteration of a call (k_thin_loop; source/admm.py:55-65).
//
// Solve H_T = P M (I x ld times ld x ld, M symmetric). A workgroup owns 32 columns and
// the whole reduction: thread (cg, kp) (cg = lane >> 3 the float4 column group, kp =
// 8 wave + (lane & 7) one of 64 k classes) holds M[k][4 cg .. 4 cg + 3] in registers for
// the k pairs (2q, 2q + 1) with q = kp (mod 64), ascending: its 9 k pairs cover ld <= 1152.
// P (NR x ld) is staged in LDS; each class is an ascending packed-FMA chain, the eight
// classes of a wave are summed by the DPP tree ((c0+c1)+(c2+c3))+((c4+c5)+(c6+c7)) and the
// eight waves in order through LDS. Every path that solves a thin factor uses this
// order, so a factor's bits never depend on its batch or on which path ran.
//
// k_thin_loop: each job is a team of ld / 32 workgroups, one per CU, and workgroup r keeps
// its M columns and H, U, F of those columns in registers for the whole loop (the
// launch-per-phase path re-streams every M from HBM / MALL each iteration and spends
// ~38 us per iteration on launch-bound kernels at C3). An iteration:
//   solve     as above, P staged with sc1 loads (the whole team wrote it);
//   max|X|    X = H_T - U; team max by an agent-scope atomicMax -> barrier 1;
//   stage 1   the search's level sums over the workgroup's elements (hist_insert_elem:
//             the same integers as every other stage 1), flushed into the team's bins by
//             64-bit atomic adds (integers: order-free), sum X^2 likewise -> barrier 2;
//   select    every workgroup computes the same rigorous candidate set S from the team
//             totals (SelCtx); |S| = 1 (nearly always) gives c* at once, otherwise the
//             canonical SSE of S over the team (atomic adds) -> barrier 2b -> first-index
//             argmin: the reference's 200-candidate sweep's answer either way;
//   finalize  k_finalize_admm's float32 operations on the owned elements (registers),
//             the next P with 16-B sc1 stores, the residual sums by atomic adds ->
//             barrier 3; the next iteration starts with the stop test on those sums
//             (source/admm.py:62-65), uniform over the team.
// Hand-offs (MI355X_MICROARCH.md, inter-workgroup visibility, first table row): every
// handed-off byte is a 16-B sc1 store or an agent-scope atomic; every storing thread
// waits vmcnt(0) before the workgroup barrier behind which one lane arrives on the team's
// counter (agent atomic add); the polling lane uses sc1 loads and the other waves read
// after a workgroup barrier it joins; all those reads are sc1 (global / buffer) loads or
// agent atomic loads. One workgroup per CU, every workgroup of the grid resident (the
// host checks grid <= CUs and the occupancy). A barrier wait is bounded: past it the
// workgroup sets flags[3] (internal fault) and leaves the loop; the caller re-runs the
// call without the fused paths (the PyTorch op does).
#include "search_device.h"

namespace admmq {

typedef float f2v __attribute__((ext_vector_type(2)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned long long gu64t;
typedef __attribute__((address_space(1))) double gf64t;
typedef __attribute__((address_space(1))) unsigned gu32t;
typedef __attribute__((address_space(1))) gf32x4 gst4t;

constexpr int kTSCols = 32;   // columns of a solve workgroup

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// sum over lane bits 0..2: xor 1, xor 2 (quad_perm), then the mirrored half-row, which is
// the xor-4 partner once each quad holds one value; every lane of the 8 gets the same
// value (a + b == b + a), so the result does not depend on the lane
__device__ __forceinline__ float lane8_sum(float v) {
  v += dppf<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dppf<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dppf<0x141>(v);   // row_half_mirror
  return v;
}

__device__ __forceinline__ unsigned long long ald_u64(unsigned long long* q) {
  return __hip_atomic_load((gu64t*)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ald_f64(double* q) {
  return __hip_atomic_load((gf64t*)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast_u64(unsigned long long* q, unsigned long long v) {
  __hip_atomic_store((gu64t*)q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast_f64(double* q, double v) {
  __hip_atomic_store((gf64t*)q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// The solve, shared by both kernels (all 512 threads call each step)
struct ThinM {
  f2v xy[kTLKPairs][2], zw[kTLKPairs][2];   // [pair][k parity] columns (x, y) and (z, w)
};
struct ThinGeo {
  int kpa, kpb, cg, kpl, JN, LDP, kc0, cw;
};
// Reduction chunk [kc0, kc0 + 1152) of ld (factors with ld > 1152 take several: each class
// chain continues across them in ascending k, so the order is the same as one long chain)
constexpr int kTSChunk = 128 * kTLKPairs;
// cw = 32: thread (cg = lane >> 3, class kpa = 8 wave + (lane & 7)), k pair slots 0..8.
// cw = 64 (persistent loop only, ld <= 512): thread (cg = lane >> 2, classes kpa = 8 wave +
// (lane & 3) in slots 0..3 and kpb = kpa + 4 in slots 4..7): the same chains, the same tree.
__device__ __forceinline__ ThinGeo thin_geo(int ld, int kc0, int cw = kTSCols) {
  ThinGeo g;
  const int lane = threadIdx.x & 63;
  const bool w64 = cw == 64;
  g.cw = cw;
  g.kpl = w64 ? (lane & 3) : (lane & 7);
  g.cg = w64 ? (lane >> 2) : (lane >> 3);
  g.kpa = 8 * (threadIdx.x >> 6) + g.kpl;
  g.kpb = g.kpa + 4;
  g.kc0 = kc0;
  g.JN = (min(ld - kc0, kTSChunk) + 127) >> 7;   // k pairs per class in this chunk (<= kTLKPairs)
  g.LDP = 128 * g.JN;                               // staged row length of P (zero tail)
  return g;
}
// M[k][col0 + 4 cg ..] for this thread's k of the chunk (plain loads: M is written by the
// prepare launches)
__device__ __forceinline__ void thin_load_m(const ProbDesc& p, int col0, const ThinGeo& g, ThinM& m) {
  const int ld = p.ld, ldm = p.ldm, cth = col0 + 4 * g.cg;
  const bool w64 = g.cw == 64;
#pragma unroll
  for (int j = 0; j < kTLKPairs; ++j)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int cls = (w64 && j >= 4) ? g.kpb : g.kpa;
      const int jj = (w64 && j >= 4) ? j - 4 : j;
      const int k = g.kc0 + 2 * (cls + 64 * jj) + e;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (jj < g.JN && k < ld && !(w64 && j >= 8)) v = gld4(p.M + (size_t)k * ldm + cth);
      m.xy[j][e] = f2v{v.x, v.y};
      m.zw[j][e] = f2v{v.z, v.w};
    }
}
// P rows [0, NR) into Ps[NR][kTSChunk] (row stride fixed so every LDS read of the FMA
// sweep is one base register plus an immediate offset; columns [0, LDP), zero past ld)
// with 16-B sc1 buffer loads: all loads first (thin_load_p), then the LDS stores
// (thin_store_p). Rows I..NR-1 of the padded P are 0.
template <int NR>
struct ThinP {
  static constexpr int kV4 = (NR * kTSChunk / 4 + kTLThreads - 1) / kTLThreads;
  float4 v[kV4];
};
template <int NR>
__device__ __forceinline__ void thin_load_p(const ProbDesc& p, const ThinGeo& g, ThinP<NR>& pv) {
  const int ld = p.ld, q4 = g.LDP >> 2, nv4 = NR * q4;
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc(p.P, 0, (int)((size_t)p.Ip * ld * sizeof(float)), 0x00020000);
#pragma unroll
  for (int r = 0; r < ThinP<NR>::kV4; ++r) {
    const int v = threadIdx.x + r * kTLThreads;
    const int i = v / q4, k4 = g.kc0 + 4 * (v - i * q4);
    pv.v[r] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (v < nv4 && k4 < ld) {
      const u32x4v w = __builtin_amdgcn_raw_buffer_load_b128(prs, (int)(((size_t)i * ld + k4) * 4), 0, 16);   // sc1
      pv.v[r] = make_float4(__uint_as_float(w.x), __uint_as_float(w.y), __uint_as_float(w.z), __uint_as_float(w.w));
    }
  }
}
template <int NR>
__device__ __forceinline__ void thin_store_p(const ThinGeo& g, const ThinP<NR>& pv, float* Ps) {
  const int q4 = g.LDP >> 2, nv4 = NR * q4;
#pragma unroll
  for (int r = 0; r < ThinP<NR>::kV4; ++r) {
    const int v = threadIdx.x + r * kTLThreads;
    if (v < nv4) {
      const int i = v / q4, k4 = 4 * (v - i * q4);
      *reinterpret_cast<float4*>(Ps + i * kTSChunk + k4) = pv.v[r];
    }
  }
}
template <int NR>
__device__ __forceinline__ void thin_stage_p(const ProbDesc& p, const ThinGeo& g, float* Ps) {
  ThinP<NR> pv;
  thin_load_p<NR>(p, g, pv);
  thin_store_p<NR>(g, pv, Ps);
}
// One chunk of the canonical class chains of class `cls` in M slots [LO, HI): acc[i] +=
// P[i][k] M[k][cols] over the class's k pairs, ascending (Ps staged and visible).
template <int NR, int LO, int HI>
__device__ __forceinline__ void thin_accumulate(const float* Ps, const ThinGeo& g, const ThinM& m, int cls,
                                                f2v (&acc)[NR][2]) {
  const float* pr0 = Ps + 2 * cls;
#pragma unroll
  for (int j = LO; j < HI; ++j) {
    if (j - LO < g.JN) {
      const float* pr = pr0 + 128 * (j - LO);
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const float2 pp = *reinterpret_cast<const float2*>(pr + i * kTSChunk);   // immediate offsets
        const f2v a = {pp.x, pp.x}, b = {pp.y, pp.y};
        acc[i][0] = __builtin_elementwise_fma(m.xy[j][0], a, acc[i][0]);
        acc[i][1] = __builtin_elementwise_fma(m.zw[j][0], a, acc[i][1]);
        acc[i][0] = __builtin_elementwise_fma(m.xy[j][1], b, acc[i][0]);
        acc[i][1] = __builtin_elementwise_fma(m.zw[j][1], b, acc[i][1]);
      }
    }
  }
}
template <int NR>
__device__ __forceinline__ void thin_zero(f2v (&acc)[NR][2]) {
#pragma unroll
  for (int i = 0; i < NR; ++i) acc[i][0] = acc[i][1] = f2v{0.f, 0.f};
}
// DPP sums of the class chains over lane bits 0..1 (quad) or 0..2 (8 lanes)
template <int NR>
__device__ __forceinline__ void thin_lane_sums(f2v (&acc)[NR][2], bool eight) {
#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float x = acc[i][h].x, y = acc[i][h].y;
      x += dppf<0xB1>(x); y += dppf<0xB1>(y);   // quad_perm [1,0,3,2]
      x += dppf<0x4E>(x); y += dppf<0x4E>(y);   // quad_perm [2,3,0,1]
      if (eight) { x += dppf<0x141>(x); y += dppf<0x141>(y); }   // row_half_mirror
      acc[i][h] = f2v{x, y};
    }
}
// The workgroup's class chains (one chunk already accumulated for cw = 32; both classes
// computed here for cw = 64) -> H_T of its cw columns: the DPP tree
// ((c0+c1)+(c2+c3))+((c4+c5)+(c6+c7)) in each wave (for cw = 64 the two quad trees are
// added in that order through `stash`, LDS of 8 x NR x 64 floats not aliasing Ps), then
// the 8 waves in order through `red`, which may alias the staged P (the first barrier
// keeps every wave's reads of it before the partial stores). Returns the quad (row
// tid / (cw/4), columns 4 (tid % (cw/4)) ..) to threads tid < NR cw / 4, zeros elsewhere.
template <int NR>
__device__ __forceinline__ float4 thin_reduce(f2v (&acc)[NR][2], float* red, const ThinGeo& g) {
  thin_lane_sums<NR>(acc, true);
  __syncthreads();
  const int wave = threadIdx.x >> 6, cw = g.cw, qpr = cw >> 2;
  if (g.kpl == 0) {
#pragma unroll
    for (int i = 0; i < NR; ++i)
      *reinterpret_cast<float4*>(red + (wave * NR + i) * cw + 4 * g.cg) =
          make_float4(acc[i][0].x, acc[i][0].y, acc[i][1].x, acc[i][1].y);
  }
  __syncthreads();
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if ((int)threadIdx.x < NR * qpr) {
    const int qi = threadIdx.x / qpr, qq = threadIdx.x - qi * qpr;
    t = *reinterpret_cast<const float4*>(red + qi * cw + 4 * qq);
#pragma unroll
    for (int w = 1; w < kTLThreads / 64; ++w) {
      const float4 b = *reinterpret_cast<const float4*>(red + (w * NR + qi) * cw + 4 * qq);
      t.x += b.x; t.y += b.y; t.z += b.z; t.w += b.w;
    }
  }
  return t;
}
// cw = 64: both classes of this thread (one chunk, ld <= 512), then the same reduction
template <int NR>
__device__ __forceinline__ float4 thin_solve64(const float* Ps, float* red, float* stash, const ThinGeo& g,
                                               const ThinM& m) {
  f2v acc[NR][2];
  thin_zero<NR>(acc);
  thin_accumulate<NR, 0, 4>(Ps, g, m, g.kpa, acc);
  thin_lane_sums<NR>(acc, false);
  const int wave = threadIdx.x >> 6;
  if (g.kpl == 0) {
#pragma unroll
    for (int i = 0; i < NR; ++i)
      *reinterpret_cast<float4*>(stash + (wave * NR + i) * 64 + 4 * g.cg) =
          make_float4(acc[i][0].x, acc[i][0].y, acc[i][1].x, acc[i][1].y);
  }
  thin_zero<NR>(acc);
  thin_accumulate<NR, 4, 8>(Ps, g, m, g.kpb, acc);
  thin_lane_sums<NR>(acc, false);
  if (g.kpl == 0) {   // T4(c0..c3) + T4(c4..c7): the 8-lane tree's last step (same lane's stash)
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const float4 a = *reinterpret_cast<const float4*>(stash + (wave * NR + i) * 64 + 4 * g.cg);
      acc[i][0] = f2v{a.x + acc[i][0].x, a.y + acc[i][0].y};
      acc[i][1] = f2v{a.z + acc[i][1].x, a.w + acc[i][1].y};
    }
  }
  __syncthreads();
  const int cw = 64, qpr = 16;
  if (g.kpl == 0) {
#pragma unroll
    for (int i = 0; i < NR; ++i)
      *reinterpret_cast<float4*>(red + (wave * NR + i) * cw + 4 * g.cg) =
          make_float4(acc[i][0].x, acc[i][0].y, acc[i][1].x, acc[i][1].y);
  }
  __syncthreads();
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if ((int)threadIdx.x < NR * qpr) {
    const int qi = threadIdx.x / qpr, qq = threadIdx.x - qi * qpr;
    t = *reinterpret_cast<const float4*>(red + qi * cw + 4 * qq);
#pragma unroll
    for (int w = 1; w < kTLThreads / 64; ++w) {
      const float4 b = *reinterpret_cast<const float4*>(red + (w * NR + qi) * cw + 4 * qq);
      t.x += b.x; t.y += b.y; t.z += b.z; t.w += b.w;
    }
  }
  return t;
}
// floats of region A (P staging, then the partials) for a launch whose largest ld is maxld
inline int thin_region_a(int nr, int maxld) {
  (void)maxld;
  return std::max(nr * kTSChunk, 8 * nr * 64);
}

// ---------------------------------------------------------------------------
// Per-iteration solve of the thin factors: one workgroup per 32 columns. Also the stop
// test (source/admm.py:59-65) and the quantizer statistics of X = H_T - U for the search
// launch (k_mse_small_admm or the generic search); the first workgroup of a problem
// zeroes that iteration's search accumulators.
template <int NR>
__global__ __launch_bounds__(kTLThreads) void k_thin_solve(const ProbDesc* __restrict__ probs,
                                                           const ThinLoopUnit* __restrict__ units, int slot, int iter,
                                                           float eps, int ncand) {
  extern __shared__ __attribute__((aligned(16))) float smemf[];
  const ThinLoopUnit u = units[blockIdx.x];
  const ProbDesc& p = probs[__builtin_amdgcn_readfirstlane(u.job)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int ld = p.ld, I = p.I, R = p.R, col0 = u.col0;
  ThinGeo g = thin_geo(ld, 0);
  const int done = gld_i32(p.flags);
  // residual replicas of the previous iteration: lane l < 32 of every wave holds entry l of [kResRep][4]
  const double rv = (iter > 0 && lane < 4 * kResRep)
                        ? *(__attribute__((address_space(1))) const double*)(p.res + 4 * kResRep * (slot ^ 1) + lane)
                        : 0.0;
  const int qi = tid >> 3, qq = tid & 7;
  const bool owner = tid < NR * 8 && qi < I;
  const int qcol = col0 + 4 * qq, qoff = qi * ld + qcol;
  float4 u4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (owner) u4 = gld4(p.U + qoff);
  ThinM m;
  thin_load_m(p, col0, g, m);
  if (done) return;
  if (iter > 0) {   // stop test, uniform over the problem's workgroups
    double t = rv;
    t += __shfl_xor(t, 4); t += __shfl_xor(t, 8); t += __shfl_xor(t, 16);   // lanes k = 0..3: sum k
    const double t0 = __shfl(t, 0), t1 = __shfl(t, 1), t2 = __shfl(t, 2), t3 = __shfl(t, 3);
    if (t0 / t1 < (double)eps && t2 / t3 < (double)eps) {
      if (col0 == 0 && tid == 0) p.flags[0] = 1;   // sticky "break"
      return;
    }
  }
  f2v acc[NR][2];
  thin_zero<NR>(acc);
  for (;;) {
    thin_stage_p<NR>(p, g, smemf);
    __syncthreads();
    thin_accumulate<NR, 0, kTLKPairs>(smemf, g, m, g.kpa, acc);
    if (g.kc0 + kTSChunk >= ld) break;
    __syncthreads();   // the next chunk's staging overwrites smemf
    g = thin_geo(ld, g.kc0 + kTSChunk);
    thin_load_m(p, col0, g, m);
  }
  const float4 t4 = thin_reduce<NR>(acc, smemf, g);
  if (col0 == 0) {   // this iteration's quantizer-search accumulators start at zero
    gu64t* sse = (gu64t*)(p.mv.sse + (size_t)slot * ncand);
    gu64t* h1 = (gu64t*)(p.mv.h1 + (size_t)slot * kHistRep * (ncand + 1));
    gu64t* h2 = (gu64t*)(p.mv.h2 + (size_t)slot * kHistRep * (ncand + 1));
    for (int c = tid; c < ncand; c += kTLThreads) sse[c] = 0ull;
    for (int c = tid; c < kHistRep * (ncand + 1); c += kTLThreads) { h1[c] = 0ull; h2[c] = 0ull; }
    if (tid == 0) {
      *(gf64t*)(p.mv.s2 + slot) = 0.0;
      *(gu32t*)(p.mv.ticket + slot) = 0u;
    }
  }
  // H_T, X = H_T - U (debug) and the statistics of the valid region
  unsigned amax = 0u, mn = 0xFFFFFFFFu, mxo = 0u;
  if (owner) {
    const float4 x4 = sub4(t4, u4);
    const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (qcol + c < R) {
        amax = max(amax, __float_as_uint(xs[c]) & 0x7FFFFFFFu);
        const unsigned e = enc_ord(xs[c]);
        mn = min(mn, e);
        mxo = max(mxo, e);
      }
    *(gst4t*)(p.HT + qoff) = gf32x4{t4.x, t4.y, t4.z, t4.w};
    if (p.X_dbg) *(gst4t*)(p.X + qoff) = gf32x4{x4.x, x4.y, x4.z, x4.w};
  }
  if (tid < 64 * ((NR * 8 + 63) / 64)) {   // the owners' waves
    amax = wave_max_u32(amax); mn = wave_min_u32(mn); mxo = wave_max_u32(mxo);
    if (lane == 0) {
      unsigned* st = p.mv.stat + 4 * slot;
      atomicMax(&st[0], amax);
      atomicMin(&st[1], mn);
      atomicMax(&st[2], mxo);
    }
  }
}

void launch_thin_solve(const ProbDesc* d, const ThinLoopUnit* units, int nunits, int nr, int maxld, int slot, int iter,
                       float eps, int ncand, hipStream_t s) {
  if (nunits <= 0) return;
  const size_t lds = (size_t)thin_region_a(nr <= 9 ? 9 : 16, maxld) * sizeof(float);
  if (nr <= 9)
    hipLaunchKernelGGL(k_thin_solve<9>, dim3(nunits), dim3(kTLThreads), lds, s, d, units, slot, iter, eps, ncand);
  else
    hipLaunchKernelGGL(k_thin_solve<16>, dim3(nunits), dim3(kTLThreads), lds, s, d, units, slot, iter, eps, ncand);
}

// ---------------------------------------------------------------------------
// Persistent loop

// Diagnostics (make TRACE=1; admmq_debug_thin_loop_trace): per workgroup, the summed
// s_memrealtime ticks (10 ns) of each phase over the loop's iterations: {P staging, solve,
// X and max, barrier 1 + max load, threshold table, stage-1 inserts, stage-1 sums + flush,
// barrier 2, team bins load, suffix sums + bounds + S, stage 2, finalize, barrier 3, slot
// reset, stop test, iterations}
// Diagnostics (admmq_debug_set_sel_widen): every candidate stays in S (stage 2 every
// iteration; the same exact answer)
__device__ int g_sel_widen_tl = 0;
int set_sel_widen_thin(int on) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_sel_widen_tl), &on, sizeof(int)) == hipSuccess ? 0 : -1;
}
constexpr int kTLTraceMax = 1024;
constexpr int kTLPhases = 16;
__device__ unsigned long long g_tl_trace[kTLTraceMax][kTLPhases];
int copy_thin_loop_trace(unsigned long long* host, int n) {
  n = n < kTLTraceMax ? n : kTLTraceMax;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tl_trace), (size_t)n * kTLPhases * sizeof(unsigned long long)) ==
                 hipSuccess
             ? n
             : -1;
}

// Team barrier number `target / nteam`: this thread's stores and atomics drained, the
// workgroup joined, one lane arrives and polls (sc1 loads, s_sleep), the workgroup joins
// again. false: the wait passed `polls` (the caller reports an internal fault). (Polling
// from every wave's lane 0 with staggered starts was slower: 1.7 -> 2.1 us per barrier.)
__device__ __forceinline__ bool team_barrier(unsigned* bar, unsigned target, unsigned polls, int* s_ok) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    unsigned n = 0;
    while (__hip_atomic_load((gu32t*)bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++n > polls) { ok = 0; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

// Dynamic LDS of k_thin_loop: region A (thin_region_a floats), the threshold table
// [qmax][n], the block's stage-1 bins (n + 1, then 64 private dummies) and the team's h2
// totals (n + 1, u64).
__host__ __device__ inline size_t tl_off_h1(int region_a, int qmax, int n) {
  return ((size_t)region_a * 4 + (size_t)qmax * n * 4 + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t tl_off_h2(int region_a, int qmax, int n) {
  return tl_off_h1(region_a, qmax, n) + (size_t)(n + 65) * 8;
}
__host__ __device__ inline size_t tl_off_H2(int region_a, int qmax, int n) {
  return (tl_off_h2(region_a, qmax, n) + (size_t)(n + 65) * 4 + 15) & ~(size_t)15;
}
size_t thin_loop_lds_bytes(int region_a, int ncand, int bits) {
  return tl_off_H2(region_a, 1 << (bits - 1), ncand) + (size_t)(ncand + 1) * 8;
}

template <int NR, int QMAX>
__global__ __launch_bounds__(kTLThreads) void k_thin_loop(const ProbDesc* __restrict__ d,
                                                          const ThinLoopUnit* __restrict__ units,
                                                          ThinSync* __restrict__ syncs, int region_a, int n_iter,
                                                          float eps, int ncand, int bits, unsigned wait_polls) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ unsigned s_amax[kTLThreads / 64];
  __shared__ double s_red[kTLThreads / 64][4];
  __shared__ unsigned long long s_part[kTLBins];
  __shared__ int s_wcnt[kTLThreads / 64];
  __shared__ int lsel[2 + kMaxSel];
  __shared__ unsigned long long s_best[kTLThreads / 64];
  __shared__ int s_bidx[kTLThreads / 64];
  __shared__ double s_res[4];
  __shared__ unsigned long long s_mx;
  __shared__ int s_ok;
  __shared__ int s_cstar;
  __shared__ __attribute__((aligned(16))) float s_x[NR * 64];   // the workgroup's X (rows < NR, cw columns)
  __shared__ float s_sc[kTLMaxCand];   // this iteration's candidate scales s_c = fl(2 t_c / den)

  const ThinLoopUnit un = units[blockIdx.x];
  const int job = __builtin_amdgcn_readfirstlane(un.job);
  const ProbDesc& p = d[job];
  ThinSync& sy = syncs[job];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ld = p.ld, I = p.I, R = p.R;
  const int col0 = un.col0, nteam = un.nteam, cw = un.cw, qpr = cw >> 2;
  const bool leader = un.rank == 0;
  const float rho = p.rho[0];
  const int n = ncand;
  const ThinGeo g = thin_geo(ld, 0, cw);   // ld <= 1152 (cw = 64: ld <= 512): one chunk (the host checks)
  float* const Ps = reinterpret_cast<float*>(smem);
  float* const stash = Ps + NR * kTSChunk;   // cw = 64: the first class's quad trees
  float* const thr = reinterpret_cast<float*>(smem + (size_t)region_a * 4);
  unsigned long long* const h1 = reinterpret_cast<unsigned long long*>(smem + tl_off_h1(region_a, QMAX, n));
  unsigned* const h2 = reinterpret_cast<unsigned*>(smem + tl_off_h2(region_a, QMAX, n));

  ThinM m;
  thin_load_m(p, col0, g, m);
  // owned quad: row qi, columns col0 + 4 qq .. + 3 (rows >= I are never owned)
  const int qi = tid / qpr, qq = tid - qi * qpr;
  const bool owner = tid < NR * qpr && qi < I;
  const int qcol = col0 + 4 * qq, qoff = qi * ld + qcol;
  float4 h4 = make_float4(0.f, 0.f, 0.f, 0.f), u4 = h4, f4 = h4;
  if (owner) { h4 = gld4(p.H + qoff); u4 = gld4(p.U + qoff); f4 = gld4(p.Fp + qoff); }
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc(p.P, 0, (int)((size_t)p.Ip * ld * sizeof(float)), 0x00020000);

  const bool widen = *(volatile int*)&g_sel_widen_tl != 0;
  unsigned nbar = 0;
  bool fault = false;
  unsigned long long ph[kTLPhases] = {}, tph = ADMMQ_NOW();
#define ADMMQ_TL_PH(k)                                   \
  if (ADMMQ_TRACE) {                                     \
    const unsigned long long tn_ = ADMMQ_NOW();          \
    ph[k] += tn_ - tph;                                  \
    tph = tn_;                                           \
  }
  for (int it = 0; it < n_iter; ++it) {
    const int slot = it & 1;
    if (ADMMQ_TRACE) ph[15] += 1;
    // the next P's loads, then the stop test's residual sums (previous iteration, team
    // totals): the test is decided after the solve, so the load's latency hides behind it;
    // nothing of this iteration is stored before the test
    ThinP<NR> pv;
    thin_load_p<NR>(p, g, pv);
    const double rsum = (it > 0 && tid < 4) ? ald_f64(&sy.res[slot ^ 1][tid]) : 0.0;
    // ---- solve
    thin_store_p<NR>(g, pv, Ps);
    __syncthreads();
    ADMMQ_TL_PH(0);
    float4 t4;
    if (cw == 64) {
      t4 = thin_solve64<NR>(Ps, Ps, stash, g, m);
    } else {
      f2v acc[NR][2];
      thin_zero<NR>(acc);
      thin_accumulate<NR, 0, kTLKPairs>(Ps, g, m, g.kpa, acc);
      t4 = thin_reduce<NR>(acc, Ps, g);
    }
    ADMMQ_TL_PH(1);
    if (it > 0) {   // stop test on the previous iteration's team sums (source/admm.py:62-65)
      if (tid < 4) s_res[tid] = rsum;
      __syncthreads();
      const double t0 = s_res[0], t1 = s_res[1], t2 = s_res[2], t3 = s_res[3];
      if (t0 / t1 < (double)eps && t2 / t3 < (double)eps) {
        if (leader && tid == 0) p.flags[0] = 1;   // sticky "break"
        break;
      }
    }
    ADMMQ_TL_PH(14);
    float4 x4 = make_float4(0.f, 0.f, 0.f, 0.f);
    unsigned amax = 0u;
    if (owner) {
      x4 = sub4(t4, u4);   // H_T - U
      const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (qcol + c < R) amax = max(amax, __float_as_uint(xs[c]) & 0x7FFFFFFFu);
      *(gst4t*)(p.HT + qoff) = gf32x4{t4.x, t4.y, t4.z, t4.w};   // read after the launch only
      if (p.X_dbg) *(gst4t*)(p.X + qoff) = gf32x4{x4.x, x4.y, x4.z, x4.w};
    }
    if (tid < NR * qpr) *reinterpret_cast<float4*>(s_x + 4 * tid) = x4;   // rows >= I: 0
    amax = wave_max_u32(amax);
    if (lane == 0) s_amax[wave] = amax;
    __syncthreads();
    // ---- barrier 1: the team's max |X|. The arrival IS the hand-off: each workgroup
    // stores (it + 1) << 32 | its max into its own word (agent scope, one lane); wave 0
    // polls the team's words, lane l word l, until every tag is this iteration's, and
    // takes their max - no counter, no drain of other stores (nothing else is handed over
    // here), no second load after the wait. The words are zeroed by the host per launch
    // and tagged per iteration, so they are never reset.
    const unsigned long long tag = (unsigned long long)(unsigned)(it + 1) << 32;
    if (tid == 0) {
      unsigned mm = 0u;
#pragma unroll
      for (int w = 0; w < kTLThreads / 64; ++w) mm = max(mm, s_amax[w]);
      ast_u64(&sy.arr1[un.rank], tag | mm);
    }
    ADMMQ_TL_PH(2);
    if (wave == 0) {
      unsigned long long w = tag;
      int ok = 1;
      if (lane < nteam) {
        unsigned n = 0;
        while (((w = ald_u64(&sy.arr1[lane])) & ~0xFFFFFFFFull) != tag) {
          if (++n > wait_polls) { ok = 0; break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      const unsigned m = wave_max_u32((unsigned)w);
      const bool all_ok = __ballot(!ok) == 0ull;
      if (lane == 0) { s_mx = m; s_ok = all_ok ? 1 : 0; }
    }
    __syncthreads();
    if (!s_ok) { fault = true; break; }
    ADMMQ_TL_PH(3);
    const float mx = __uint_as_float((unsigned)s_mx);
    QParams qp;
    if (mse_degenerate(mx)) {
      qp = qparams_mse(bits, __builtin_nanf(""));
    } else {
      // ---- stage 1 over the workgroup's elements, one per thread
      {   // thr[k-1][c] = fill_thresholds' values; thread (c, half of the levels): s_c computed once
        constexpr int KH = (QMAX + 1) / 2;
        const float den = (float)(2 * QMAX - 1);
        for (int e = tid; e < 2 * n; e += kTLThreads) {
          const int c = e >> 1, k0 = 1 + (e & 1) * KH;
          const float sc = (2.0f * cand_t(mx, c, n)) / den;
          if (!(e & 1)) s_sc[c] = sc;
#pragma unroll
          for (int k = k0; k < k0 + KH; ++k)
            if (k <= QMAX) thr[(k - 1) * n + c] = level_threshold_fast(sc, k);
        }
      }
      for (int b = tid; b < n + 65; b += kTLThreads) { h1[b] = 0ull; h2[b] = 0u; }
      __syncthreads();
      ADMMQ_TL_PH(4);
      const float S0 = (float)(0.2 * (double)mx);
      const float E0 = (float)(1.2 * (double)mx);
      const float inv_step = (float)(n - 1) / (E0 - S0);
      const int K1 = hist_fixed_exp(mx, p.mv.nelem, QMAX);
      double s2 = 0.0;
      unsigned long long full1 = 0ull;
      unsigned full2 = 0u;
      {
        float tlo0[QMAX], thin[QMAX];
#pragma unroll
        for (int k = 0; k < QMAX; ++k) { tlo0[k] = thr[k * n]; thin[k] = thr[k * n + n - 1]; }
        const int ne = min(I, NR) * cw;   // rows >= I and columns >= R hold 0: they add nothing
        for (int e = tid; e < ne; e += kTLThreads)   // cw = 64: up to 1024 elements
          hist_insert_elem<QMAX>(s_x[e], thr, n, S0, inv_step, K1, n + 1 + lane, tlo0, thin, h1, h2, s2, full1,
                                 full2);
      }
      ADMMQ_TL_PH(5);
      s2 = wave_sum_f64(s2);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        full1 += __shfl_xor(full1, off);
        full2 += (unsigned)__shfl_xor((int)full2, off);
      }
      if (lane == 0) {
        s_red[wave][0] = s2;
        if (full1) atomicAdd(&h1[n], full1);
        if (full2) atomicAdd(&h2[n], full2);
      }
      __syncthreads();
      for (int b = tid; b <= n; b += kTLThreads) {
        if (h1[b]) atomicAdd(&sy.h1[slot][b], h1[b]);
        if (h2[b]) atomicAdd(&sy.h2[slot][b], (unsigned long long)h2[b]);
      }
      if (tid == 0) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < kTLThreads / 64; ++w) t += s_red[w][0];
        if (t != 0.0) atomicAdd(&sy.s2[slot], t);
      }
      // ---- barrier 2: the team's stage-1 totals
      ADMMQ_TL_PH(6);
      if (!team_barrier(&sy.bar, nteam * ++nbar, wait_polls, &s_ok)) { fault = true; break; }
      ADMMQ_TL_PH(7);
      // ---- the selection by ONE wave (no block barrier inside): lane l owns candidates
      // 4l .. 4l + 3 (n <= kTLMaxCand = 256) and reads their team totals straight from the
      // team's bins; T(c) = sum_{b > c} H[b] = the lane's own suffix over its four c plus
      // the wave suffix of the later lanes' totals; the rigorous bounds of each c, min(A + E)
      // over the wave, and the ascending list S = {c : A - E <= min} (the same integers and
      // fp64 operations per candidate as the block form, so the same S)
      if (wave == 0) {
        const double S2 = ald_f64(&sy.s2[slot]);
        unsigned long long a1[4], a2[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = 4 * lane + j;
          a1[j] = c < n ? ald_u64(&sy.h1[slot][c + 1]) : 0ull;
          a2[j] = c < n ? ald_u64(&sy.h2[slot][c + 1]) : 0ull;
        }
        ADMMQ_TL_PH(8);
        unsigned long long l1[4], l2[4], r1 = 0ull, r2 = 0ull;
#pragma unroll
        for (int j = 3; j >= 0; --j) { r1 += a1[j]; r2 += a2[j]; l1[j] = r1; l2[j] = r2; }
        const unsigned long long e1 = wave_suffix_u64(r1) - r1, e2 = wave_suffix_u64(r2) - r2;
        SelCtx cx;
        cx.S2 = S2; cx.mx = mx; cx.n = n; cx.denf = (float)(2 * QMAX - 1);
        cx.u = 0x1p-24;
        cx.fixu = ldexp(1.0, -K1);
        cx.Kterm = (double)p.nq * ldexp(1.0, -fixed_exp(mx, p.nq));
        cx.Nterm = (double)((long long)p.mv.nelem * QMAX);
        cx.tiny = 8.0 * (double)p.mv.nelem * 0x1p-149;
        double lo[4], hi[4], hmin = 1e300;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = 4 * lane + j;
          lo[j] = hi[j] = 1e300;
          if (c < n) cx.bounds_s((double)s_sc[c], l1[j] + e1, l2[j] + e2, lo[j], hi[j]);
          hmin = fmin(hmin, hi[j]);
        }
        const double mn = wave_min_f64(hmin);
        unsigned cnt = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) cnt += (4 * lane + j < n && (lo[j] <= mn || widen)) ? 1u : 0u;
        const unsigned suf = wave_suffix_u32(cnt);   // keeps in lanes >= this one
        const unsigned tot = __builtin_amdgcn_readfirstlane(suf);   // lane 0: all of them
        int pos = (int)(tot - suf);                  // keeps in lanes below this one
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = 4 * lane + j;
          if (c < n && (lo[j] <= mn || widen)) {
            if (pos < kMaxSel) lsel[2 + pos] = c;
            ++pos;
          }
        }
        if (lane == 0) s_wcnt[0] = (int)tot;
      }
      __syncthreads();
      const int total = s_wcnt[0];
      const bool all = total > kMaxSel || total == 0;
      const int ns = all ? n : total;
      int cstar;
      ADMMQ_TL_PH(9);
      if (ns == 1) {
        cstar = lsel[2];
      } else {
        // ---- stage 2 (rare): the canonical SSE of S over the team (oracle/quant_oracle.py)
        const int K = fixed_exp(mx, p.nq);
        const int q = 1 << (bits - 1);
        const float qlo = (float)(-q), qhi = (float)(q - 1);
        for (int j = tid; j < ns; j += kTLThreads) s_part[j] = 0ull;
        __syncthreads();
        for (int j = 0; j < ns; ++j) {
          const int c = all ? j : lsel[2 + j];
          unsigned long long gq = 0ull;
          if (owner) {
            const float s = s_sc[c];
            const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
            float dd[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float qv = nan_clamp(__builtin_rintf(xs[e] / s), qlo, qhi);
              dd[e] = xs[e] - qv * s;
            }
            gq = to_fixed((dd[0] * dd[0] + dd[1] * dd[1]) + (dd[2] * dd[2] + dd[3] * dd[3]), K);
          }
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) gq += __shfl_xor(gq, off);
          if (lane == 0 && gq) atomicAdd(&s_part[j], gq);
        }
        __syncthreads();
        for (int j = tid; j < ns; j += kTLThreads)
          if (s_part[j]) atomicAdd(&sy.sse[slot][all ? j : lsel[2 + j]], s_part[j]);
        // ---- barrier 2b: the team's SSE of S
        if (!team_barrier(&sy.bar, nteam * ++nbar, wait_polls, &s_ok)) { fault = true; break; }
        unsigned long long best = ~0ull;
        int bi = 0x7fffffff;
        for (int j = tid; j < ns; j += kTLThreads) {
          const int c = all ? j : lsel[2 + j];
          const unsigned long long v = ald_u64(&sy.sse[slot][c]);
          if (v < best || (v == best && c < bi)) { best = v; bi = c; }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          const unsigned long long ov = __shfl_xor(best, off);
          const int oi = __shfl_xor(bi, off);
          if (ov < best || (ov == best && oi < bi)) { best = ov; bi = oi; }
        }
        if (lane == 0) { s_best[wave] = best; s_bidx[wave] = bi; }
        __syncthreads();
        if (tid == 0) {
          unsigned long long b = s_best[0];
          int c = s_bidx[0];
          for (int w = 1; w < kTLThreads / 64; ++w)
            if (s_best[w] < b || (s_best[w] == b && s_bidx[w] < c)) { b = s_best[w]; c = s_bidx[w]; }
          s_cstar = c;
        }
        __syncthreads();
        cstar = s_cstar;
      }
      qp = qparams_mse(bits, cand_t(mx, cstar, n));
    }
    // ---- finalize (admm_finalize_block's float32 operations, in the same order)
    ADMMQ_TL_PH(10);
    double r1 = 0.0, r2 = 0.0, r3 = 0.0, r4 = 0.0;
    if (owner) {
      const float ts[4] = {t4.x, t4.y, t4.z, t4.w}, xs[4] = {x4.x, x4.y, x4.z, x4.w};
      const float hs[4] = {h4.x, h4.y, h4.z, h4.w}, us[4] = {u4.x, u4.y, u4.z, u4.w};
      const float fs[4] = {f4.x, f4.y, f4.z, f4.w};
      float a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
      float ho[4], uo[4], po[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = qcol + k < R;
        const float hq = apply_quant_mse(xs[k], qp);   // H = quantize(H_T - U)
        const float hn = ok ? hq : 0.f;
        const float dh = ok ? hn - ts[k] : 0.f;
        const float un2 = ok ? us[k] + dh : 0.f;        // U += H - H_T
        ho[k] = hn; uo[k] = un2;
        po[k] = ok ? fs[k] + rho * (hn + un2) : 0.f;    // next rhs F + rho(H+U)
        const float dp = ok ? hn - hs[k] : 0.f;
        a1 += dh * dh; a2 += hn * hn; a3 += dp * dp; a4 += un2 * un2;
      }
      r1 = (double)a1; r2 = (double)a2; r3 = (double)a3; r4 = (double)a4;
      h4 = make_float4(ho[0], ho[1], ho[2], ho[3]);
      u4 = make_float4(uo[0], uo[1], uo[2], uo[3]);
      const u32x4v w = {__float_as_uint(po[0]), __float_as_uint(po[1]), __float_as_uint(po[2]), __float_as_uint(po[3])};
      __builtin_amdgcn_raw_buffer_store_b128(w, prs, qoff * 4, 0, 16);   // sc1 (write-through)
    }
    r1 = wave_sum_f64(r1); r2 = wave_sum_f64(r2); r3 = wave_sum_f64(r3); r4 = wave_sum_f64(r4);
    if (lane == 0) { s_red[wave][0] = r1; s_red[wave][1] = r2; s_red[wave][2] = r3; s_red[wave][3] = r4; }
    __syncthreads();
    if (tid < 4) {
      double v = 0.0;
#pragma unroll
      for (int w = 0; w < kTLThreads / 64; ++w) v += s_red[w][tid];
      atomicAdd(&sy.res[slot][tid], v);
    }
    if (leader && tid == 0) p.flags[1] = it + 1;
    // ---- barrier 3: the next P and the residual sums
    ADMMQ_TL_PH(11);
    if (!team_barrier(&sy.bar, nteam * ++nbar, wait_polls, &s_ok)) { fault = true; break; }
    ADMMQ_TL_PH(12);
    if (leader) {   // every reader of this slot (and of the other slot's residuals) is past it
      for (int b = tid; b <= n; b += kTLThreads) {
        ast_u64(&sy.h1[slot][b], 0ull);
        ast_u64(&sy.h2[slot][b], 0ull);
        ast_u64(&sy.sse[slot][b], 0ull);
      }
      if (tid == 0) ast_f64(&sy.s2[slot], 0.0);
      if (tid < 4) ast_f64(&sy.res[slot ^ 1][tid], 0.0);
    }
    ADMMQ_TL_PH(13);
  }
#undef ADMMQ_TL_PH
  if (ADMMQ_TRACE && tid == 0 && blockIdx.x < kTLTraceMax)
    for (int k = 0; k < kTLPhases; ++k) g_tl_trace[blockIdx.x][k] = ph[k];
  if (fault) {
    if (tid == 0) p.flags[3] = 1;   // internal fault: the caller re-runs without this loop
    return;
  }
  if (owner) {
    *(gst4t*)(p.H + qoff) = gf32x4{h4.x, h4.y, h4.z, h4.w};
    *(gst4t*)(p.U + qoff) = gf32x4{u4.x, u4.y, u4.z, u4.w};
  }
}

static_assert(1152 / 32 <= kTLMaxTeam, "a team of ld / 32 workgroups polls in one wave");
int launch_thin_loop(const ProbDesc* d, const ThinLoopUnit* units, int nunits, ThinSync* sync, int nr, int maxld,
                     int n_iter, float eps, int ncand, int bits, unsigned wait_polls, int ncu, hipStream_t s) {
  if (nunits <= 0 || nunits > ncu || n_iter <= 0 || maxld > 1152) return -1;
  if (ncand < 2 || ncand > kTLMaxCand || bits < 2 || bits > 5) return -1;
  const int NRv = nr <= 9 ? 9 : 16;
  const int region_a = NRv * kTSChunk + 8 * NRv * 64;   // staged P / partials, then the cw = 64 stash
  const size_t lds = thin_loop_lds_bytes(region_a, ncand, bits);
  if (lds > 160 * 1024 - 12 * 1024) return -1;   // leaves room for the static LDS
  auto run = [&](auto kern) -> int {
    int nb = 0;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return -2;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, kTLThreads, lds) != hipSuccess || nb < 1) return -2;
    hipLaunchKernelGGL(kern, dim3(nunits), dim3(kTLThreads), lds, s, d, units, sync, region_a, n_iter, eps, ncand,
                       bits, wait_polls);
    return 0;
  };
#define ADMMQ_TL(NRV)                            \
  switch (bits) {                                \
    case 2: return run(k_thin_loop<NRV, 2>);     \
    case 3: return run(k_thin_loop<NRV, 4>);     \
    case 4: return run(k_thin_loop<NRV, 8>);     \
    default: return run(k_thin_loop<NRV, 16>);   \
  }
  if (NRv == 9) { ADMMQ_TL(9) }
  ADMMQ_TL(16)
#undef ADMMQ_TL
}

}  // namespace admmq

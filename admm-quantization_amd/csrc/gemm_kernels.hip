// ADMM primal solve (source/admm.py:56-57):  H_T = (F + rho(H+U)) (G + rho I)^-1
// as one grouped MFMA GEMM  HT[Ip x ld] = P[Ip x ld] . M[ld x ld]  over every active
// (layer, mode) problem. P is produced by the previous iteration's finalize kernel; M is
// symmetric, so the B operand is read as rows of M.
//
// Two operand forms (admmq_set_solve_mode):
//   kSolveF32    P and M in fp32, v_mfma_f32_32x32x2_f32 (an fp32 FMA chain).
//   kSolveSplit  P and M each stored as two fp16 planes per row, scaled by a power of
//                two per row: x 2^e = hi + lo with hi = fp16(x 2^e), lo = fp16(x 2^e - hi)
//                (|x - (hi + lo) 2^-e| <= 2^-22 |x|). Then
//                    H_T = 2^-(eP_i + eM_j) (Ph Mh + Ph Ml + Pl Mh)
//                on v_mfma_f32_32x32x16_f16 (16x the fp32 MFMA rate, 3 products, fp32
//                accumulation): per product about 2^-21 relative, the size of the fp32
//                GEMM's own accumulation error at K ~ 1000. The planes take the bytes of
//                the fp32 operand, so the kernel moves the same data at 5x less MFMA time.
//
// Tile (32*WM) x 64 per workgroup of 2*WM*KS waves; the KS waves (ks, wm, wn) own the
// 32 x 32 sub-tile at (32 wm, 32 wn), each with one accumulator chain over its 1/KS slice
// of every K-step, summed in fixed order through LDS at the end. WM = 2 (64 x 64 tiles)
// for factors with I > 32, WM = 1 (32 x 64) for 17..32-row factors.
//
// Staging: K-step 32 (128 B per operand row in both forms: 32 floats, or 32 hi + 32 lo
// halfs). Both operands go global -> LDS by global_load_lds_dwordx4 (no VGPR round trip)
// into an NS-deep ring of stages, NS-1 K-steps in flight; each wave waits with a counted
// vmcnt for its own pieces of the stage it is about to read and a raw s_barrier publishes
// the stage (a __syncthreads would drain every in-flight load). A stage image is
// row-major, 128 B per row, with the 16-B chunk c of row r stored at chunk position
// c ^ ((r >> 1) & 7) - applied on the global source address, since an LDS-DMA writes
// lane-linear - so the fragment reads (ds_read_b128) are bank-conflict free.
// fp32: the k-order inside a K-step is k = 16 h + m (lane half h, MFMA m); split: chunk
// 2 kc + h holds hi halfs k = 16 kc + 8 h .. +7 (the f16 MFMA's lane-half k group), chunk
// 4 + 2 kc + h the matching lo halfs. A and B use the same order in either form.
//
// Epilogue: store HT (split: scaled back by ldexp), and fold max|X|, min X, max X of
// X = HT - U over the valid region into the problem's per-iteration stat slot.
#include <algorithm>
#include <cstdlib>

#include <hip/hip_ext.h>

#include "quant_device.h"

// Diagnostic builds only (EXTRA=-DADMMQ_GEMM_DIAG=n, never the product library; results
// are garbage): 1 = the fp32 K-loop without its MFMAs (staging + fragment reads only),
// 2 = without its global -> LDS staging after the first stages (fragment reads + MFMAs).
#ifndef ADMMQ_GEMM_DIAG
#define ADMMQ_GEMM_DIAG 0
#endif

namespace admmq {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int BN = 64, BK = 32;

__device__ __forceinline__ bool converged_before(const ProbDesc& p, int slot_prev, int iter, float eps) {
  if (iter == 0) return false;
  const double* r = p.res + 4 * kResRep * slot_prev;   // kResRep replicas of {S1, S2, S3, S4}
  double t[4] = {0.0, 0.0, 0.0, 0.0};
  for (int q = 0; q < kResRep; ++q)
    for (int k = 0; k < 4; ++k) t[k] += r[4 * q + k];
  const double rr = t[0] / t[1];
  const double ss = t[2] / t[3];
  return (rr < (double)eps) && (ss < (double)eps);
}

// 16 B per lane global -> LDS (global_load_lds_dwordx4): LDS bytes [lds + 16 lane, +16).
// The builtin exists only for the device pass (its LDS pointer type does not form on
// the host, and a template kernel using it would silently lose its host launch stub).
typedef __attribute__((address_space(3))) void lds_void;

// The same from a buffer descriptor: LDS bytes [lds + 16 lane, +16) <- rs[voff + soff],
// voff per lane, soff scalar (device pass only, like glds16)
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t rs, float* lds, unsigned voff, unsigned soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds, 16, voff, soff, 0, 0);
#endif
}

__device__ __forceinline__ void glds16(const float* g, float* lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(g, lds, 16, 0, 0);
#endif
}

// Plain loads through a global (not flat) pointer: flat loads count in lgkmcnt too, so
// an LDS wait would also drain them.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const float gfloat;
typedef __attribute__((address_space(1))) const f32x4 gfloat4;
__device__ __forceinline__ float ldg(const float* q) { return *(gfloat*)q; }
__device__ __forceinline__ float4 ldg4(const float* q) {
  const f32x4 v = *(gfloat4*)q;
  return make_float4(v.x, v.y, v.z, v.w);
}

// Workgroup barrier that is also a compiler barrier for memory operations (the builtin
// s_barrier is not: LDS reads of the next stage could be hoisted above it) and adds
// no waitcnt of its own (unlike __syncthreads, which would drain in-flight glds).
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

// s_waitcnt vmcnt(n) only (expcnt / lgkmcnt left at their no-wait maxima), gfx9 encoding
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ f16x8 as_h8(float4 v) { return __builtin_bit_cast(f16x8, v); }

// K-split combine of a 64 x 64 fp32 tile (4 waves, 256 threads, one f32x16 accumulator
// per thread in the 32x32x2 C/D layout; api.hip ksplit_pieces). Piece pc of np has summed
// K-steps [k0, k0 + nk) of the tile. Every piece publishes its partial: 4 x 16-B sc1
// (write-through) stores per thread into slot pc of the tile's partial images, laid out
// by thread, so each thread later reads back exactly the elements it owns; each storing
// wave drains them (vmcnt(0)) before the workgroup barrier behind which one lane adds to
// the tile's arrival counter (agent scope). The workgroup whose add completes the tile
// (the counter advances by np per iteration: (old + 1) % np == 0) reads the other slots
// with sc1 loads after a barrier its lane joined (MI355X_MICROARCH.md, inter-workgroup
// visibility, first row) and forms ((p0 + p1) + p2) + ... in piece order - the same float32
// additions whichever piece arrives last, so the tile's bits are fixed by (I, R) alone.
// Returns false for the other pieces (they end without an epilogue).
typedef unsigned u32x4g __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bool ksplit_combine(const GemmTile& tl, f32x16& acc, int* lds_last) {
  const int tid = threadIdx.x;
  const int np = tl.np, pc = tl.pc;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(tl.part, 0, np * 16384, 0x00020000);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const u32x4g w = {__float_as_uint(acc[4 * q]), __float_as_uint(acc[4 * q + 1]), __float_as_uint(acc[4 * q + 2]),
                      __float_as_uint(acc[4 * q + 3])};
    __builtin_amdgcn_raw_buffer_store_b128(w, rs, ((pc * 4 + q) * 256 + tid) * 16, 0, 16);   // sc1
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(tl.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *lds_last = ((old + 1u) % (unsigned)np) == 0u ? 1 : 0;
  }
  __syncthreads();
  if (!*lds_last) return false;
  u32x4g v[kKsplitMax][4];
#pragma unroll
  for (int s = 0; s < kKsplitMax; ++s)
    if (s < np && s != pc)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[s][q] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((s * 4 + q) * 256 + tid) * 16, 0, 16);
  f32x16 sum;
#pragma unroll
  for (int s = 0; s < kKsplitMax; ++s) {
    if (s >= np) break;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float x = s == pc ? acc[r] : __uint_as_float(v[s][r >> 2][r & 3]);
      sum[r] = s == 0 ? x : sum[r] + x;
    }
  }
  acc = sum;
  return true;
}

// Diagnostics (make TRACE=1 only): per workgroup of the last k_gemm launch {start, end,
// (block << 48) | (K-steps << 40) | (XCC_ID << 32) | HW_ID} (admmq_debug_gemm_trace, tools/gemm_timeline.py)
constexpr int kGemmTraceMax = 8192;
__device__ unsigned long long g_gemm_trace[kGemmTraceMax][4];   // + shader-clock cycles of the workgroup
// ... and per workgroup {K-loop end, K-split combine end} (k_gemm_f32b; 0 where not reached)
__device__ unsigned long long g_gemm_trace2[kGemmTraceMax][2];
int copy_gemm_trace2(unsigned long long* host, int n) {
  n = n < kGemmTraceMax ? n : kGemmTraceMax;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_trace2), (size_t)n * 2 * sizeof(unsigned long long)) == hipSuccess
             ? n : -1;
}
// ... and per workgroup the set of SIMDs its waves ran on (bit per SIMD id, k_gemm_f32b)
__device__ unsigned g_gemm_simd[kGemmTraceMax];
int copy_gemm_simd(unsigned* host, int n) {
  n = n < kGemmTraceMax ? n : kGemmTraceMax;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_simd), (size_t)n * sizeof(unsigned)) == hipSuccess ? n : -1;
}
int copy_gemm_trace(unsigned long long* host, int n) {
  n = n < kGemmTraceMax ? n : kGemmTraceMax;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_trace), (size_t)n * 4 * sizeof(unsigned long long)) == hipSuccess
             ? n : -1;
}

// One workgroup per tile (the grid is the tile list, longest K first, CU-balanced by the
// planner). SPLIT selects the operand form (see the file header).
// CW: 32-column sub-tiles per wave (1: BN = 64 columns per tile; 2: 128, each wave's A
// fragment feeding two sub-tiles - the wide tiles of large launches, CW = 2 with WM = 4:
// 128 x 128, 8 waves, a third fewer operand bytes per MAC than 128 x 64).
template <int WM, int KS, int NS, bool SPLIT, int CW = 1>
__global__ __launch_bounds__(128 * WM * KS) __attribute__((amdgpu_waves_per_eu(
    WM == 8 ? 4 : (WM == 2 && KS == 2 ? 5 : (NS <= 3 ? (WM == 4 ? 4 : 3) : 1))))) void k_gemm(
    const ProbDesc* __restrict__ probs, const GemmTile* __restrict__ tiles, int slot, int iter, float eps, int ncand) {
  constexpr int BM = 32 * WM;
  constexpr int BNT = BN * CW;                 // tile columns
  constexpr int NSUB = 2 * WM;                 // waves per K-slice (each: 32 rows x 32 CW columns)
  constexpr int NW = NSUB * KS;                // waves
  constexpr int NT = 64 * NW;
  constexpr int ROWS = BM + BNT;               // image rows per stage (A then B)
  constexpr int STAGE = ROWS * 32;             // floats per stage
  constexpr int NG = ROWS / 8;                 // glds wave-instructions per stage (8 rows each)
  constexpr int GPW = NG / NW;                 // ... per wave
  constexpr int QS = 4 / KS;                   // fp32: b128 fragment reads per operand per wave per K-step
  constexpr int KCW = 2 / KS;                  // split: 16-deep k chunks per wave per K-step
  static_assert(KS == 1 || (KS - 1) * NSUB * 1024 <= STAGE, "split-K partials fit in one stage");
  static_assert(CW == 1 || (CW == 2 && KS == 1), "CW");
  static_assert(NG % NW == 0, "stage rows must split evenly over the waves");
  static_assert(KS == 1 || KS == 2 || (!SPLIT && KS == 4), "KS");
  static_assert(NS >= 2 && NS <= 4 && GPW * (NS - 2) < 64, "NS");

  // one __shared__ object per stage: the compiler then sees that a stage being read is
  // not the one being filled and does not drain the in-flight loads before the reads
  __shared__ __attribute__((aligned(16))) float st0[STAGE];
  __shared__ __attribute__((aligned(16))) float st1[STAGE];
  __shared__ __attribute__((aligned(16))) float st2[NS > 2 ? STAGE : 4];
  __shared__ __attribute__((aligned(16))) float st3[NS > 3 ? STAGE : 4];
  float* const stp[4] = {st0, st1, st2, st3};
  __shared__ unsigned red[3][NSUB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // scalar: the LDS bases of the staging stay in SGPRs
  const int sub = wave % NSUB, ks = wave / NSUB;
  const int wm = sub / 2, wn = sub & 1;
  const int i = lane & 31, h = lane >> 5;
  const int swz = (i >> 1) & 7;
  const int aoff = (32 * wm + i) * 32, boff = (BM + 32 * CW * wn + i) * 32;   // sub-tile c: boff + 32 * 32 c

  const unsigned long long T0 = ADMMQ_NOW();
  const unsigned long long C0 = ADMMQ_TRACE ? __builtin_amdgcn_s_memtime() : 0ull;
  const GemmTile tl = tiles[blockIdx.x];
  if (tl.nk <= 0) return;   // grid padding (order_tiles_for_cus)
  const ProbDesc& p = probs[tl.prob];
  const int ld = tl.ld, ldm = tl.ldm;
  const int row0 = tl.tm * BM, col0 = tl.tn * BNT;
  const int nk = tl.nk;
  // the epilogue's U entries (X = H_T - U) and, split form, the row / column exponents:
  // loaded before the first stages so their latency is spent under the K-loop (vector
  // loads complete in issue order: the stage waits below then also cover these)
  // (wide tiles, WM = 4: loaded in the epilogue instead - those launches run many rounds
  // of tiles, so other workgroups cover the latency, and the registers stay free)
  constexpr bool PRE = WM < 4 && !(WM == 2 && KS == 2);   // (WM >= 4 and the 8-wave 64 x 64 tiles: the epilogue loads after the K-loop)
  float upre[CW][16];
  int epre[16];
  int ecol[CW] = {};
  auto load_epi = [&]() {
#pragma unroll
    for (int c = 0; c < CW; ++c) {
      const int col = col0 + 32 * (CW * wn + c) + i;
      const int colc = col < ld ? col : 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
        upre[c][r] = ldg(tl.U + (size_t)row * ld + colc);
        if (SPLIT && c == 0) epre[r] = *(__attribute__((address_space(1))) const int*)(tl.eP + row);
      }
      if (SPLIT) ecol[c] = *(__attribute__((address_space(1))) const int*)(tl.eM + colc);
    }
  };
  if constexpr (PRE) load_epi();
  // the staging pieces: buffer_load ... lds with descriptors rebased to the tile (P at its
  // first row, M at its first column's row), a per-lane offset fixed for the tile and the
  // K-step's byte offset in an SGPR - no VALU address arithmetic in the K-loop (the fp32
  // MFMA shares the VALU's pipe; k_gemm_f32b). A piece is 8 image rows,
  // all P rows or all M rows (BM is a multiple of 8), so its descriptor is wave-uniform.
  // (a K-split piece, fp32 64 x 64 tiles only, starts at K-step k0: 128 B per K-step in both forms)
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)(tl.P + (size_t)row0 * ld + tl.k0 * BK), 0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)(tl.M + (size_t)col0 * ldm + tl.k0 * BK), 0, 0x7FFFFFFF, 0x00020000);
  unsigned voff[GPW];
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int g = wave * GPW + j;
    const int r = 8 * g + (lane >> 3);                       // image row
    const int c = (lane & 7) ^ ((r >> 1) & 7);               // source chunk of LDS position lane & 7
    // B rows past ldm (the last 128-column tile of a CW = 2 launch) read the last row: they
    // only feed columns >= ld, which are never stored
    voff[j] = (r < BM) ? (unsigned)((r * ld + 4 * c) * 4) : (unsigned)((min(r - BM, ldm - 1 - col0) * ldm + 4 * c) * 4);
  }
#define ADMMQ_ISSUE(s, kt)                                                                                      \
  _Pragma("unroll") for (int j = 0; j < GPW; ++j)                                                              \
    blds16(8 * (wave * GPW + j) < BM ? rsA : rsB, stp[s] + (wave * GPW + j) * 256, voff[j], (kt) * (BK * 4))
  // the first NS-1 stages go out before the stop test, whose inputs (flag, residual
  // sums) are one dependent read further away; a stopped problem drains them unused
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) ADMMQ_ISSUE(s, min(s, nk - 1));
  bool skip = p.flags[0] != 0;
  if (!skip && converged_before(p, slot ^ 1, iter, eps)) {
    if (tl.first && tid == 0) p.flags[0] = 1;   // sticky "break" (source/admm.py:64-65)
    skip = true;
  }
  if (skip) {
    wait_vmcnt<0>();   // the speculative stage loads land before the wave ends
    return;
  }
  if (tl.first) {   // this iteration's quantizer-search accumulators start at zero
    unsigned long long* sse = p.mv.sse + (size_t)slot * ncand;
    unsigned long long* h1 = p.mv.h1 + (size_t)slot * kHistRep * (ncand + 1);
    unsigned long long* h2 = p.mv.h2 + (size_t)slot * kHistRep * (ncand + 1);
    for (int c = tid; c < ncand; c += NT) sse[c] = 0ull;
    for (int c = tid; c < kHistRep * (ncand + 1); c += NT) { h1[c] = 0ull; h2[c] = 0ull; }
    if (tid == 0) { p.mv.s2[slot] = 0.0; p.mv.ticket[slot] = 0u; }
  }

  f32x16 acc[CW], psum;
#pragma unroll
  for (int c = 0; c < CW; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = psum[r] = 0.f;
  // serial K-split (fp32 64 x 64 tiles only: k_gemm_f32b's fold, the same order)
  constexpr bool FOLD = !SPLIT && WM == 2 && KS == 1 && CW == 1;
  const int ser = FOLD ? tl.ser : 1;
  int pf = 1, kb = ser > 1 ? nk / ser : nk;

  // Per K-step kt on stage s = kt % NS: wait for it (counted vmcnt: the NS-2 later
  // stages stay in flight), publish it (barrier), refill the stage consumed one step
  // ago with K-step kt + NS - 1, multiply. Every step issues exactly GPW loads (past
  // the end the last K-step is re-read into a stage nobody reads), so the wait count
  // is one constant and the compiler's own wait tracking stays exact. The main loop
  // runs whole groups of NS steps (stage static, no branches around the MFMAs, which
  // would move the accumulators out of AGPRs); the last < NS steps run guarded.
#define ADMMQ_STEP(s, kt)                                                                     \
  do {                                                                                        \
    wait_vmcnt<GPW * (NS - 2)>();                                                             \
    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): reads of the refilled stage done */    \
    raw_barrier();                                                                            \
    if (ADMMQ_GEMM_DIAG != 2 || SPLIT) ADMMQ_ISSUE(((s) + NS - 1) % NS, min((kt) + NS - 1, nk - 1)); \
    if (FOLD && (kt) == kb && (kt) > 0) {                                                     \
      _Pragma("unroll") for (int r = 0; r < 16; ++r) {                                        \
        psum[r] = pf == 1 ? acc[0][r] : psum[r] + acc[0][r];                                  \
        acc[0][r] = 0.f;                                                                      \
      }                                                                                       \
      ++pf;                                                                                   \
      kb = pf * nk / ser;                                                                     \
    }                                                                                         \
    const float* st = stp[s];                                                                 \
    if constexpr (SPLIT) {                                                                    \
      _Pragma("unroll") for (int q = 0; q < KCW; ++q) {                                       \
        const int kc = KCW * ks + q;                                                          \
        const int ch = ((2 * kc + h) ^ swz) * 4, cl = ((4 + 2 * kc + h) ^ swz) * 4;           \
        const f16x8 ah = as_h8(*reinterpret_cast<const float4*>(st + aoff + ch));             \
        const f16x8 al = as_h8(*reinterpret_cast<const float4*>(st + aoff + cl));             \
        _Pragma("unroll") for (int c = 0; c < CW; ++c) {                                      \
          const f16x8 bh = as_h8(*reinterpret_cast<const float4*>(st + boff + 1024 * c + ch)); \
          const f16x8 bl = as_h8(*reinterpret_cast<const float4*>(st + boff + 1024 * c + cl)); \
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[c], 0, 0, 0);           \
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[c], 0, 0, 0);           \
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[c], 0, 0, 0);           \
        }                                                                                     \
      }                                                                                       \
    } else {   /* fragments of group qq + 1 read while group qq's MFMAs run (2 register sets) */ \
      float4 fa[2], fb[2][CW];                                                                \
      _Pragma("unroll") for (int qq = 0; qq < QS; ++qq) {                                     \
        if (qq == 0) {                                                                        \
          const int cp = ((4 * h + QS * ks) ^ swz) * 4;                                       \
          fa[0] = *reinterpret_cast<const float4*>(st + aoff + cp);                           \
          _Pragma("unroll") for (int c = 0; c < CW; ++c)                                      \
            fb[0][c] = *reinterpret_cast<const float4*>(st + boff + 1024 * c + cp);           \
          __builtin_amdgcn_sched_group_barrier(0x100, 1 + CW, 0);                             \
        }                                                                                     \
        if (qq + 1 < QS) {                                                                    \
          const int cn = ((4 * h + QS * ks + qq + 1) ^ swz) * 4;                              \
          fa[(qq + 1) & 1] = *reinterpret_cast<const float4*>(st + aoff + cn);                \
          _Pragma("unroll") for (int c = 0; c < CW; ++c)                                      \
            fb[(qq + 1) & 1][c] = *reinterpret_cast<const float4*>(st + boff + 1024 * c + cn); \
          __builtin_amdgcn_sched_group_barrier(0x100, 1 + CW, 0);                             \
        }                                                                                     \
        _Pragma("unroll") for (int c = 0; c < CW; ++c) {                                      \
          const float4 a = fa[qq & 1], b = fb[qq & 1][c];                                     \
          if (ADMMQ_GEMM_DIAG == 1) {                                                         \
            acc[c][0] += a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;                       \
          } else {                                                                            \
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc[c], 0, 0, 0);           \
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc[c], 0, 0, 0);           \
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc[c], 0, 0, 0);           \
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc[c], 0, 0, 0);           \
          }                                                                                   \
        }                                                                                     \
        __builtin_amdgcn_sched_group_barrier(0x008, 4 * CW, 0);                               \
      }                                                                                       \
    }                                                                                         \
  } while (0)
  const int nfull = nk / NS * NS;
  for (int kt0 = 0; kt0 < nfull; kt0 += NS) {
#pragma unroll
    for (int s = 0; s < NS; ++s) ADMMQ_STEP(s, kt0 + s);
  }
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (nfull + s < nk) ADMMQ_STEP(s, nfull + s);
#undef ADMMQ_STEP
#undef ADMMQ_ISSUE
  __syncthreads();   // nothing in flight any more; the stages may be reused
  if (KS > 1) {      // fixed-order reduction of the KS partial accumulators (deterministic)
    if (ks > 0) {
      float* dst = st0 + ((ks - 1) * NSUB + sub) * 1024;
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[r * 64 + lane] = acc[0][r];
    }
    __syncthreads();
    if (ks == 0) {
#pragma unroll
      for (int j = 1; j < KS; ++j) {
        const float* s2 = st0 + ((j - 1) * NSUB + sub) * 1024;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[0][r] += s2[r * 64 + lane];
      }
    }
  }
  if constexpr (FOLD) {   // K-split: the serial form's last piece, or a parallel piece (k_gemm_f32b's combine)
    if (ser > 1)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[0][r] = psum[r] + acc[0][r];
    if (tl.np > 1) {
      __shared__ int klast;
      if (!ksplit_combine(tl, acc[0], &klast)) return;
    }
  }

  // epilogue (waves ks == 0): C/D map col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  if (ks == 0) {
    if constexpr (!PRE) load_epi();
    unsigned amax = 0u, mn = 0xFFFFFFFFu, mxo = 0u;
    // descriptor fields once into registers (the stores below may alias the descriptor)
    typedef __attribute__((address_space(1))) float gf32;
    gf32* const HTg = (gf32*)p.HT;
    gf32* const Xg = p.X_dbg ? (gf32*)p.X : nullptr;   // X = H_T - U is re-formed by its readers; debug output only
    const int pI = p.I, pR = p.R;
#pragma unroll
    for (int c = 0; c < CW; ++c) {
      const int col = col0 + 32 * (CW * wn + c) + i;
      if (col < ld) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = row0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
          const size_t off = (size_t)row * ld + col;
          const float ht = SPLIT ? __builtin_ldexpf(acc[c][r], -(epre[r] + ecol[c])) : acc[c][r];
          const float x = ht - upre[c][r];
          HTg[off] = ht;
          if (Xg) Xg[off] = x;
          if (row < pI && col < pR) {
            amax = max(amax, __float_as_uint(x) & 0x7FFFFFFFu);
            const unsigned e = enc_ord(x);
            mn = min(mn, e);
            mxo = max(mxo, e);
          }
        }
      }
    }
    amax = wave_max_u32(amax); mn = wave_min_u32(mn); mxo = wave_max_u32(mxo);
    if (lane == 0) { red[0][sub] = amax; red[1][sub] = mn; red[2][sub] = mxo; }
  }
  __syncthreads();
  if (tid == 0) {
    unsigned a0 = red[0][0], a1 = red[1][0], a2 = red[2][0];
#pragma unroll
    for (int w = 1; w < NSUB; ++w) { a0 = max(a0, red[0][w]); a1 = min(a1, red[1][w]); a2 = max(a2, red[2][w]); }
    unsigned* st = p.mv.stat + 4 * slot;
    atomicMax(&st[0], a0);
    atomicMin(&st[1], a1);
    atomicMax(&st[2], a2);
    if (ADMMQ_TRACE && blockIdx.x < kGemmTraceMax) {
      const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
      g_gemm_trace[blockIdx.x][0] = T0;
      g_gemm_trace[blockIdx.x][3] = __builtin_amdgcn_s_memtime() - C0;
      g_gemm_trace[blockIdx.x][1] = ADMMQ_NOW();
      g_gemm_trace[blockIdx.x][2] = ((unsigned long long)blockIdx.x << 48) | ((unsigned long long)(nk & 0xFF) << 40) |
                                    ((unsigned long long)(xcc & 0xFF) << 32) | hw;
    }
  }
}

// ---------------------------------------------------------------------------
// Persistent fp32 solve (kSolveF32, launches without wide tiles): kF32Slots workgroups
// per CU, workgroup b runs the tiles list[off[b] .. off[b+1]) one after another. The host
// (api.hip: plan_f32_lists) places the tiles by LPT over the CUs on their MFMA work
// (workgroups b and b + ncu share CU b, round-robin dispatch; placement is only for
// speed), so a launch's length is set by the CU total rather than by how the largest
// tiles happen to land. Tile shapes (fixed per problem, so every element's result is
// independent of the batch):
//   BM 128 x 64  (4 waves of 32 x 64: one A fragment feeding two accumulators)
//   BM  64 x 64  (2 x 2 waves of 32 x 32)          - the same MFMA chain per element as
//   BM  32 x 64  (2 waves of 32 x 32 x 2 K-halves)   k_gemm<2,1,..> / k_gemm<1,2,..>
// Every element's MFMA sequence (k = 16 h + 4 qq + j per K-step, KS = 1) is the one of
// the 64 x 64 tiles, so BM 128 and BM 64 give identical bits; BM 32 sums two K-halves
// like k_gemm<1, 2, ..>. Staging as k_gemm: K-step 32, LDS-DMA into an NS-deep ring of
// (128 + 64)-row stages (the rows of smaller tiles use the front of each stage).
template <int BM, int NS>
__device__ __forceinline__ void f32_tile(const ProbDesc* __restrict__ probs, const GemmTile& tl, int slot, int iter,
                                         float eps, int ncand, float* const (&stp)[4], unsigned (*red)[4]) {
  constexpr int CW = BM == 128 ? 2 : 1;           // 32-column accumulators per wave
  constexpr int NSUB = (BM / 32) * (2 / CW);      // sub-tiles (waves per K-slice)
  constexpr int KS = 4 / NSUB;                    // K-slices
  constexpr int QS = 4 / KS;                      // b128 fragment reads per operand per wave per K-step
  constexpr int ROWS = BM + 64;                   // image rows per stage (A then B)
  constexpr int NG = ROWS / 8;                    // glds wave-instructions per stage
  constexpr int GPW = NG / 4;                     // ... per wave
  static_assert(NG % 4 == 0 && GPW * (NS - 2) < 64, "stage split");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = wave % NSUB, ks = wave / NSUB;
  const int wm = sub / (2 / CW), wn = sub % (2 / CW);
  const int i = lane & 31, h = lane >> 5;
  const int swz = (i >> 1) & 7;
  const int aoff = (32 * wm + i) * 32, boff = (BM + 32 * CW * wn + i) * 32;   // sub-tile c: boff + 1024 c
  const ProbDesc& p = probs[tl.prob];
  const int ld = tl.ld, ldm = tl.ldm;
  const int row0 = tl.tm * BM, col0 = tl.tn * 64;
  const int nk = tl.nk;
  // the epilogue's U entries: loaded first (their latency is spent under the K-loop),
  // except for the two-accumulator waves (BM 128), which load them after the K-loop
  constexpr bool PRE = CW == 1;
  float upre[CW][16];
  auto load_u = [&]() {
#pragma unroll
    for (int c = 0; c < CW; ++c) {
      const int col = col0 + 32 * (CW * wn + c) + i;
      const int colc = col < ld ? col : 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
        upre[c][r] = ldg(tl.U + (size_t)row * ld + colc);
      }
    }
  };
  if constexpr (PRE) load_u();
  const float* src[GPW];
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int g = wave * GPW + j;
    const int r = 8 * g + (lane >> 3);                       // image row
    const int c = (lane & 7) ^ ((r >> 1) & 7);               // source chunk of LDS position lane & 7
    src[j] = (r < BM) ? tl.P + (size_t)(row0 + r) * ld + 4 * c
                      : tl.M + (size_t)min(col0 + r - BM, ldm - 1) * ldm + 4 * c;
  }
#define ADMMQ_ISSUE(s, kt)                                                 \
  _Pragma("unroll") for (int j = 0; j < GPW; ++j)                         \
    glds16(src[j] + (kt) * BK, stp[s] + (wave * GPW + j) * 256)
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) ADMMQ_ISSUE(s, min(s, nk - 1));
  bool skip = p.flags[0] != 0;
  if (!skip && converged_before(p, slot ^ 1, iter, eps)) {
    if (tl.first && tid == 0) p.flags[0] = 1;   // sticky "break" (source/admm.py:64-65)
    skip = true;
  }
  if (skip) {
    wait_vmcnt<0>();   // the speculative stage loads land before the stages are reused
    return;
  }
  if (tl.first) {   // this iteration's quantizer-search accumulators start at zero
    unsigned long long* sse = p.mv.sse + (size_t)slot * ncand;
    unsigned long long* h1 = p.mv.h1 + (size_t)slot * kHistRep * (ncand + 1);
    unsigned long long* h2 = p.mv.h2 + (size_t)slot * kHistRep * (ncand + 1);
    for (int c = tid; c < ncand; c += 256) sse[c] = 0ull;
    for (int c = tid; c < kHistRep * (ncand + 1); c += 256) { h1[c] = 0ull; h2[c] = 0ull; }
    if (tid == 0) { p.mv.s2[slot] = 0.0; p.mv.ticket[slot] = 0u; }
  }
  f32x16 acc[CW];
#pragma unroll
  for (int c = 0; c < CW; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
#define ADMMQ_STEP(s, kt)                                                                     \
  do {                                                                                        \
    wait_vmcnt<GPW * (NS - 2)>();                                                             \
    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): reads of the refilled stage done */    \
    raw_barrier();                                                                            \
    ADMMQ_ISSUE(((s) + NS - 1) % NS, min((kt) + NS - 1, nk - 1));                             \
    const float* st = stp[s];                                                                 \
    _Pragma("unroll") for (int qq = 0; qq < QS; ++qq) {                                       \
      const int cpos = ((4 * h + QS * ks + qq) ^ swz) * 4;                                    \
      const float4 a = *reinterpret_cast<const float4*>(st + aoff + cpos);                    \
      float4 b[CW];                                                                           \
      _Pragma("unroll") for (int c = 0; c < CW; ++c)                                          \
        b[c] = *reinterpret_cast<const float4*>(st + boff + 1024 * c + cpos);                 \
      _Pragma("unroll") for (int c = 0; c < CW; ++c)                                          \
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b[c].x, acc[c], 0, 0, 0);          \
      _Pragma("unroll") for (int c = 0; c < CW; ++c)                                          \
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b[c].y, acc[c], 0, 0, 0);          \
      _Pragma("unroll") for (int c = 0; c < CW; ++c)                                          \
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b[c].z, acc[c], 0, 0, 0);          \
      _Pragma("unroll") for (int c = 0; c < CW; ++c)                                          \
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b[c].w, acc[c], 0, 0, 0);          \
    }                                                                                         \
  } while (0)
  const int nfull = nk / NS * NS;
  for (int kt0 = 0; kt0 < nfull; kt0 += NS) {
#pragma unroll
    for (int s = 0; s < NS; ++s) ADMMQ_STEP(s, kt0 + s);
  }
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (nfull + s < nk) ADMMQ_STEP(s, nfull + s);
#undef ADMMQ_STEP
#undef ADMMQ_ISSUE
  __syncthreads();   // nothing in flight any more; the stages may be reused
  if (KS > 1) {      // fixed-order reduction of the K-slice partial accumulators (deterministic)
    if (ks > 0) {
      float* dst = stp[0] + ((ks - 1) * NSUB + sub) * 1024;
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[r * 64 + lane] = acc[0][r];
    }
    __syncthreads();
    if (ks == 0) {
#pragma unroll
      for (int j = 1; j < KS; ++j) {
        const float* s2 = stp[0] + ((j - 1) * NSUB + sub) * 1024;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[0][r] += s2[r * 64 + lane];
      }
    }
  }
  // epilogue (waves ks == 0): C/D map col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  if (ks == 0) {
    if constexpr (!PRE) load_u();
    unsigned amax = 0u, mn = 0xFFFFFFFFu, mxo = 0u;
    typedef __attribute__((address_space(1))) float gf32;
    gf32* const HTg = (gf32*)p.HT;
    gf32* const Xg = p.X_dbg ? (gf32*)p.X : nullptr;   // X = H_T - U is re-formed by its readers; debug output only
    const int pI = p.I, pR = p.R;
#pragma unroll
    for (int c = 0; c < CW; ++c) {
      const int col = col0 + 32 * (CW * wn + c) + i;
      if (col < ld) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = row0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
          const size_t off = (size_t)row * ld + col;
          const float ht = acc[c][r];
          const float x = ht - upre[c][r];
          HTg[off] = ht;
          if (Xg) Xg[off] = x;
          if (row < pI && col < pR) {
            amax = max(amax, __float_as_uint(x) & 0x7FFFFFFFu);
            const unsigned e = enc_ord(x);
            mn = min(mn, e);
            mxo = max(mxo, e);
          }
        }
      }
    }
    amax = wave_max_u32(amax); mn = wave_min_u32(mn); mxo = wave_max_u32(mxo);
    if (lane == 0) { red[0][sub] = amax; red[1][sub] = mn; red[2][sub] = mxo; }
  }
  __syncthreads();
  if (tid == 0) {
    unsigned a0 = red[0][0], a1 = red[1][0], a2 = red[2][0];
#pragma unroll
    for (int w = 1; w < NSUB; ++w) { a0 = max(a0, red[0][w]); a1 = min(a1, red[1][w]); a2 = max(a2, red[2][w]); }
    unsigned* stt = p.mv.stat + 4 * slot;
    atomicMax(&stt[0], a0);
    atomicMin(&stt[1], a1);
    atomicMax(&stt[2], a2);
  }
}

template <int NS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_gemm_f32p(
    const ProbDesc* __restrict__ probs, const GemmTile* __restrict__ tiles, const int* __restrict__ list_off, int slot,
    int iter, float eps, int ncand) {
  constexpr int STAGE = (128 + 64) * 32;   // floats per stage
  __shared__ __attribute__((aligned(16))) float st0[STAGE];
  __shared__ __attribute__((aligned(16))) float st1[STAGE];
  __shared__ __attribute__((aligned(16))) float st2[NS > 2 ? STAGE : 4];
  __shared__ __attribute__((aligned(16))) float st3[NS > 3 ? STAGE : 4];
  float* const stp[4] = {st0, st1, st2, st3};
  __shared__ unsigned red[3][4];
  const int t1 = list_off[blockIdx.x + 1];
  for (int t = list_off[blockIdx.x]; t < t1; ++t) {
    const GemmTile tl = tiles[t];
    if (tl.bm == 128) f32_tile<128, NS>(probs, tl, slot, iter, eps, ncand, stp, red);
    else if (tl.bm == 64) f32_tile<64, NS>(probs, tl, slot, iter, eps, ncand, stp, red);
    else f32_tile<32, NS>(probs, tl, slot, iter, eps, ncand, stp, red);
    __syncthreads();   // the stages and `red` are reused by the next tile
  }
}

// One fp32 tile per workgroup (k_gemm's grid form) with the persistent kernel's tile
// shapes: BM 128 x 64 (4 waves of 32 x 64) for the large factors, 64 x 64 (2 x 2 waves)
// for the others, in one launch; a 2-deep ring of (128 + 64)-row stages (48 KB: three
// workgroups per CU, like k_gemm's 64 x 64 tiles). With three workgroups sharing a CU,
// one K-step of a workgroup spans ~3 K-steps of MFMA time, longer than a load's latency,
// so one stage in flight is enough.
template <int NS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_gemm_f32t(
    const ProbDesc* __restrict__ probs, const GemmTile* __restrict__ tiles, int slot, int iter, float eps, int ncand) {
  constexpr int STAGE = (128 + 64) * 32;   // floats per stage
  __shared__ __attribute__((aligned(16))) float st0[STAGE];
  __shared__ __attribute__((aligned(16))) float st1[STAGE];
  __shared__ __attribute__((aligned(16))) float st2[NS > 2 ? STAGE : 4];
  __shared__ __attribute__((aligned(16))) float st3[NS > 3 ? STAGE : 4];
  float* const stp[4] = {st0, st1, st2, st3};
  __shared__ unsigned red[3][4];
  const GemmTile tl = tiles[blockIdx.x];
  if (tl.nk <= 0) return;   // grid padding (order_tiles_for_cus)
  if (tl.bm == 128) f32_tile<128, NS>(probs, tl, slot, iter, eps, ncand, stp, red);
  else if (tl.bm == 64) f32_tile<64, NS>(probs, tl, slot, iter, eps, ncand, stp, red);
  else f32_tile<32, NS>(probs, tl, slot, iter, eps, ncand, stp, red);
}

void launch_gemm_f32t(const ProbDesc* d, const GemmTile* tiles, int ntiles, int slot, int iter, float eps, int ncand,
                      hipStream_t s) {
  if (ntiles > 0)
    hipLaunchKernelGGL(k_gemm_f32t<2>, dim3(ntiles), dim3(256), 0, s, d, tiles, slot, iter, eps, ncand);
}

void launch_gemm_f32p(const ProbDesc* d, const GemmTile* tiles, const int* list_off, int nslots, int slot, int iter,
                      float eps, int ncand, hipStream_t s) {
  if (nslots > 0)
    hipLaunchKernelGGL(k_gemm_f32p<3>, dim3(nslots), dim3(256), 0, s, d, tiles, list_off, slot, iter, eps, ncand);
}

// ---------------------------------------------------------------------------
// fp32 64 x 64 tiles with scalar-offset staging (kSolveF32, the C3 / C4 launches): the
// same tile, wave layout, K order and epilogue as k_gemm<2, 1, NS, false> (identical
// bits), but the global -> LDS pieces are buffer_load ... lds with a per-lane offset fixed
// for the whole tile and the K-step's byte offset in an SGPR, and the pieces' LDS bases
// (M0) are wave-uniform scalars: the K-loop issues no VALU address arithmetic (the fp32
// MFMA runs on the same SIMD pipe as the VALU, so every VALU instruction in the loop
// costs MFMA time; tools/probes/mix_probe.hip). The buffer descriptors are rebased per
// tile (P at the tile's first row, M at its first column's row), so every offset stays
// far below 2^31 whatever the problem size. PRE: the epilogue's U entries are loaded
// before the K-loop (their latency hidden, 16 more VGPRs).
template <int NS, bool PRE, bool PRIO = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NS == 2 ? 4 : 3))) void k_gemm_f32b(
    const ProbDesc* __restrict__ probs, const GemmTile* __restrict__ tiles, int slot, int iter, float eps, int ncand) {
  constexpr int BM = 64, ROWS = 128, STAGE = ROWS * 32, GPW = 4;
  __shared__ __attribute__((aligned(16))) float st0[STAGE];
  __shared__ __attribute__((aligned(16))) float st1[STAGE];
  __shared__ __attribute__((aligned(16))) float st2[NS > 2 ? STAGE : 4];
  float* const stp[3] = {st0, st1, st2};
  __shared__ unsigned red[3][4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // scalar: the LDS bases below stay in SGPRs
  const int wm = wave >> 1, wn = wave & 1;
  const int i = lane & 31, h = lane >> 5;
  const int swz = (i >> 1) & 7;
  const int aoff = (32 * wm + i) * 32, boff = (BM + 32 * wn + i) * 32;
  const unsigned long long T0 = ADMMQ_NOW();
  const unsigned long long C0 = ADMMQ_TRACE ? __builtin_amdgcn_s_memtime() : 0ull;
  const GemmTile tl = tiles[blockIdx.x];
  if (tl.nk <= 0) return;   // grid padding (order_tiles_for_cus)
  if (ADMMQ_TRACE && blockIdx.x < kGemmTraceMax) {   // (uniform over the workgroup)
    if (tid == 0) g_gemm_simd[blockIdx.x] = 0u;
    __syncthreads();
    if (lane == 0) atomicOr(&g_gemm_simd[blockIdx.x], 1u << ((__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3));
  }
  const ProbDesc& p = probs[tl.prob];
  const int ld = tl.ld, ldm = tl.ldm;
  const int row0 = tl.tm * BM, col0 = tl.tn * 64;
  const int nk = tl.nk;
  float upre[16];
  auto load_u = [&]() {
    const int col = col0 + 32 * wn + i;
    const int colc = col < ld ? col : 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = row0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
      upre[r] = ldg(tl.U + (size_t)row * ld + colc);
    }
  };
  if constexpr (PRE) load_u();
  // waves 0, 1 stage the 64 P rows (image rows 0..63), waves 2, 3 the 64 M rows; a K-split
  // piece starts at K-step k0 (the descriptors' bases move along the rows)
  const bool isA = wave < 2;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      isA ? (void*)(tl.P + (size_t)row0 * ld + tl.k0 * BK) : (void*)(tl.M + (size_t)col0 * ldm + tl.k0 * BK), 0,
      0x7FFFFFFF, 0x00020000);
  unsigned voff[GPW];
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int r = 8 * (wave * GPW + j) + (lane >> 3);        // image row
    const int c = (lane & 7) ^ ((r >> 1) & 7);               // source chunk of LDS position lane & 7
    voff[j] = isA ? (unsigned)((r * ld + 4 * c) * 4) : (unsigned)((min(r - BM, ldm - 1 - col0) * ldm + 4 * c) * 4);
  }
#define ADMMQ_ISSUE(s, kt)                                                                            \
  _Pragma("unroll") for (int j = 0; j < GPW; ++j)                                                    \
    blds16(rs, stp[s] + (wave * GPW + j) * 256, voff[j], (kt) * (BK * 4))
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) ADMMQ_ISSUE(s, min(s, nk - 1));
  bool skip = p.flags[0] != 0;
  if (!skip && converged_before(p, slot ^ 1, iter, eps)) {
    if (tl.first && tid == 0) p.flags[0] = 1;   // sticky "break" (source/admm.py:64-65)
    skip = true;
  }
  if (skip) {
    wait_vmcnt<0>();
    return;
  }
  if (tl.first) {   // this iteration's quantizer-search accumulators start at zero
    unsigned long long* sse = p.mv.sse + (size_t)slot * ncand;
    unsigned long long* h1 = p.mv.h1 + (size_t)slot * kHistRep * (ncand + 1);
    unsigned long long* h2 = p.mv.h2 + (size_t)slot * kHistRep * (ncand + 1);
    for (int c = tid; c < ncand; c += 256) sse[c] = 0ull;
    for (int c = tid; c < kHistRep * (ncand + 1); c += 256) { h1[c] = 0ull; h2[c] = 0ull; }
    if (tid == 0) { p.mv.s2[slot] = 0.0; p.mv.ticket[slot] = 0u; }
  }
  f32x16 acc, psum;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = psum[r] = 0.f;
  // serial K-split (tl.ser pieces): at the first K-step of piece pf, fold the finished
  // piece into the running sum ((p0 + p1) + ...: ksplit_combine's order) and restart
  const int ser = tl.ser;
  int pf = 1, kb = ser > 1 ? nk / ser : nk;
#define ADMMQ_STEP(s, kt)                                                                     \
  do {                                                                                        \
    wait_vmcnt<GPW * (NS - 2)>();                                                             \
    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): reads of the refilled stage done */    \
    raw_barrier();                                                                            \
    ADMMQ_ISSUE(((s) + NS - 1) % NS, min((kt) + NS - 1, nk - 1));                             \
    if ((kt) == kb && (kt) > 0) {                                                             \
      _Pragma("unroll") for (int r = 0; r < 16; ++r) {                                        \
        psum[r] = pf == 1 ? acc[r] : psum[r] + acc[r];                                        \
        acc[r] = 0.f;                                                                         \
      }                                                                                       \
      ++pf;                                                                                   \
      kb = pf * nk / ser;                                                                     \
    }                                                                                         \
    const float* st = stp[s];                                                                 \
    float4 fa[2], fb[2];                                                                      \
    if (PRIO) __builtin_amdgcn_s_setprio(1);                                                  \
    _Pragma("unroll") for (int qq = 0; qq < 4; ++qq) {                                        \
      if (qq == 0) {                                                                          \
        const int cp = ((4 * h) ^ swz) * 4;                                                   \
        fa[0] = *reinterpret_cast<const float4*>(st + aoff + cp);                             \
        fb[0] = *reinterpret_cast<const float4*>(st + boff + cp);                             \
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);                                    \
      }                                                                                       \
      if (qq + 1 < 4) {                                                                       \
        const int cn = ((4 * h + qq + 1) ^ swz) * 4;                                          \
        fa[(qq + 1) & 1] = *reinterpret_cast<const float4*>(st + aoff + cn);                  \
        fb[(qq + 1) & 1] = *reinterpret_cast<const float4*>(st + boff + cn);                  \
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);                                    \
      }                                                                                       \
      const float4 a = fa[qq & 1], b = fb[qq & 1];                                            \
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);                     \
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);                     \
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);                     \
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);                     \
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                      \
    }                                                                                         \
    if (PRIO) __builtin_amdgcn_s_setprio(0);                                                  \
  } while (0)
  const int nfull = nk / NS * NS;
  for (int kt0 = 0; kt0 < nfull; kt0 += NS) {
#pragma unroll
    for (int s = 0; s < NS; ++s) ADMMQ_STEP(s, kt0 + s);
  }
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (nfull + s < nk) ADMMQ_STEP(s, nfull + s);
#undef ADMMQ_STEP
#undef ADMMQ_ISSUE
  wait_vmcnt<0>();   // the refills past the end land before the workgroup ends
  const unsigned long long TK = ADMMQ_NOW();
  if (ser > 1) {     // serial K-split: the last piece
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = psum[r] + acc[r];
  }
  if (tl.np > 1) {   // K-split piece: only the piece that completes the tile goes on
    __shared__ int klast;
    const bool go = ksplit_combine(tl, acc, &klast);
    if (ADMMQ_TRACE && tid == 0 && blockIdx.x < kGemmTraceMax) {
      g_gemm_trace2[blockIdx.x][0] = TK;
      g_gemm_trace2[blockIdx.x][1] = ADMMQ_NOW();
      if (!go) {   // a piece that did not complete its tile: {start, end, info | 1 << 63}
        g_gemm_trace[blockIdx.x][0] = T0;
        g_gemm_trace[blockIdx.x][3] = __builtin_amdgcn_s_memtime() - C0;
        g_gemm_trace[blockIdx.x][1] = ADMMQ_NOW();
        g_gemm_trace[blockIdx.x][2] = (1ull << 63) | ((unsigned long long)blockIdx.x << 48) |
                                      ((unsigned long long)(nk & 0xFF) << 40) |
                                      ((unsigned long long)(__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xFF) << 32) |
                                      __builtin_amdgcn_s_getreg((31 << 11) | 4);
      }
    }
    if (!go) return;
  } else if (ADMMQ_TRACE && tid == 0 && blockIdx.x < kGemmTraceMax) {
    g_gemm_trace2[blockIdx.x][0] = TK;
    g_gemm_trace2[blockIdx.x][1] = TK;
  }
  if constexpr (!PRE) load_u();
  unsigned amax = 0u, mn = 0xFFFFFFFFu, mxo = 0u;
  typedef __attribute__((address_space(1))) float gf32;
  [[maybe_unused]] gf32* const HTg = (gf32*)p.HT;
  [[maybe_unused]] const __amdgpu_buffer_rsrc_t htrs = __builtin_amdgcn_make_buffer_rsrc(p.HT, 0, 0x7FFFFFFF, 0x00020000);
  gf32* const Xg = p.X_dbg ? (gf32*)p.X : nullptr;   // debug output only
  const int pI = p.I, pR = p.R;
  const int col = col0 + 32 * wn + i;
  if (col < ld) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = row0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
      const size_t off = (size_t)row * ld + col;
      const float ht = acc[r];
      const float x = ht - upre[r];
#if ADMMQ_SC1_STORES & 4
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ht), htrs, (int)(off * 4), 0, 16);
#elif ADMMQ_NT_STORES & 4
      __builtin_nontemporal_store(ht, HTg + off);
#else
      HTg[off] = ht;
#endif
      if (Xg) Xg[off] = x;
      if (row < pI && col < pR) {
        amax = max(amax, __float_as_uint(x) & 0x7FFFFFFFu);
        const unsigned e = enc_ord(x);
        mn = min(mn, e);
        mxo = max(mxo, e);
      }
    }
  }
  amax = wave_max_u32(amax); mn = wave_min_u32(mn); mxo = wave_max_u32(mxo);
  if (lane == 0) { red[0][wave] = amax; red[1][wave] = mn; red[2][wave] = mxo; }
  __syncthreads();
  if (tid == 0) {
    unsigned a0 = red[0][0], a1 = red[1][0], a2 = red[2][0];
#pragma unroll
    for (int w = 1; w < 4; ++w) { a0 = max(a0, red[0][w]); a1 = min(a1, red[1][w]); a2 = max(a2, red[2][w]); }
    unsigned* stt = p.mv.stat + 4 * slot;
    atomicMax(&stt[0], a0);
    atomicMin(&stt[1], a1);
    atomicMax(&stt[2], a2);
    if (ADMMQ_TRACE && blockIdx.x < kGemmTraceMax) {
      const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
      g_gemm_trace[blockIdx.x][0] = T0;
      g_gemm_trace[blockIdx.x][3] = __builtin_amdgcn_s_memtime() - C0;
      g_gemm_trace[blockIdx.x][1] = ADMMQ_NOW();
      g_gemm_trace[blockIdx.x][2] = ((unsigned long long)blockIdx.x << 48) | ((unsigned long long)(nk & 0xFF) << 40) |
                                    ((unsigned long long)(xcc & 0xFF) << 32) | hw;
    }
  }
}

// fp32 64 x 64 tiles: 0 = k_gemm<2, 1, 3, false>, 1 = k_gemm_f32b<3, true>, 2 = k_gemm_f32b<2, false>,
// 3 = k_gemm_f32b<3, false> (same bits)
int g_gemm_f32_stage = 3;

// One block per (problem, row): rows [0, Ip) of P (fp32, padded, zero pads) -> P2 / eP.
// `which` 0: P of every split problem; 1: M (rows [0, ldm)) -> M2 / eM.
__global__ __launch_bounds__(256) void k_split_rows(const ProbDesc* __restrict__ probs, int which) {
  const ProbDesc& p = probs[blockIdx.y];
  if (!p.split) return;
  const int nrows = which ? p.ldm : p.Ip;
  const int row = blockIdx.x;
  if (row >= nrows) return;
  const int n = which ? p.ldm : p.ld;
  const float* src = (which ? p.M : p.P) + (size_t)row * n;
  _Float16* dst = (which ? p.M2 : p.P2) + (size_t)row * 2 * n;
  float m = 0.f;
  for (int c = 4 * threadIdx.x; c < n; c += 1024) {
    const float4 v = *reinterpret_cast<const float4*>(src + c);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  m = __uint_as_float(wave_max_u32(__float_as_uint(m)));
  __shared__ unsigned wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = __float_as_uint(m);
  __syncthreads();
  const float amax = __uint_as_float(max(max(wm[0], wm[1]), max(wm[2], wm[3])));
  const int e = split_exponent(amax);
  for (int c = 4 * threadIdx.x; c < n; c += 1024) split_store4(dst, c, *reinterpret_cast<const float4*>(src + c), e);
  if (threadIdx.x == 0) (which ? p.eM : p.eP)[row] = e;
}

void launch_split_rows(const ProbDesc* d, int nprob, int maxrows, int which, hipStream_t s) {
  if (nprob > 0 && maxrows > 0) hipLaunchKernelGGL(k_split_rows, dim3(maxrows, nprob), dim3(256), 0, s, d, which);
}

// fp32 64 x 64 tiles: 1 = four waves of 32 x 32 (default), 2 = eight waves, each pair
// splitting a sub-tile's K-step (two half chains summed in fixed order: other bits)
int g_gemm_ks_f32 = 1;

void launch_gemm(const ProbDesc* d, const GemmTile* tiles, int ntiles_wide, int ntiles_small, int ntiles_big,
                 bool split, int slot, int iter, float eps, int ncand, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1,
                 bool prefetch_u) {
  // tiles[0 .. ntiles_wide) are 256x128 (WM = 8, CW = 2: sixteen waves of 32 x 64, the
  // launches with many rounds of tiles), then ntiles_big 64x64 tiles (WM = 2, four
  // waves, 3-deep ring), then ntiles_small 32x64 tiles (WM = 1: the 17..32-row factors,
  // 2 waves per sub-tile splitting each K-step, 4-deep ring).
  // ev0 / ev1 (profiling, may be null) are recorded by the dispatches themselves: ev0 at
  // the start of the first launch, ev1 at the end of the last
  const int nl = (ntiles_wide > 0) + (ntiles_big > 0) + (ntiles_small > 0);
  int li = 0;
  hipEvent_t a = nullptr, b = nullptr;
  auto evs = [&]() { a = li == 0 ? ev0 : nullptr; b = li == nl - 1 ? ev1 : nullptr; ++li; };
#define ADMMQ_LAUNCH(K, N, T, TILES) \
  hipExtLaunchKernelGGL(K, dim3(N), dim3(T), 0, s, a, b, 0u, d, TILES, slot, iter, eps, ncand)
  if (ntiles_wide > 0) {   // 256 x 128 tiles (WM = 8, CW = 2: 16 waves of 32 x 64), three-deep ring, one workgroup per CU
    evs();
    if (split) ADMMQ_LAUNCH((k_gemm<8, 1, 3, true, 2>), ntiles_wide, 1024, tiles);
    else ADMMQ_LAUNCH((k_gemm<8, 1, 3, false, 2>), ntiles_wide, 1024, tiles);
  }
  if (ntiles_big > 0) {
    evs();
    const GemmTile* t = tiles + ntiles_wide;
    if (split) ADMMQ_LAUNCH((k_gemm<2, 1, 3, true>), ntiles_big, 256, t);
    else if (g_gemm_ks_f32 == 2)   // 8 waves per 64 x 64 tile, each K-step split over two waves (A/B)
      ADMMQ_LAUNCH((k_gemm<2, 2, 3, false>), ntiles_big, 512, t);
    else if (g_gemm_f32_stage == 1) ADMMQ_LAUNCH((k_gemm_f32b<3, true>), ntiles_big, 256, t);
    else if (g_gemm_f32_stage == 2) ADMMQ_LAUNCH((k_gemm_f32b<2, false>), ntiles_big, 256, t);
    else if (g_gemm_f32_stage == 3 && prefetch_u)   // latency-bound launches (parallel K-split pieces): U before the K-loop
      ADMMQ_LAUNCH((k_gemm_f32b<3, true>), ntiles_big, 256, t);
    else if (g_gemm_f32_stage == 3) ADMMQ_LAUNCH((k_gemm_f32b<3, false>), ntiles_big, 256, t);
    else if (g_gemm_f32_stage == 4) ADMMQ_LAUNCH((k_gemm_f32b<3, false, true>), ntiles_big, 256, t);
    else ADMMQ_LAUNCH((k_gemm<2, 1, 3, false>), ntiles_big, 256, t);
  }
  if (ntiles_small > 0) {
    evs();
    const GemmTile* t = tiles + ntiles_wide + ntiles_big;
    if (split) ADMMQ_LAUNCH((k_gemm<1, 2, 4, true>), ntiles_small, 256, t);
    else ADMMQ_LAUNCH((k_gemm<1, 2, 4, false>), ntiles_small, 256, t);
  }
#undef ADMMQ_LAUNCH
}


}  // namespace admmq

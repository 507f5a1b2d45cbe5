// Device-side quantizer arithmetic shared by the ADMM projection (admm_kernels.hip)
// and standalone quantize_tensor (quant_kernels.hip).
//
// Every operation below is a float32 IEEE operation in the same order as the
// reference's torch-CPU code (source/quantization.py), compiled with
// -ffp-contract=off so no multiply/add pair is fused behind our back.
#pragma once

// Store policy of the per-iteration outputs (same bits under every policy; C3 / C4 per step,
// interleaved runs, profiles/r06_nt_stores_ab.json and r06_store_policy_ab.json):
// ADMMQ_SC1_STORES (default 7): write-through (sc1) stores - bit 0 H / U of the fused
// finalize, bit 1 its next P, bit 2 H_T of the fp32 solve GEMM's epilogue. Every one of them
// is read by the next launch; written through, its lines reach the MALL as they are stored,
// so a kernel's end has no dirty L2 lines to write back (on MI355X the eight XCD L2s are
// written back at every kernel's release), while they stay valid in the writing XCD's L2.
// C3 192.6 -> 187.8 ms (GEMM 49.0 -> 47.9 us, search 30.5 -> 29.0), C4 241.0 -> 239.9 ms.
// ADMMQ_NT_STORES (bits as above; used where SC1 is off): nontemporal stores, which skip L2
// instead - 193.7 -> 192.0 ms at C3 for H_T + H / U, but the C4 search lost 4.7 us with H / U
// streamed (its finalize re-reads U, H, F), so H / U stream only in the two-group form.
#ifndef ADMMQ_NT_STORES
#define ADMMQ_NT_STORES 5
#endif
#ifndef ADMMQ_SC1_STORES
#define ADMMQ_SC1_STORES 7
#endif
#include "admmq_internal.h"

namespace admmq {

// torch.linspace(0.2*mx.item(), 1.2*mx.item(), n)[c]   (source/quantization.py:130)
// Pinned by tests/golden/f5_linspace.npz: fma(step, c, start) below n/2,
// fma(-step, n-1-c, end) above.
__device__ __forceinline__ float cand_t(float mx, int c, int n) {
  const float S = (float)(0.2 * (double)mx);
  const float E = (float)(1.2 * (double)mx);
  if (n == 1) return S;
  const float step = (E - S) / (float)(n - 1);
  if (c < (n >> 1)) return __builtin_fmaf(step, (float)c, S);
  return __builtin_fmaf(-step, (float)(n - 1 - c), E);
}

__device__ __forceinline__ bool mse_degenerate(float mx) { return !(mx > 0.f && mx < __builtin_inff()); }

// Fixed-point exponent of the canonical SSE rule (oracle/quant_oracle.py):
// K = 56 - ceil_log2(nquads) - 2*E, mx = m*2^E with m in [0.5,1).
__device__ __forceinline__ int fixed_exp(float mx, int nq) {
  int e;
  (void)__builtin_frexpf(mx, &e);
  const int cl = (nq > 1) ? (32 - __builtin_clz((unsigned)(nq - 1))) : 0;
  return 56 - cl - 2 * e;
}

// floor(g * 2^K) as uint64, exact (g >= 0 float32; the planner guarantees < 2^63).
__device__ __forceinline__ unsigned long long to_fixed(float g, int K) {
  const float v = __builtin_ldexpf(g, K);
  const float vh = v * 0x1p-32f;
  const unsigned hi = __float2uint_rz(vh);
  const float r = v - (float)hi * 0x1p32f;           // exact: representable remainder
  const unsigned lo = __float2uint_rz(r);
  return ((unsigned long long)hi << 32) + (unsigned long long)lo;
}

struct QParams {
  int scheme;
  int bits;
  float scale;
  float qlo, qhi;
  int zp;
  float mn, rng, n;
  int nan_all;
  float rcp;    // MSE: 1 / scale (IEEE), for apply_quant_mse's reciprocal fast path
  int fast;     // MSE: the fast path is valid (scale and 1 / scale normal and finite)
};

__device__ __forceinline__ float nan_clamp(float q, float lo, float hi) {
  // torch.clamp propagates NaN; fmin/fmax would not.
  return (q != q) ? q : __builtin_fminf(__builtin_fmaxf(q, lo), hi);
}

// int64 conversion of a float the way x86 torch-CPU does it (`.to(int)`): NaN /
// out-of-range -> INT64_MIN.
__device__ __forceinline__ long long to_i64_x86(float v) {
  if (!(v == v) || v >= 9.2233720368547758e18f || v < -9.2233720368547758e18f) return (long long)0x8000000000000000ull;
  return (long long)v;
}
__device__ __forceinline__ int to_i32_x86(float v) {
  if (!(v == v) || v >= 2147483648.0f || v < -2147483648.0f) return (int)0x80000000u;
  return (int)v;
}

// Parameters of the non-MSE schemes from tensor min/max (source/quantization.py:48-66, 91-106).
__device__ __forceinline__ QParams qparams_stats(int scheme, int bits, float tmin, float tmax, int has_nan,
                                                 int has_kw, float kw_min, float kw_max) {
  QParams p;
  p.scheme = scheme;
  p.bits = bits;
  p.nan_all = 0;
  p.scale = 0.f; p.zp = 0; p.mn = 0.f; p.rng = 0.f; p.n = 0.f;
  const int q = 1 << (bits - 1);
  p.qlo = (float)(-q);
  p.qhi = (float)(q - 1);
  const float den = (float)(2 * q - 1);
  if (has_nan) { tmin = __builtin_nanf(""); tmax = __builtin_nanf(""); }
  if (scheme == kSymmetric) {
    const float am = __builtin_fabsf(tmin);
    const float m = (am > tmax) ? am : tmax;
    p.scale = (2.0f * m) / den;
  } else if (scheme == kAffine) {
    if (has_kw) { tmin = kw_min; tmax = kw_max; }
    p.scale = (tmax - tmin) / den;
    const int t = to_i32_x86(tmin / p.scale);
    int zp = (int)((unsigned)(-q) - (unsigned)t);   // int32 wrap like torch
    zp = zp < -q ? -q : (zp > q - 1 ? q - 1 : zp);
    p.zp = zp;
  } else {  // kMinMax
    p.mn = tmin;
    p.rng = tmax - tmin;
    p.n = (float)((1 << bits) - 1);
  }
  return p;
}

__device__ __forceinline__ QParams qparams_mse(int bits, float t) {
  QParams p;
  p.scheme = kMse;
  p.bits = bits;
  const int q = 1 << (bits - 1);
  p.qlo = (float)(-q);
  p.qhi = (float)(q - 1);
  p.scale = (2.0f * t) / (float)(2 * q - 1);
  p.nan_all = (t == t) ? 0 : 1;
  p.zp = 0; p.mn = 0.f; p.rng = 0.f; p.n = 0.f;
  p.rcp = 1.0f / p.scale;
  const float as = __builtin_fabsf(p.scale), ar = __builtin_fabsf(p.rcp);
  p.fast = (as >= 0x1p-126f && as < __builtin_inff() && ar >= 0x1p-126f && ar < __builtin_inff()) ? 1 : 0;
  return p;
}

__device__ __forceinline__ float apply_quant(float x, const QParams& p) {
  if (p.scheme == kMse) {
    if (p.nan_all) return __builtin_nanf("");
    const float q = nan_clamp(__builtin_rintf(x / p.scale), p.qlo, p.qhi);
    return q * p.scale;
  }
  if (p.scheme == kSymmetric) {
    const float q = nan_clamp(__builtin_rintf(x / p.scale), p.qlo, p.qhi);
    return (float)to_i64_x86(q) * p.scale;
  }
  if (p.scheme == kAffine) {
    const float lv = nan_clamp(__builtin_rintf(x / p.scale) + (float)p.zp, p.qlo, p.qhi);
    const long long li = to_i64_x86(lv);
    const long long d = (long long)((unsigned long long)li - (unsigned long long)(long long)p.zp);
    return (float)d * p.scale;
  }
  // kMinMax (source/quantization.py:48-66)
  if (p.bits == 1) {
    const float sg = (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : ((x == x) ? 0.f : x));
    return sg - 1.f;
  }
  const float r = (x - p.mn) / p.rng;
  const float qi = __builtin_floorf(r * p.n + 0.5f);
  return (qi * p.rng) / p.n + p.mn;
}

// The MSE projection clamp(rint(fl(x / s)), qlo, qhi) * s with the quotient from the
// reciprocal: y = x * (1 / s) is within |y| 2^-23 of x / s (two roundings), so rint(y)
// is rint(fl(x / s)) unless y lies within |y| 2^-21 of a half-integer - then the IEEE
// quotient decides (rare). NaN / inf inputs take the same values either way; a
// non-normal scale or reciprocal (p.fast == 0) always divides. Same bits as
// apply_quant (GPU parity tests).
__device__ __forceinline__ float apply_quant_mse(float x, const QParams& p) {
  if (p.nan_all) return __builtin_nanf("");
  const float y = x * p.rcp;
  float q = __builtin_rintf(y);
  if (!p.fast || __builtin_fabsf(__builtin_fabsf(y - q) - 0.5f) < __builtin_fabsf(y) * 0x1p-21f)
    q = __builtin_rintf(x / p.scale);
  return nan_clamp(q, p.qlo, p.qhi) * p.scale;
}

// First-index argmin of sse[0..n) by ONE wave (all 64 lanes must call).
__device__ __forceinline__ int wave_argmin_u64(const unsigned long long* sse, int n) {
  const int lane = threadIdx.x & 63;
  unsigned long long best = ~0ull;
  int bi = 0x7fffffff;
  for (int c = lane; c < n; c += 64) {
    const unsigned long long v = sse[c];
    if (v < best) { best = v; bi = c; }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long ov = __shfl_xor(best, off);
    const int oi = __shfl_xor(bi, off);
    if (ov < best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  return bi;
}

// ---------------------------------------------------------------------------
// Canonical SSE of a candidate list over one chunk of quads held in LDS (stage 2 of
// the search, or the exhaustive sweep when list == nullptr: candidates 0..nc-1).
// Lane -> candidate mapping per 64-candidate group g: cnt = min(64, nc-64g)
// candidates over p2 = pow2ceil(cnt) lanes and S = 64/p2 interleaved quad streams;
// when there are fewer groups than waves, the waves of a group split the quads too.
// Each lane accumulates the canonical fixed-point SSE; streams fold with xor-shuffles
// and stream 0 adds into sse[candidate] atomically (integer adds: order-free).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void sse_group(const float4* __restrict__ xs, int nqc, float mx, int K, int ncand,
                                          int bits, const int* list, int nc, int g, int wsub, int wpg,
                                          unsigned long long* __restrict__ sse) {
  const int lane = threadIdx.x & 63;
  const int q = 1 << (bits - 1);
  const float qlo = (float)(-q), qhi = (float)(q - 1);
  const float den = (float)(2 * q - 1);
  // near-half-integer window for the reciprocal fast path: > 3 ulp of |y| <= q+1
  const float delta = (float)(q + 1) * 0x1p-21f;
  const int cnt = min(64, nc - 64 * g);
  int lg = 0;
  while ((1 << lg) < cnt) ++lg;
  const int p2 = 1 << lg;
  const int S = 64 >> lg;
  const int csub = lane & (p2 - 1);
  const int stream = lane >> lg;
  const bool active = csub < cnt;
  const int j = 64 * g + (active ? csub : 0);
  const int c = list ? list[j] : j;
  const float t = cand_t(mx, c, ncand);
  const float s = (2.0f * t) / den;
  const float rcp = 1.0f / s;
  unsigned long long acc = 0;
  for (int k = wsub * S + stream; k < nqc; k += wpg * S) {
    const float4 v = xs[k];
    const float y0 = v.x * rcp, y1 = v.y * rcp, y2 = v.z * rcp, y3 = v.w * rcp;
    float q0 = __builtin_rintf(y0), q1 = __builtin_rintf(y1), q2 = __builtin_rintf(y2), q3 = __builtin_rintf(y3);
    // distance of each y to the nearest half-integer; one compare per quad
    const float e0 = __builtin_fabsf(__builtin_fabsf(y0 - q0) - 0.5f);
    const float e1 = __builtin_fabsf(__builtin_fabsf(y1 - q1) - 0.5f);
    const float e2 = __builtin_fabsf(__builtin_fabsf(y2 - q2) - 0.5f);
    const float e3 = __builtin_fabsf(__builtin_fabsf(y3 - q3) - 0.5f);
    const bool nb = __builtin_fminf(__builtin_fminf(e0, e1), __builtin_fminf(e2, e3)) < delta;
    if (__builtin_expect(nb, 0)) {   // rare: decide the rounding with the exact IEEE quotient
      q0 = __builtin_rintf(v.x / s); q1 = __builtin_rintf(v.y / s);
      q2 = __builtin_rintf(v.z / s); q3 = __builtin_rintf(v.w / s);
    }
    q0 = __builtin_amdgcn_fmed3f(q0, qlo, qhi);
    q1 = __builtin_amdgcn_fmed3f(q1, qlo, qhi);
    q2 = __builtin_amdgcn_fmed3f(q2, qlo, qhi);
    q3 = __builtin_amdgcn_fmed3f(q3, qlo, qhi);
    const float d0 = v.x - q0 * s, d1 = v.y - q1 * s, d2 = v.z - q2 * s, d3 = v.w - q3 * s;
    const float gq = (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    acc += to_fixed(gq, K);
  }
  for (int off = p2; off < 64; off <<= 1) acc += __shfl_xor(acc, off);
  if (active && stream == 0) atomicAdd(&sse[c], acc);
}

__device__ __forceinline__ void sse_sweep_list(const float4* __restrict__ xs, int nqc, float mx, int K, int ncand,
                                               int bits, const int* list, int nc, unsigned long long* __restrict__ sse) {
  const int wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const int ngroups = (nc + 63) >> 6;
  if (ngroups >= nwaves) {
    for (int g = wave; g < ngroups; g += nwaves) sse_group(xs, nqc, mx, K, ncand, bits, list, nc, g, 0, 1, sse);
  } else {
    const int wpg = nwaves / ngroups;
    if (wave < wpg * ngroups) sse_group(xs, nqc, mx, K, ncand, bits, list, nc, wave % ngroups, wave / ngroups, wpg, sse);
  }
}

// Wave reductions and scans on DPP (row_shr / row_shl 1, 2, 4, 8 inside each 16-lane row,
// then the four row results read as scalars): no LDS permutes (ds_bpermute), whose
// waits would chain. Fixed order, so the results are deterministic.
// dpp_zero: the neighbour's value, 0 where it lies outside the row (sums);
// dpp_keep: ... the lane's own value there (max / min).
template <int CTRL>
__device__ __forceinline__ unsigned dpp_zero(unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ unsigned dpp_keep(unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ unsigned readlane_u32(unsigned v, int l) { return (unsigned)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ unsigned long long u64_of(unsigned lo, unsigned hi) {
  return ((unsigned long long)hi << 32) | lo;
}
template <int CTRL>
__device__ __forceinline__ unsigned long long dpp_zero_u64(unsigned long long v) {
  return u64_of(dpp_zero<CTRL>((unsigned)v), dpp_zero<CTRL>((unsigned)(v >> 32)));
}
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
  return u64_of(readlane_u32((unsigned)v, l), readlane_u32((unsigned)(v >> 32), l));
}
template <int CTRL>
__device__ __forceinline__ double dpp_zero_f64(double v) {   // out of row: +0.0
  return __longlong_as_double((long long)dpp_zero_u64<CTRL>((unsigned long long)__double_as_longlong(v)));
}
template <int CTRL>
__device__ __forceinline__ double dpp_keep_f64(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  return __longlong_as_double((long long)u64_of(dpp_keep<CTRL>((unsigned)b), dpp_keep<CTRL>((unsigned)(b >> 32))));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  return __longlong_as_double((long long)readlane_u64((unsigned long long)__double_as_longlong(v), l));
}
// results are wave-uniform
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
  v = max(v, dpp_keep<0x111>(v));
  v = max(v, dpp_keep<0x112>(v));
  v = max(v, dpp_keep<0x114>(v));
  v = max(v, dpp_keep<0x118>(v));
  return max(max(readlane_u32(v, 15), readlane_u32(v, 31)), max(readlane_u32(v, 47), readlane_u32(v, 63)));
}
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
  v = min(v, dpp_keep<0x111>(v));
  v = min(v, dpp_keep<0x112>(v));
  v = min(v, dpp_keep<0x114>(v));
  v = min(v, dpp_keep<0x118>(v));
  return min(min(readlane_u32(v, 15), readlane_u32(v, 31)), min(readlane_u32(v, 47), readlane_u32(v, 63)));
}
__device__ __forceinline__ double wave_min_f64(double v) {
  v = fmin(v, dpp_keep_f64<0x111>(v));
  v = fmin(v, dpp_keep_f64<0x112>(v));
  v = fmin(v, dpp_keep_f64<0x114>(v));
  v = fmin(v, dpp_keep_f64<0x118>(v));
  return fmin(fmin(readlane_f64(v, 15), readlane_f64(v, 31)), fmin(readlane_f64(v, 47), readlane_f64(v, 63)));
}
__device__ __forceinline__ double wave_sum_f64(double v) {
  v += dpp_zero_f64<0x111>(v);
  v += dpp_zero_f64<0x112>(v);
  v += dpp_zero_f64<0x114>(v);
  v += dpp_zero_f64<0x118>(v);
  return (readlane_f64(v, 15) + readlane_f64(v, 31)) + (readlane_f64(v, 47) + readlane_f64(v, 63));
}
// inclusive suffix sums over the wave (lane l: sum over lanes >= l), row_shl steps
__device__ __forceinline__ unsigned long long wave_suffix_u64(unsigned long long v) {
  v += dpp_zero_u64<0x101>(v);
  v += dpp_zero_u64<0x102>(v);
  v += dpp_zero_u64<0x104>(v);
  v += dpp_zero_u64<0x108>(v);
  const unsigned long long t1 = readlane_u64(v, 16), t2 = readlane_u64(v, 32), t3 = readlane_u64(v, 48);
  const int row = (threadIdx.x & 63) >> 4;
  return v + (row < 1 ? t1 : 0ull) + (row < 2 ? t2 : 0ull) + (row < 3 ? t3 : 0ull);
}
__device__ __forceinline__ unsigned wave_suffix_u32(unsigned v) {
  v += dpp_zero<0x101>(v);
  v += dpp_zero<0x102>(v);
  v += dpp_zero<0x104>(v);
  v += dpp_zero<0x108>(v);
  const unsigned t1 = readlane_u32(v, 16), t2 = readlane_u32(v, 32), t3 = readlane_u32(v, 48);
  const int row = (threadIdx.x & 63) >> 4;
  return v + (row < 1 ? t1 : 0u) + (row < 2 ? t2 : 0u) + (row < 3 ? t3 : 0u);
}

// Resolve the quantization parameters of a job inside a block (all threads call).
// MSE: the select record gives c* directly (|S| = 1), or the canonical SSE of the
// list / of every candidate decides (first index on ties, like torch.argmin).
__device__ __forceinline__ QParams block_qparams(int scheme, int bits, const MseView& v, int slot, int ncand,
                                                 int has_kw, float kw_min, float kw_max) {
  __shared__ int s_idx;
  const unsigned* stat = v.stat + 4 * slot;
  const unsigned ab = stat[0];
  const bool has_nan = ab > 0x7F800000u;
  if (scheme == kMse) {
    const float mx = __uint_as_float(ab);
    if (mse_degenerate(mx)) return qparams_mse(bits, __builtin_nanf(""));
    const int* sel = v.sel + (size_t)slot * (2 + kMaxSel);
    const unsigned long long* sse = v.sse + (size_t)slot * ncand;
    if (threadIdx.x < 64) {
      const int ns = sel[0];
      int idx;
      if (ns == 1) {
        idx = sel[2];
      } else if (ns >= ncand) {
        idx = wave_argmin_u64(sse, ncand);
      } else {
        const int lane = threadIdx.x & 63;
        unsigned long long best = ~0ull;
        int bi = 0x7fffffff;
        for (int j = lane; j < ns; j += 64) {
          const int c = sel[2 + j];
          const unsigned long long x = sse[c];
          if (x < best || (x == best && c < bi)) { best = x; bi = c; }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          const unsigned long long ov = __shfl_xor(best, off);
          const int oi = __shfl_xor(bi, off);
          if (ov < best || (ov == best && oi < bi)) { best = ov; bi = oi; }
        }
        idx = bi;
      }
      if (threadIdx.x == 0) s_idx = idx;
    }
    __syncthreads();
    return qparams_mse(bits, cand_t(mx, s_idx, ncand));
  }
  return qparams_stats(scheme, bits, dec_ord(stat[1]), dec_ord(stat[2]), has_nan ? 1 : 0, has_kw, kw_min, kw_max);
}

// ---------------------------------------------------------------------------
// Split operand planes (kSolveSplit). A row of n values (n a multiple of 32) becomes
// n/32 blocks of [32 hi halfs][32 lo halfs] (the fp32 row's bytes) with the row's
// exponent e = 14 - floor(log2 max|x|) (max|x| 2^e in [2^14, 2^15): no fp16 overflow):
//   hi = fp16(x 2^e), lo = fp16(x 2^e - hi)   (x 2^e and the difference are exact in fp32)
__device__ __forceinline__ int split_exponent(float amax) {
  if (!(amax > 0.f) || !(amax < __builtin_inff())) return 0;
  int e;
  (void)__builtin_frexpf(amax, &e);   // amax = m 2^e, m in [0.5, 1): floor(log2 amax) = e - 1
  return 15 - e;
}
__device__ __forceinline__ void split_store4(_Float16* dst_row, int col, float4 v, int e) {
  const float s[4] = {__builtin_ldexpf(v.x, e), __builtin_ldexpf(v.y, e), __builtin_ldexpf(v.z, e),
                      __builtin_ldexpf(v.w, e)};
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  h4 hi, lo;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    hi[k] = (_Float16)s[k];
    lo[k] = (_Float16)(s[k] - (float)hi[k]);
  }
  _Float16* b = dst_row + (col >> 5) * 64 + (col & 31);
  *reinterpret_cast<h4*>(b) = hi;
  *reinterpret_cast<h4*>(b + 32) = lo;
}

// ---------------------------------------------------------------------------
// ADMM finalize of one unit of whole rows [start, end) of problem p (source/admm.py:58-63):
// H = Q(X) with X = H_T - U re-formed here, U += H - H_T, the next right-hand side
// P = F + rho (H + U) (split form: fp16 planes with the row's exponent), and the
// residual sums of the r / s stop test into replica `rep`. The float4 group g of thread
// t is element start + 4 t + 4 NT g; t4 = H_T, u4 = U, h4 = H (current), f4 = F.
// rmax: LDS of >= the unit's rows. Every thread of the block calls it. Used by
// k_finalize_admm and by the search kernel's fused finalize (k_mse_hist3<.., true>).
// The descriptor fields are read once into registers (the stores below would otherwise
// force their reloads: they go through pointers that may alias the descriptor), element
// offsets are 32-bit (a problem holds < 2^31 elements: plan_admm), stores are global.
// STREAM: every input is already in registers (the fused search's finalize): each group is
// stored as soon as it is computed (no arrays of results live across the groups: the fused
// search kernel spilled 62 VGPRs holding them); the split form then re-reads its fp32 P for
// the planes after the row-max barrier. Same float32 / fp64 operations in the same order.
template <int NT, int NG, bool STREAM = false>
__device__ __forceinline__ void admm_finalize_block(const ProbDesc& p, long long start, long long end,
                                                    const float4* t4, const float4* u4, const float4* h4,
                                                    const float4* f4, const QParams& qp, int slot, int iter, int rep,
                                                    unsigned* rmax, unsigned long long* trace = nullptr) {
  // diagnostics (make TRACE=1): stamps {rho read, elements stored, row max, split stores,
  // the block's loads complete (before the elements; trace builds wait for them there)}
#define ADMMQ_FIN_STAMP(k) \
  if (ADMMQ_TRACE && trace && threadIdx.x == 0) trace[k] = ADMMQ_NOW()
  typedef __attribute__((address_space(1))) gf32x4 gst4;
  __shared__ double red[NT / 64][4];
  float* const Hd = p.H;
  float* const Ud = p.U;
  float* const Pd = p.P;
  _Float16* const P2 = p.P2;
  int* const eP = p.eP;
  double* const res = p.res;
  const int ld = p.ld, R = p.R;
  const bool split = p.split != 0;
  const bool mse = qp.scheme == kMse;
  const float rho = p.rho[0];
  ADMMQ_FIN_STAMP(0);
  const int s32 = (int)start, e32 = (int)end;
  const int row0 = s32 / ld;
  if (split) {
    const int nrows = (e32 - s32 + ld - 1) / ld;
    for (int r = threadIdx.x; r < nrows; r += NT) rmax[r] = 0u;
    __syncthreads();
  }
  if (ADMMQ_TRACE && trace) {
    __builtin_amdgcn_s_waitcnt(0);
    ADMMQ_FIN_STAMP(4);
  }
  double s1 = 0.0, s2 = 0.0, s3 = 0.0, s4 = 0.0;
  const int lane = threadIdx.x & 63;
  if constexpr (STREAM) {
    typedef unsigned sc1u4 __attribute__((ext_vector_type(4)));
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(Hd, 0, 0x7FFFFFFF, 0x00020000);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t urs = __builtin_amdgcn_make_buffer_rsrc(Ud, 0, 0x7FFFFFFF, 0x00020000);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(Pd, 0, 0x7FFFFFFF, 0x00020000);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the inputs are complete: stores below wait for nothing
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int e = s32 + 4 * (int)threadIdx.x + 4 * NT * g;
      const bool in = e < e32;
      const int row = e / ld;
      float4 pv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (in) {
        const int c0 = e - row * ld;
        const float ts[4] = {t4[g].x, t4[g].y, t4[g].z, t4[g].w};
        const float hs[4] = {h4[g].x, h4[g].y, h4[g].z, h4[g].w}, us[4] = {u4[g].x, u4[g].y, u4[g].z, u4[g].w};
        const float xs[4] = {ts[0] - us[0], ts[1] - us[1], ts[2] - us[2], ts[3] - us[3]};   // H_T - U
        const float fs[4] = {f4[g].x, f4[g].y, f4[g].z, f4[g].w};
        float a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
        gf32x4 hv, uv;
        float po[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool ok = c0 + k < R;
          const float hq = mse ? apply_quant_mse(xs[k], qp) : apply_quant(xs[k], qp);
          const float hn = ok ? hq : 0.f;
          const float dh = ok ? hn - ts[k] : 0.f;
          const float un = ok ? us[k] + dh : 0.f;
          hv[k] = hn; uv[k] = un;
          po[k] = ok ? fs[k] + rho * (hn + un) : 0.f;
          const float dp = ok ? hn - hs[k] : 0.f;
          a1 += dh * dh; a2 += hn * hn; a3 += dp * dp; a4 += un * un;
        }
        s1 += (double)a1; s2 += (double)a2; s3 += (double)a3; s4 += (double)a4;
        pv = make_float4(po[0], po[1], po[2], po[3]);
        if constexpr ((ADMMQ_SC1_STORES & 1) != 0) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sc1u4, hv), hrs, e * 4, 0, 16);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sc1u4, uv), urs, e * 4, 0, 16);
        } else if constexpr ((ADMMQ_NT_STORES & 1) != 0 && NG <= 4) {   // (see ADMMQ_NT_STORES)
          __builtin_nontemporal_store(hv, (gst4*)(Hd + e));
          __builtin_nontemporal_store(uv, (gst4*)(Ud + e));
        } else {
          *(gst4*)(Hd + e) = hv;
          *(gst4*)(Ud + e) = uv;
        }
#if ADMMQ_SC1_STORES & 2
        if (!split) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sc1u4, gf32x4{pv.x, pv.y, pv.z, pv.w}), prs, e * 4, 0, 16);
        else
#elif ADMMQ_NT_STORES & 2
        if (!split) __builtin_nontemporal_store(gf32x4{pv.x, pv.y, pv.z, pv.w}, (gst4*)(Pd + e));
        else
#endif
        *(gst4*)(Pd + e) = gf32x4{pv.x, pv.y, pv.z, pv.w};   // (split: the planes are formed from it below)
      }
      if (split) {   // row max of |next P| per (wave, row), as the non-streaming form
        const int rg = in ? row : -1;
        const unsigned mv = in ? __float_as_uint(fmaxf(fmaxf(fabsf(pv.x), fabsf(pv.y)), fmaxf(fabsf(pv.z), fabsf(pv.w))))
                               : 0u;
        int r = __builtin_amdgcn_readfirstlane(rg);
        if (r >= 0) {
          for (;;) {
            const unsigned m = wave_max_u32(rg == r ? mv : 0u);
            if (lane == 0) atomicMax(&rmax[r - row0], m);
            if (__ballot(rg > r) == 0ull) break;
            ++r;
          }
        }
      }
    }
    ADMMQ_FIN_STAMP(1);
    if (split) {
      __syncthreads();
      ADMMQ_FIN_STAMP(2);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int e = s32 + 4 * (int)threadIdx.x + 4 * NT * g;
        if (e >= e32) continue;
        const int row = e / ld;
        const int c0 = e - row * ld;
        const float4 pv = *reinterpret_cast<const float4*>(Pd + e);   // this thread's own store
        const int ex = split_exponent(__uint_as_float(rmax[row - row0]));
        split_store4(P2 + (size_t)row * 2 * ld, c0, pv, ex);
        if (c0 == 0) eP[row] = ex;
      }
    }
  } else {
  float4 p4[NG];
  int rows[NG];
  gf32x4 ho[NG], uo[NG];
  // every group's arithmetic first, then every store: a store issued between two groups
  // would be waited for (vmcnt) by the next group's first register read the compiler
  // cannot prove complete
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int e = s32 + 4 * (int)threadIdx.x + 4 * NT * g;
    p4[g] = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool in = e < e32;
    const int row = e / ld;
    rows[g] = in ? row : -1;
    if (in) {
      const int c0 = e - row * ld;
      const float ts[4] = {t4[g].x, t4[g].y, t4[g].z, t4[g].w};
      const float hs[4] = {h4[g].x, h4[g].y, h4[g].z, h4[g].w}, us[4] = {u4[g].x, u4[g].y, u4[g].z, u4[g].w};
      const float xs[4] = {ts[0] - us[0], ts[1] - us[1], ts[2] - us[2], ts[3] - us[3]};   // H_T - U
      const float fs[4] = {f4[g].x, f4[g].y, f4[g].z, f4[g].w};
      float a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;   // the group's residual terms (fp32, in order)
      float po[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = c0 + k < R;   // select, not a branch (the pads stay exactly 0)
        const float hq = mse ? apply_quant_mse(xs[k], qp) : apply_quant(xs[k], qp);   // H = quantize(H_T - U)
        const float hn = ok ? hq : 0.f;
        const float dh = ok ? hn - ts[k] : 0.f;
        const float un = ok ? us[k] + dh : 0.f;              // U += H - H_T
        ho[g][k] = hn; uo[g][k] = un;
        po[k] = ok ? fs[k] + rho * (hn + un) : 0.f;          // next rhs F + rho(H+U)
        const float dp = ok ? hn - hs[k] : 0.f;
        a1 += dh * dh; a2 += hn * hn; a3 += dp * dp; a4 += un * un;
      }
      s1 += (double)a1; s2 += (double)a2; s3 += (double)a3; s4 += (double)a4;
      p4[g] = make_float4(po[0], po[1], po[2], po[3]);
    }
  }
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if (rows[g] < 0) continue;
    const int e = s32 + 4 * (int)threadIdx.x + 4 * NT * g;
    *(gst4*)(Hd + e) = ho[g];
    *(gst4*)(Ud + e) = uo[g];
    if (!split) *(gst4*)(Pd + e) = gf32x4{p4[g].x, p4[g].y, p4[g].z, p4[g].w};
  }
  if (split) {   // row max of |next P| per (wave, row): rows are contiguous lane ranges
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const unsigned mv = rows[g] >= 0 ? __float_as_uint(fmaxf(fmaxf(fabsf(p4[g].x), fabsf(p4[g].y)),
                                                               fmaxf(fabsf(p4[g].z), fabsf(p4[g].w))))
                                       : 0u;
      int r = __builtin_amdgcn_readfirstlane(rows[g]);   // lane 0 is in whenever any lane is
      if (r < 0) continue;
      for (;;) {
        const unsigned m = wave_max_u32(rows[g] == r ? mv : 0u);
        if (lane == 0) atomicMax(&rmax[r - row0], m);
        if (__ballot(rows[g] > r) == 0ull) break;
        ++r;
      }
    }
  }
  ADMMQ_FIN_STAMP(1);
  if (split) {
    __syncthreads();
    ADMMQ_FIN_STAMP(2);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (rows[g] < 0) continue;
      const int e = s32 + 4 * (int)threadIdx.x + 4 * NT * g;
      const int row = rows[g];
      const int c0 = e - row * ld;
      const int ex = split_exponent(__uint_as_float(rmax[row - row0]));
      split_store4(P2 + (size_t)row * 2 * ld, c0, p4[g], ex);
      if (c0 == 0) eP[row] = ex;
    }
  }
  }   // (non-streaming form)
  ADMMQ_FIN_STAMP(3);
#undef ADMMQ_FIN_STAMP
  s1 = wave_sum_f64(s1); s2 = wave_sum_f64(s2);
  s3 = wave_sum_f64(s3); s4 = wave_sum_f64(s4);
  const int w = threadIdx.x >> 6;
  if (lane == 0) { red[w][0] = s1; red[w][1] = s2; red[w][2] = s3; red[w][3] = s4; }
  __syncthreads();
  if (threadIdx.x < 4) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) v += red[k][threadIdx.x];
    atomicAdd(&res[4 * (kResRep * slot + rep) + threadIdx.x], v);
  }
  if (start == 0 && threadIdx.x == 0) {
    p.flags[1] = iter + 1;
    unsigned* st = p.mv.stat + 4 * (slot ^ 1);
    st[0] = 0u; st[1] = 0xFFFFFFFFu; st[2] = 0u; st[3] = 0u;
    double* rs = res + 4 * kResRep * (slot ^ 1);
    for (int k = 0; k < 4 * kResRep; ++k) rs[k] = 0.0;
  }
}

}  // namespace admmq

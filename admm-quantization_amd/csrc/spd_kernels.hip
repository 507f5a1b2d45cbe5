// M = (G + rho I)^-1 once per admm_iteration call (replaces torch.linalg.cholesky +
// torch.cholesky_solve of source/admm.py:54,56 by an explicit inverse so that every
// inner iteration is one GEMM). Computed in fp64 and rounded once to fp32.
//
// 32 x 32 blocked, batched over problems, fp64 VALU:
//   for k:  k_chol_panel(k)   factor A_kk in LDS (-> D64); L_ik = A_ik L_kk^-T (i > k)
//           k_chol_update(k)  A_ij -= L_ik L_jk^T                       (k < j <= i)
//   for i:  k_linv_row(i)     Linv_ij = -Linv_ii sum_{t=j}^{i-1} L_it Linv_tj
//   once:   k_minv            M_ij = sum_{t>=i} Linv_ti^T Linv_tj  (fp32, symmetric,
//                              zero outside R x R)
// A non-positive pivot sets flags[2] (the reference raises torch.linalg.LinAlgError).
#include "admmq_internal.h"

namespace admmq {

constexpr int NB = 32;
constexpr int LS = NB + 1;  // LDS row stride (doubles) to spread banks

__device__ __forceinline__ void load_regs(double r[4], const double* A, int ldm, int bi, int bj);
__device__ __forceinline__ void store_regs(double* dst, const double r[4]);
// blocks of 256 threads: all four loads of a thread issue before the first LDS store
__device__ __forceinline__ void load_block(double* dst, const double* A, int ldm, int bi, int bj) {
  double r[4];
  load_regs(r, A, ldm, bi, bj);
  store_regs(dst, r);
}
__device__ __forceinline__ void store_block(double* A, int ldm, int bi, int bj, const double* src) {
  for (int t = threadIdx.x; t < NB * NB; t += blockDim.x) {
    const int r = t >> 5, c = t & 31;
    A[(size_t)(bi * NB + r) * ldm + bj * NB + c] = src[r * LS + c];
  }
}

// A 32x32 block through registers (blocks of 256 threads: 4 doubles each), so the next
// block's loads can be in flight while the current one is multiplied.
__device__ __forceinline__ void load_regs(double r[4], const double* A, int ldm, int bi, int bj) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int t = threadIdx.x + 256 * q;
    r[q] = A[(size_t)(bi * NB + (t >> 5)) * ldm + bj * NB + (t & 31)];
  }
}
__device__ __forceinline__ void store_regs(double* dst, const double r[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int t = threadIdx.x + 256 * q;
    dst[(t >> 5) * LS + (t & 31)] = r[q];
  }
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double shfl_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __shfl((int)b, lane, 64);
  const int hi = __shfl((int)(b >> 32), lane, 64);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// In-LDS Cholesky of a 32x32 SPD block (lower); upper part zeroed. One wave, all 64 lanes:
// lane (r, h) = r + 32 h holds row r's columns 2 j + h in registers, so each of the 32
// right-looking steps (pivot by readlane, l_r = a_rc / sqrt(pivot), a_rs -= l_r l_s with l_s
// shuffled from lane s) is about half the instructions per lane of a one-row-per-lane form
// (which also kept ~60 broadcast values in SGPRs and spilled them): 17.0 -> 10.6 us per
// block, the same operations per element (same bits; tools/probes/chol_probe.hip). No
// workgroup barrier inside.
__device__ void chol32(double* a, int* err) {
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

// Inverse of a lower-triangular 32x32 block: column c by thread c, held in registers.
// Reciprocal pivots are formed first, off the chain; each row's entries of l are read into
// registers before its FMA chains (read at their use, every LDS read was waited for on
// its own: 50.6 -> 21.1 us for chol32 + trinv32 over 576 blocks, tools/spd_probe.hip, same
// bits), and each row's sum runs as two interleaved FMA chains.
// The 32 reciprocal pivots are divided once, one per thread, into x's spare column 32 (every
// thread dividing all 32 was ~1000 VALU instructions per thread; the same quotients).
__device__ __forceinline__ void trinv32(const double* l, double* x) {
  if (threadIdx.x < NB) {
    const int c = threadIdx.x;
    x[c * LS + NB] = 1.0 / l[c * LS + c];
    __builtin_amdgcn_wave_barrier();   // (one wave: its LDS writes land before its later reads)
    asm volatile("" ::: "memory");
    double rinv[NB], col[NB];
#pragma unroll
    for (int r = 0; r < NB; ++r) rinv[r] = x[r * LS + NB];
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      double lr[NB];
#pragma unroll
      for (int t = 0; t < r; ++t) lr[t] = l[r * LS + t];
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int t = 0; t + 1 < r; t += 2) {   // col[t] = 0 for t < c
        s0 += lr[t] * col[t];
        s1 += lr[t + 1] * col[t + 1];
      }
      if (r & 1) s0 += lr[r - 1] * col[r - 1];
      col[r] = r < c ? 0.0 : (r == c ? rinv[r] : -(s0 + s1) * rinv[r]);
    }
#pragma unroll
    for (int r = 0; r < NB; ++r) x[r * LS + c] = col[r];
  }
  __syncthreads();
}

// acc[4] += A(rows r0..) * B^T or A * B for a 32x32x32 product; thread owns 4 outputs.
// out(r, c) for r = tid>>3 (0..31), c = (tid&7)*4 + q
__device__ __forceinline__ void mm_nt(const double* a, const double* b, double acc[4]) {  // a * b^T
  const int r = threadIdx.x >> 3, cb = (threadIdx.x & 7) * 4;
  for (int t = 0; t < NB; ++t) {
    const double av = a[r * LS + t];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] += av * b[(cb + q) * LS + t];
  }
}
__device__ __forceinline__ void mm_nn(const double* a, const double* b, double acc[4]) {  // a * b
  const int r = threadIdx.x >> 3, cb = (threadIdx.x & 7) * 4;
  for (int t = 0; t < NB; ++t) {
    const double av = a[r * LS + t];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] += av * b[t * LS + cb + q];
  }
}
__device__ __forceinline__ void mm_tn(const double* a, const double* b, double acc[4]) {  // a^T * b
  const int r = threadIdx.x >> 3, cb = (threadIdx.x & 7) * 4;
  for (int t = 0; t < NB; ++t) {
    const double av = a[t * LS + r];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] += av * b[t * LS + cb + q];
  }
}

__global__ __launch_bounds__(256) void k_chol_panel(const ProbDesc* __restrict__ probs, int k) {
  const ProbDesc& p = probs[blockIdx.y];
  const int i = k + blockIdx.x;
  if (k >= p.nbk || i >= p.nbk) return;
  __shared__ double lkk[NB * LS], x[NB * LS], aik[NB * LS];
  __shared__ int err;
  if (threadIdx.x == 0) err = 0;
  double ra[4];                      // A_ik in flight while L_kk is factored and inverted
  if (i != k) load_regs(ra, p.A64, p.ldm, i, k);
  load_block(lkk, p.A64, p.ldm, k, k);
  __syncthreads();
  chol32(lkk, &err);
  if (i == k) {   // siblings still read A_kk in this launch: L_kk goes to the diagonal store
    if (err && threadIdx.x == 0) p.flags[2] = 1;
    store_block(p.D64, NB, k, 0, lkk);
    return;
  }
  trinv32(lkk, x);                   // x = L_kk^-1
  store_regs(aik, ra);
  __syncthreads();
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  mm_nt(aik, x, acc);                // L_ik = A_ik * (L_kk^-1)^T
  __syncthreads();
  const int r = threadIdx.x >> 3, cb = (threadIdx.x & 7) * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) aik[r * LS + cb + q] = acc[q];
  __syncthreads();
  store_block(p.A64, p.ldm, i, k, aik);
}

__global__ __launch_bounds__(256) void k_chol_update(const ProbDesc* __restrict__ probs, int k) {
  const ProbDesc& p = probs[blockIdx.y];
  const int n = p.nbk - k - 1;
  if (n <= 0) return;
  const int q = blockIdx.x;
  if (q >= n * (n + 1) / 2) return;
  // q -> (ii, jj) with 0 <= jj <= ii < n, row-major lower triangle
  int ii = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
  while ((ii + 1) * (ii + 2) / 2 <= q) ++ii;
  while (ii * (ii + 1) / 2 > q) --ii;
  const int jj = q - ii * (ii + 1) / 2;
  const int i = k + 1 + ii, j = k + 1 + jj;
  __shared__ double li[NB * LS], lj[NB * LS];
  load_block(li, p.A64, p.ldm, i, k);
  load_block(lj, p.A64, p.ldm, j, k);
  __syncthreads();
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  mm_nt(li, lj, acc);
  const int r = threadIdx.x >> 3, cb = (threadIdx.x & 7) * 4;
  double* dst = p.A64 + (size_t)(i * NB + r) * p.ldm + j * NB + cb;
#pragma unroll
  for (int t = 0; t < 4; ++t) dst[t] -= acc[t];
}

__global__ __launch_bounds__(256) void k_linv_row(const ProbDesc* __restrict__ probs, int i) {
  const ProbDesc& p = probs[blockIdx.y];
  const int j = blockIdx.x;
  if (i >= p.nbk || j > i) return;
  __shared__ double lii[NB * LS], xi[NB * LS], ta[NB * LS], tb[NB * LS];
  load_block(lii, p.D64, NB, i, 0);
  __syncthreads();
  trinv32(lii, xi);
  if (j == i) {
    store_block(p.L64, p.ldm, i, i, xi);
    return;
  }
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  // the blocks of step t + 1 are loaded into registers while step t multiplies
  double ra[4], rb[4];
  if (j < i) { load_regs(ra, p.A64, p.ldm, i, j); load_regs(rb, p.L64, p.ldm, j, j); }
  for (int t = j; t < i; ++t) {
    store_regs(ta, ra);   // L_it
    store_regs(tb, rb);   // Linv_tj
    __syncthreads();
    if (t + 1 < i) { load_regs(ra, p.A64, p.ldm, i, t + 1); load_regs(rb, p.L64, p.ldm, t + 1, j); }
    mm_nn(ta, tb, acc);
    __syncthreads();
  }
  const int r = threadIdx.x >> 3, cb = (threadIdx.x & 7) * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) ta[r * LS + cb + q] = acc[q];
  __syncthreads();
  double out[4] = {0.0, 0.0, 0.0, 0.0};
  mm_nn(xi, ta, out);                     // Linv_ii * S
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) tb[r * LS + cb + q] = -out[q];
  __syncthreads();
  store_block(p.L64, p.ldm, i, j, tb);
}

// Diagonal blocks of Linv: Linv_ii = L_ii^-1, all i of all problems in one launch.
__global__ __launch_bounds__(256) void k_diag_inv(const ProbDesc* __restrict__ probs) {
  const ProbDesc& p = probs[blockIdx.y];
  const int i = blockIdx.x;
  if (i >= p.nbk) return;
  __shared__ double lii[NB * LS], xi[NB * LS];
  load_block(lii, p.D64, NB, i, 0);
  __syncthreads();
  trinv32(lii, xi);
  store_block(p.L64, p.ldm, i, i, xi);
}

// Off-diagonal blocks of Linv by column slices: the columns of Linv are independent
// forward substitutions, so one workgroup owns a 4-column slice of block column j and
// produces its blocks i = j+1 .. nbk-1 with the finished ones kept in LDS:
//   Linv_ij = -Linv_ii S_i,   S_i = sum_{t=j}^{i-1} L_it Linv_tj
// One launch replaces the nbk dependent row launches. Right-looking: as soon as block t
// of the slice is final, every pending S_i (i > t) takes its L_it Linv_tj term. The
// 1024 threads are 8 groups of 128; group g owns the S_i with i = j+1+g (mod 8) in
// registers (thread (r, c) of a group: row r, slice column c), so per block t the
// pending products run 8 wide and the serial chain is ~1/8 of the slice's work.
// Sums run over t, then k, in order (the row-launch order).
constexpr int kLinvCols = 4;
constexpr int kLinvGroups = 8;
constexpr int kLinvMaxNbk = 56;   // LDS panel: nbk x 32 x 4 doubles (56 KB at the cap)
constexpr int kLinvPer = (kLinvMaxNbk + kLinvGroups - 1) / kLinvGroups;
__global__ __launch_bounds__(1024) void k_linv_cols(const ProbDesc* __restrict__ probs) {
  // grid ((maxnbk-1) * nsl, nprob). Measured: a j-major grid (every problem's long small-j
  // slices dispatched together) is 3x slower - the 8 slices of a block column each stream
  // the same L rows, and all of them at once thrash L2.
  const ProbDesc& p = probs[blockIdx.y];
  constexpr int nsl = NB / kLinvCols;
  const int j = blockIdx.x / nsl, c0 = (blockIdx.x % nsl) * kLinvCols;
  const int nbk = p.nbk, ldm = p.ldm;
  if (j >= nbk - 1) return;
  // dynamic LDS: panel [maxnbk][32][4] (block rows t >= j used), then sbuf [32][4]
  extern __shared__ double linv_lds[];
  double* panel = linv_lds;
  double* sbuf = linv_lds + (size_t)(gridDim.x / nsl + 1) * NB * kLinvCols;
  const int g = threadIdx.x >> 7, lt = threadIdx.x & 127;
  const int r = lt >> 2, c = lt & 3;
  const double* A64 = p.A64;
  double* L64 = p.L64;
  if (g == 0)   // block (j, j) of the slice: Linv_jj, written by k_diag_inv
    panel[(j * NB + r) * kLinvCols + c] = L64[(size_t)(j * NB + r) * ldm + j * NB + c0 + c];
  double acc[kLinvPer];
#pragma unroll
  for (int q = 0; q < kLinvPer; ++q) acc[q] = 0.0;
  __syncthreads();
  for (int t = j; t < nbk - 1; ++t) {
    const double* pt = panel + t * NB * kLinvCols + c;
    // pending S_i of this group, i = j + 1 + g + 8q > t
#pragma unroll
    for (int q = 0; q < kLinvPer; ++q) {
      const int i = j + 1 + g + kLinvGroups * q;
      if (i > t && i < nbk) {
        const double2* lp = reinterpret_cast<const double2*>(A64 + (size_t)(i * NB + r) * ldm + t * NB);
        double a = acc[q];
#pragma unroll
        for (int k = 0; k < NB; k += 2) {
          const double2 x = lp[k / 2];
          a += x.x * pt[k * kLinvCols];
          a += x.y * pt[(k + 1) * kLinvCols];
        }
        acc[q] = a;
      }
    }
    // S_{t+1} is complete: its owner group publishes it, then forms Linv_{t+1, j}
    const int i = t + 1;
    const int og = (i - j - 1) % kLinvGroups, oq = (i - j - 1) / kLinvGroups;
    if (g == og) {
      double v = 0.0;
#pragma unroll
      for (int q = 0; q < kLinvPer; ++q) v = q == oq ? acc[q] : v;
      sbuf[r * kLinvCols + c] = v;
    }
    __syncthreads();
    if (g == og) {
      const double2* dp = reinterpret_cast<const double2*>(L64 + (size_t)(i * NB + r) * ldm + i * NB);
      double o = 0.0;
#pragma unroll
      for (int k = 0; k < NB; k += 2) {
        const double2 d = dp[k / 2];
        o += d.x * sbuf[k * kLinvCols + c];
        o += d.y * sbuf[(k + 1) * kLinvCols + c];
      }
      panel[(i * NB + r) * kLinvCols + c] = -o;
      L64[(size_t)(i * NB + r) * ldm + j * NB + c0 + c] = -o;
    }
    __syncthreads();   // block i of the panel is read by every group next step; sbuf is rewritten
  }
}

__global__ __launch_bounds__(256) void k_minv(const ProbDesc* __restrict__ probs) {
  const ProbDesc& p = probs[blockIdx.y];
  const int q = blockIdx.x;
  const int n = p.nbk;
  if (q >= n * (n + 1) / 2) return;
  int i = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= q) ++i;
  while (i * (i + 1) / 2 > q) --i;
  const int j = q - i * (i + 1) / 2;      // j <= i
  __shared__ double ta[NB * LS], tb[NB * LS];
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  double ra[4], rb[4];
  load_regs(ra, p.L64, p.ldm, i, i);
  load_regs(rb, p.L64, p.ldm, i, j);
  for (int t = i; t < n; ++t) {
    store_regs(ta, ra);   // Linv_ti
    store_regs(tb, rb);   // Linv_tj
    __syncthreads();
    if (t + 1 < n) { load_regs(ra, p.L64, p.ldm, t + 1, i); load_regs(rb, p.L64, p.ldm, t + 1, j); }
    mm_tn(ta, tb, acc);
    __syncthreads();
  }
  const int r = threadIdx.x >> 3, cb = (threadIdx.x & 7) * 4;
  const int gr = i * NB + r;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int gc = j * NB + cb + t;
    const float v = (gr < p.R && gc < p.R) ? (float)acc[t] : 0.f;
    p.M[(size_t)gr * p.ldm + gc] = v;
    p.M[(size_t)gc * p.ldm + gr] = v;
  }
}

// L (lower, in A64) and Linv = L^-1 (lower blocks of L64; the upper off-diagonal blocks are
// not written) of A64 = L L^T; flags[2] on a non-positive pivot. Every launch reads the block
// count from the descriptor, so a descriptor whose nbk is 0 turns them all into no-ops (the
// blocked EPC step's rounds after its search is done, solve64.hip).
void launch_spd_linv(const ProbDesc* d, int nprob, int maxnbk, hipStream_t s) {
  for (int k = 0; k < maxnbk; ++k) {
    hipLaunchKernelGGL(k_chol_panel, dim3(maxnbk - k, nprob), dim3(256), 0, s, d, k);
    const int n = maxnbk - k - 1;
    if (n > 0) hipLaunchKernelGGL(k_chol_update, dim3(n * (n + 1) / 2, nprob), dim3(256), 0, s, d, k);
  }
  if (maxnbk <= kLinvMaxNbk) {
    hipLaunchKernelGGL(k_diag_inv, dim3(maxnbk, nprob), dim3(256), 0, s, d);
    if (maxnbk > 1)
      hipLaunchKernelGGL(k_linv_cols, dim3((maxnbk - 1) * (NB / kLinvCols), nprob), dim3(1024),
                         (size_t)(maxnbk + 1) * NB * kLinvCols * sizeof(double), s, d);
  } else {   // panel would not fit in LDS: one launch per block row
    for (int i = 0; i < maxnbk; ++i) hipLaunchKernelGGL(k_linv_row, dim3(i + 1, nprob), dim3(256), 0, s, d, i);
  }
}

void launch_spd_inverse(const ProbDesc* d, int nprob, int maxnbk, hipStream_t s) {
  launch_spd_linv(d, nprob, maxnbk, s);
  hipLaunchKernelGGL(k_minv, dim3(maxnbk * (maxnbk + 1) / 2, nprob), dim3(256), 0, s, d);
}

}  // namespace admmq

// Quantizer kernels: the MSE-minmax candidate search (source/quantization.py:118-144)
// and the tensor_* schemes (:48-66, :91-106), for standalone quantize_tensor calls
// and for the ADMM projection step.
#include "quant_device.h"

namespace admmq {

// Load a chunk of quads into LDS and run the candidate sweep.
__device__ __forceinline__ void sse_chunk(const float* __restrict__ X, int ld, int qpr, int nq, int q0,
                                          const unsigned* stat, unsigned long long* sse, int ncand, int bits) {
  __shared__ float4 xs[kSseQuads];
  const float mx = __uint_as_float(stat[0]);
  if (mse_degenerate(mx)) return;
  const int nqc = min(kSseQuads, nq - q0);
  for (int t = threadIdx.x; t < nqc; t += blockDim.x) {
    const int qi = q0 + t;
    const int row = qi / qpr;
    const int qc = qi - row * qpr;
    xs[t] = *reinterpret_cast<const float4*>(X + (size_t)row * ld + 4 * qc);
  }
  __syncthreads();
  sse_sweep(xs, nqc, mx, fixed_exp(mx, nq), ncand, bits, sse);
}

// ADMM projection: SSE pass over X = H_T - U of every active problem.
__global__ __launch_bounds__(256) void k_sse_admm(const ProbDesc* __restrict__ probs, const Chunk* __restrict__ chunks,
                                                  int ncand, int bits, int slot) {
  const Chunk ck = chunks[blockIdx.x];
  const ProbDesc& p = probs[ck.job];
  if (p.flags[0]) return;
  const int qpr = (p.R + 3) >> 2;
  sse_chunk(p.X, p.ld, qpr, p.nq, ck.start, p.stat + 4 * slot, p.sse + (size_t)slot * ncand, ncand, bits);
}

// Standalone: pack rows x cols -> rows x ld (zero pads) and gather min/max/absmax.
__global__ __launch_bounds__(256) void k_qpack(const QJob* __restrict__ jobs, const Chunk* __restrict__ chunks) {
  const Chunk ck = chunks[blockIdx.x];
  const QJob& j = jobs[ck.job];
  const long long total = (long long)j.rows * j.ld;
  const long long e = (long long)ck.start + 4LL * threadIdx.x;
  unsigned amax = 0u, mn = 0xFFFFFFFFu, mxo = 0u;
  if (e < total) {
    const int row = (int)(e / j.ld);
    const int c0 = (int)(e - (long long)row * j.ld);
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = c0 + k;
      if (c < j.cols) {
        v[k] = j.src[(size_t)row * j.cols + c];
        amax = max(amax, __float_as_uint(v[k]) & 0x7FFFFFFFu);
        mn = min(mn, enc_ord(v[k]));
        mxo = max(mxo, enc_ord(v[k]));
      } else {
        v[k] = 0.f;
      }
    }
    *reinterpret_cast<float4*>(j.Xp + e) = make_float4(v[0], v[1], v[2], v[3]);
  }
  __shared__ unsigned red[3][4];
  amax = wave_max_u32(amax); mn = wave_min_u32(mn); mxo = wave_max_u32(mxo);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = amax; red[1][w] = mn; red[2][w] = mxo; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      amax = max(amax, red[0][k]); mn = min(mn, red[1][k]); mxo = max(mxo, red[2][k]);
    }
    atomicMax(&j.stat[0], amax);
    atomicMin(&j.stat[1], mn);
    atomicMax(&j.stat[2], mxo);
  }
}

__global__ __launch_bounds__(256) void k_sse_q(const QJob* __restrict__ jobs, const Chunk* __restrict__ chunks,
                                               int ncand, int bits) {
  const Chunk ck = chunks[blockIdx.x];
  const QJob& j = jobs[ck.job];
  sse_chunk(j.Xp, j.ld, j.ld >> 2, j.nq, ck.start, j.stat, j.sse, ncand, bits);
}

__global__ __launch_bounds__(256) void k_qfinal(const QJob* __restrict__ jobs, const Chunk* __restrict__ chunks,
                                                int ncand, int bits, int scheme) {
  const Chunk ck = chunks[blockIdx.x];
  const QJob& j = jobs[ck.job];
  const QParams qp = block_qparams(scheme, bits, j.stat, j.sse, ncand, j.has_kw, j.tmin_kw, j.tmax_kw);
  const long long total = (long long)j.rows * j.ld;
  const long long e = (long long)ck.start + 4LL * threadIdx.x;
  if (e >= total) return;
  const int row = (int)(e / j.ld);
  const int c0 = (int)(e - (long long)row * j.ld);
  const float4 v = *reinterpret_cast<const float4*>(j.Xp + e);
  const float xv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + k;
    if (c < j.cols) j.dst[(size_t)row * j.cols + c] = apply_quant(xv[k], qp);
  }
}

void launch_sse_admm(const ProbDesc* d, const Chunk* chunks, int nchunks, int ncand, int bits, int slot,
                     hipStream_t s) {
  if (nchunks > 0) hipLaunchKernelGGL(k_sse_admm, dim3(nchunks), dim3(256), 0, s, d, chunks, ncand, bits, slot);
}
void launch_qpack(const QJob* jobs, const Chunk* chunks, int nchunks, hipStream_t s) {
  if (nchunks > 0) hipLaunchKernelGGL(k_qpack, dim3(nchunks), dim3(256), 0, s, jobs, chunks);
}
void launch_sse_q(const QJob* jobs, const Chunk* chunks, int nchunks, int ncand, int bits, hipStream_t s) {
  if (nchunks > 0) hipLaunchKernelGGL(k_sse_q, dim3(nchunks), dim3(256), 0, s, jobs, chunks, ncand, bits);
}
void launch_qfinal(const QJob* jobs, const Chunk* chunks, int nchunks, int ncand, int bits, int qscheme,
                   hipStream_t s) {
  if (nchunks > 0)
    hipLaunchKernelGGL(k_qfinal, dim3(nchunks), dim3(256), 0, s, jobs, chunks, ncand, bits, qscheme);
}

}  // namespace admmq

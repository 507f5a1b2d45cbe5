// Standalone quantize_tensor kernels (source/quantization.py:69-115): pack + tensor
// statistics, and the final elementwise quantization with the resolved parameters.
// The MSE-minmax candidate search itself lives in mse_search.hip.
#include "quant_device.h"

namespace admmq {

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
    atomicMax(&j.mv.stat[0], amax);
    atomicMin(&j.mv.stat[1], mn);
    atomicMax(&j.mv.stat[2], mxo);
  }
}

__global__ __launch_bounds__(256) void k_qfinal(const QJob* __restrict__ jobs, const Chunk* __restrict__ chunks,
                                                int ncand, int bits, int scheme) {
  const Chunk ck = chunks[blockIdx.x];
  const QJob& j = jobs[ck.job];
  const QParams qp = block_qparams(scheme, bits, j.mv, 0, ncand, j.has_kw, j.tmin_kw, j.tmax_kw);
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

void launch_qpack(const QJob* jobs, const Chunk* chunks, int nchunks, hipStream_t s) {
  if (nchunks > 0) hipLaunchKernelGGL(k_qpack, dim3(nchunks), dim3(256), 0, s, jobs, chunks);
}
void launch_qfinal(const QJob* jobs, const Chunk* chunks, int nchunks, int ncand, int bits, int qscheme,
                   hipStream_t s) {
  if (nchunks > 0)
    hipLaunchKernelGGL(k_qfinal, dim3(nchunks), dim3(256), 0, s, jobs, chunks, ncand, bits, qscheme);
}

}  // namespace admmq

// What a per-mode persistent loop would pay per ADMM iteration for its hand-offs, against
// the kernel boundaries of the per-iteration launches it would replace (VERDICT r04 item 1;
// DESIGN §7r5). A persistent team of G workgroups (256 threads, one team = one factor's
// tiles) needs three team-wide hand-offs per iteration (max|X|, the stage-1 totals, the next
// right-hand side); the launch-per-phase form has two dependent kernel boundaries (solve ->
// search -> next solve). Both are timed here with no work in between:
//   mode 0: persistent grid, `iters` x 3 barriers, each the thin loop's counter form (every
//           thread's stores drained, workgroup barrier, lane 0 adds to an agent-scope counter
//           and polls it with sc1 loads + s_sleep 1, workgroup barrier); bounded polls.
//   mode 1: the same grid as an empty kernel, 2 x `iters` launches back to back on one stream.
// Usage: barrier_probe MODE G ITERS  -> prints us per iteration (hipEvent timing).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ bool team_barrier(unsigned* bar, unsigned target, unsigned polls, int* s_ok) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    unsigned n = 0;
    while (__hip_atomic_load((gu32*)bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++n > polls) { ok = 0; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

__global__ __launch_bounds__(256) void k_persist(unsigned* bar, int iters, int* fault) {
  __shared__ int s_ok;
  const unsigned G = gridDim.x;
  unsigned nbar = 0;
  for (int it = 0; it < iters; ++it)
    for (int b = 0; b < 3; ++b)
      if (!team_barrier(bar, G * ++nbar, 1u << 22, &s_ok)) {
        if (threadIdx.x == 0) atomicAdd(fault, 1);
        return;
      }
}

__global__ __launch_bounds__(256) void k_empty(int* sink) {
  if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) *sink = 1;
}

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: %s MODE G ITERS\n", argv[0]); return 2; }
  const int mode = atoi(argv[1]), G = atoi(argv[2]), iters = atoi(argv[3]);
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  int per = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_persist, 256, 0);
  if (mode == 0 && G > per * cus) { fprintf(stderr, "grid %d exceeds resident %d\n", G, per * cus); return 2; }
  unsigned* bar;
  int* fault;
  hipMalloc(&bar, 64);
  hipMalloc(&fault, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(bar, 0, 64);
    hipMemset(fault, 0, 64);
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    if (mode == 0) {
      hipLaunchKernelGGL(k_persist, dim3(G), dim3(256), 0, 0, bar, iters, fault);
    } else {
      for (int i = 0; i < 2 * iters; ++i) hipLaunchKernelGGL(k_empty, dim3(G), dim3(256), 0, 0, fault);
    }
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  int hf = 0;
  hipMemcpy(&hf, fault, sizeof(int), hipMemcpyDeviceToHost);
  printf("mode %d (%s) grid %d: %.2f us per iteration (%s per iteration), faults %d\n", mode,
         mode == 0 ? "persistent" : "launches", G, 1e3f * best / iters,
         mode == 0 ? "3 team barriers" : "2 kernel boundaries", hf);
  return hf ? 1 : 0;
}

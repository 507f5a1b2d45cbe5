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
//   mode 2 (round 6, VERDICT r05 item 2: no single-address counter): tagged arrival words,
//           one per workgroup (its barrier number, an sc1 store - no read-modify-write), one
//           poller (workgroup 0's first wave: lane l checks words l, l + 64, ...) that then
//           writes the release word, which every workgroup polls (sc1 loads + s_sleep 1).
//   mode 3: the same two-level: groups of 32 consecutive workgroups, the group's first
//           workgroup polls its members' words and publishes a group word; workgroup 0 polls
//           the group words and releases: three hops, at most 32 words per poll.
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

__device__ __forceinline__ unsigned ld_sc1(const unsigned* q) {
  return __hip_atomic_load((gu32*)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(unsigned* q, unsigned v) {
  __hip_atomic_store((gu32*)q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// wave 0 of the calling workgroup waits until words[0 .. n) all reach `tag` (bounded)
__device__ __forceinline__ bool wave_poll_all(const unsigned* words, int n, unsigned tag, unsigned polls) {
  const int lane = threadIdx.x & 63;
  unsigned k = 0;
  for (;;) {
    int ok = 1;
    for (int i = lane; i < n; i += 64) ok &= ld_sc1(words + i) >= tag ? 1 : 0;
    if (__all(ok)) return true;
    if (++k > polls) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ bool poll_one(const unsigned* w, unsigned tag, unsigned polls) {
  unsigned k = 0;
  while (ld_sc1(w) < tag) {
    if (++k > polls) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}
// words: [0, G) arrivals, [G, G + 64) group words, [G + 64] release
__device__ __forceinline__ bool slot_barrier(unsigned* words, unsigned tag, int hier, int* s_ok) {
  const int G = gridDim.x, b = blockIdx.x;
  unsigned* grp = words + G;
  unsigned* rel = words + G + 64;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  int ok = 1;
  if (threadIdx.x == 0) st_sc1(words + b, tag);
  if (threadIdx.x < 64) {
    if (!hier) {
      if (b == 0) { ok = wave_poll_all(words, G, tag, 1u << 22) ? 1 : 0; if (threadIdx.x == 0) st_sc1(rel, tag); }
    } else {
      const int g0 = b & ~31, gn = min(32, G - g0), ng = (G + 31) / 32;
      if (b == g0) { ok = wave_poll_all(words + g0, gn, tag, 1u << 22) ? 1 : 0; if (threadIdx.x == 0) st_sc1(grp + b / 32, tag); }
      if (b == 0) { ok &= wave_poll_all(grp, ng, tag, 1u << 22) ? 1 : 0; if (threadIdx.x == 0) st_sc1(rel, tag); }
    }
    if (threadIdx.x == 0) { ok &= poll_one(rel, tag, 1u << 22) ? 1 : 0; *s_ok = ok; }
  }
  __syncthreads();
  return *s_ok != 0;
}

__global__ __launch_bounds__(256) void k_persist_slots(unsigned* words, int iters, int hier, int* fault) {
  __shared__ int s_ok;
  unsigned tag = 0;
  for (int it = 0; it < iters; ++it)
    for (int b = 0; b < 3; ++b)
      if (!slot_barrier(words, ++tag, hier, &s_ok)) {
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
  if (mode != 1 && G > per * cus) { fprintf(stderr, "grid %d exceeds resident %d\n", G, per * cus); return 2; }
  unsigned* bar;
  int* fault;
  hipMalloc(&bar, (size_t)(G + 128) * 4);
  hipMalloc(&fault, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(bar, 0, (size_t)(G + 128) * 4);
    hipMemset(fault, 0, 64);
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    if (mode == 0) {
      hipLaunchKernelGGL(k_persist, dim3(G), dim3(256), 0, 0, bar, iters, fault);
    } else if (mode >= 2) {
      hipLaunchKernelGGL(k_persist_slots, dim3(G), dim3(256), 0, 0, bar, iters, mode - 2, fault);
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
  const char* nm[4] = {"persistent, counter", "launches", "persistent, arrival words", "persistent, 2-level words"};
  printf("mode %d (%s) grid %d: %.2f us per iteration (%s per iteration), faults %d\n", mode, nm[mode], G,
         1e3f * best / iters, mode == 1 ? "2 kernel boundaries" : "3 team barriers", hf);
  return hf ? 1 : 0;
}

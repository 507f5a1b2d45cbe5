// C-ABI of libadmmq: workspace planning and stream-ordered launch sequences.
// See include/admmq.h for the contract and the reference interfaces replaced.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <array>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/admmq.h"
#include "admmq_internal.h"

namespace admmq {

static thread_local std::string g_err;

static int fail(int code, const char* msg) {
  g_err = msg;
  return code;
}
int set_error(int code, const char* msg) { return fail(code, msg); }

static int check_hip(const char* where) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string(where) + ": " + hipGetErrorString(e);
    return ADMMQ_ERR_HIP;
  }
  return ADMMQ_OK;
}

// Host -> device uploads of the plans (descriptors, tile and unit lists) through pinned
// staging chunks, so that hipMemcpyAsync is truly asynchronous: a pageable source makes
// the copy wait for the stream, which put every call's host planning on the GPU's
// critical path (the host could not run ahead of the device by one mode call). A chunk
// is reused once the event recorded after its copy has completed; one pool per device -
// the device the STREAM belongs to (the event must be on it), not the caller's current
// one. The pool is capped by bytes (kPinMaxBytes per device): when every chunk that could
// hold the plan is still in flight and the cap is reached, the plan goes up by a plain
// pageable hipMemcpyAsync instead (HIP stages a pageable source before it returns, so the
// host buffer may be reused at once; that copy may wait for the stream - the only case in
// which an entry point can block, include/admmq.h), never by waiting on a chunk's event.
struct PinnedChunk { char* p; size_t cap; hipEvent_t ev; bool used; };
static std::mutex g_pin_mu;
static std::vector<PinnedChunk> g_pin[64];
static size_t g_pin_bytes[64];
static constexpr size_t kPinMaxBytes = size_t(64) << 20;
int upload_async(void* dst, const void* src, size_t n, hipStream_t s) {
  if (n == 0) return ADMMQ_OK;
  int dev = -1;
  if (hipStreamGetDevice(s, &dev) != hipSuccess) {
    (void)hipGetLastError();
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  }
  if (dev < 0 || dev >= 64) dev = 0;
  std::lock_guard<std::mutex> g(g_pin_mu);
  std::vector<PinnedChunk>& pool = g_pin[dev];
  PinnedChunk* c = nullptr;
  for (PinnedChunk& k : pool)
    if (k.cap >= n && (!k.used || hipEventQuery(k.ev) == hipSuccess)) { c = &k; break; }
  size_t cap = 4096;
  while (cap < n) cap *= 2;
  if (!c && g_pin_bytes[dev] + cap > kPinMaxBytes) {   // pool full and busy: pageable copy
    const hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) {
      g_err = std::string("upload (pageable): ") + hipGetErrorString(e);
      return ADMMQ_ERR_HIP;
    }
    return ADMMQ_OK;
  }
  if (!c) {
    PinnedChunk k;
    k.cap = cap;
    k.used = false;
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (cur != dev) (void)hipSetDevice(dev);   // the event (and the chunk's mapping) on the stream's device
    const hipError_t ea = hipHostMalloc(reinterpret_cast<void**>(&k.p), k.cap, hipHostMallocDefault);
    const hipError_t ee = ea == hipSuccess ? hipEventCreateWithFlags(&k.ev, hipEventDisableTiming) : ea;
    if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
    if (ea != hipSuccess) {
      (void)hipGetLastError();
      g_err = "upload: pinned staging allocation failed";
      return ADMMQ_ERR_HIP;
    }
    if (ee != hipSuccess) {
      (void)hipHostFree(k.p);
      g_err = "upload: event creation failed";
      return ADMMQ_ERR_HIP;
    }
    pool.push_back(k);
    g_pin_bytes[dev] += k.cap;
    c = &pool.back();
  }
  std::memcpy(c->p, src, n);
  hipError_t e = hipMemcpyAsync(dst, c->p, n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipEventRecord(c->ev, s);
  c->used = true;
  if (e != hipSuccess) {
    g_err = std::string("upload: ") + hipGetErrorString(e);
    return ADMMQ_ERR_HIP;
  }
  return ADMMQ_OK;
}
static int h2d(void* dst, const void* src, size_t n, hipStream_t s) { return upload_async(dst, src, n, s); }

static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
static inline int rup(int v, int a) { return (v + a - 1) / a * a; }

// Optional per-launch HIP-event timing (bench.py measures the dominant kernel live on
// the stream it runs on). Events are created in admmq_profile_begin, never in a launch path.
struct Prof {
  bool on = false;
  std::vector<hipEvent_t> ev;
  std::vector<int> cls;
  size_t next = 0;
  int every = 1;        // time one ADMM iteration in `every` (events add inter-kernel gaps)
  bool sampled = true;  // the current iteration is timed
};
static Prof g_prof;
// Process-wide switches (atomics: set from any thread, read by the launch sequences).
// exhaustive: evaluate all candidates (reference-style) instead of the two-stage search;
// legacy stage 1: the per-level stage-1 form instead of merged thresholds (same integers);
// solve mode: the process default (kSolveF32: the reference's fp32 arithmetic; kSolveSplit
// opt-in) of the plain entry points, read once at prepare and recorded per workspace.
static std::atomic<bool> g_exhaustive{false};
static std::atomic<bool> g_legacy_stage1{false};
static std::atomic<int> g_solve_mode{kSolveF32};
// fused finalize (k_mse_hist3<.., true>) where the residency check allows it; 0: the
// separate k_finalize_admm launch (A/B and cross-check, same integers)
static std::atomic<bool> g_fused_finalize{true};
// stage-1 units per block of the non-fused search launch (0: sized by the planner)
static std::atomic<int> g_hist_reps{0};
// polls of the fused finalize's bounded wait for its job's selection (diagnostics can
// shrink it to force the timeout path)
static std::atomic<unsigned> g_fin_wait_polls{kFinWaitPollsDefault};
// diagnostics: a smaller resident-block budget for the fused finalize (0: the device's),
// to exercise its several-units-per-block form on small batches
static std::atomic<int> g_fin_cap_override{0};
static std::atomic<int> g_fin_nv3{1};   // diagnostics: 0 = never three float4 groups per search thread
// persistent loop of the thin factors (k_thin_loop) for calls whose problems are all
// thin: 1 on, 0 off (the per-iteration launches: A/B and cross-check), 2 on with 64-column
// workgroups wherever allowed (exercises that form on batches that fit without it)
static std::atomic<int> g_thin_loop{1};

// Tile rows of the persistent fp32 solve per problem (fixed by the problem's shape, never
// by the batch, so every element's result is batch-independent): 0 = 64 x 64 tiles
// (32-row factors: 32 x 64); 1 = 128 x 64 tiles for the factors with ld >= 1024 whose I
// is a multiple of 128, 32 x 64 tiles for the others (finer filler tiles: the CU-level
// LPT of a launch then balances to ~0.99 at C3 instead of 0.89, where the 36-K-step 64 x 64
// tiles of the R = 1141 layers left gaps only coarse tiles could not fill); 2 = 64 x 64 for
// ld >= 1024, 32 x 64 for the others; 3 = 128 x 64 for ld >= 1024, 64 x 64 for the others.
static std::atomic<int> g_f32_rule{1};
// fp32 solve kernel: 0 = k_gemm (64 x 64 tiles), 1 = persistent tile lists (k_gemm_f32p,
// slower: DESIGN §7), 2 = one tile per workgroup with per-problem tile rows (k_gemm_f32t)
static std::atomic<int> g_f32_kernel{0};
static std::atomic<int> g_even_units{1};   // big-job stage-1 units sized to fill the resident round evenly
static int f32_tile_rows(int I, int ld) {
  if (I <= 32) return 32;
  const int rule = g_f32_rule.load();
  const bool big = ld >= 1024;
  switch (rule) {
    case 0: return 64;
    case 2: return big ? 64 : 32;
    case 3: return (big && I % 128 == 0) ? 128 : 64;
    default: return (big && I % 128 == 0) ? 128 : 32;
  }
}
static constexpr int kF32Slots = 2;   // k_gemm_f32p workgroups per CU (72 KB of LDS each)

// K-split of the fp32 64 x 64 solve tiles (gemm_kernels.hip ksplit_combine): 1 = by
// ksplit_pieces, 0 = never (A/B). A factor whose tiles alone leave most of the chip idle
// (a lone layer4 conv: 144 tiles of 36 K-steps on 256 CUs, the busiest shard of a
// multi-GPU run) splits every tile's K range into np pieces summed in piece order.
static std::atomic<int> g_ksplit{1};
// 64x64 tiles of a launch from which its I > 64 factors without a K-split take the 256x128
// tiles (default kWideMinTiles; diagnostics: admmq_debug_set_wide_min_tiles; same bits)
static std::atomic<long long> g_wide_min_tiles{kWideMinTiles};
// execution form of the pieces (same bits either way): 1 = parallel only where the 64 x 64
// launch's whole tiles leave CUs idle, else serial (default); 0 = always serial; 2 = always parallel
static std::atomic<int> g_ksplit_par{1};
// Pieces per tile, a function of (I, R) ONLY (never of the batch, the device or the
// launch), so a factor's bits are the same in every batch: the np in 1..kKsplitMax with
// pieces of >= kKsplitMinSteps K-steps that minimises the factor's own launch length on
// a 256-CU chip, ceil(tiles np / 256) ceil(nk / np) K-steps plus kKsplitCost for the
// partial hand-off, ties to the smaller np. Only factors with fewer tiles than CUs split.
static constexpr int kKsplitChipCUs = 256;
static constexpr int kKsplitCost = 4;   // K-steps (~2.5 us): partial stores, arrival, sc1 reads
// Balance (launches that fill the chip): 1 = run the pieces of the longest split tiles in
// parallel where that lowers the launch's CU-level LPT makespan (same bits), 0 = never;
// a parallel piece is priced kKsplitCost... g_ksplit_cost K-steps above its own.
static std::atomic<int> g_ksplit_bal{1};
static std::atomic<int> g_ksplit_cost{1};
// Resident 64 x 64 fp32 solve workgroups per CU (the LPT's slots): 3 for the default 3-deep
// staging ring (48 KB of LDS), 4 for the 2-deep ring (k_gemm_f32b<2>, 32 KB, 4 waves per SIMD)
static int f32_slots() { return g_gemm_f32_stage == 2 ? 4 : 3; }
// Makespan (K-steps of the busiest CU) of an LPT placement of `costs` over ncu CUs with at
// most `slots` items each (order_tiles_for_cus' rule without its XCD tie-break); -1 when
// the items do not fit one resident round.
static long long lpt_makespan(std::vector<long long> costs, int ncu, int slots) {
  if ((long long)costs.size() > (long long)ncu * slots) return -1;
  std::sort(costs.begin(), costs.end(), std::greater<long long>());
  // min-heap of (load, cu) over the CUs with a free slot
  std::vector<std::pair<long long, int>> heap;
  std::vector<int> used(ncu, 0);
  for (int b = 0; b < ncu; ++b) heap.push_back({0, b});
  auto cmp = [](const std::pair<long long, int>& a, const std::pair<long long, int>& b) { return a > b; };
  std::make_heap(heap.begin(), heap.end(), cmp);
  long long mx = 0;
  for (long long c : costs) {
    std::pop_heap(heap.begin(), heap.end(), cmp);
    auto [ld, b] = heap.back();
    heap.pop_back();
    ld += c;
    mx = std::max(mx, ld);
    if (++used[b] < slots) {
      heap.push_back({ld, b});
      std::push_heap(heap.begin(), heap.end(), cmp);
    }
  }
  return mx;
}
// How many of the split tiles `cand` (longest first; (nk, np)) to run as parallel pieces so
// that the launch's LPT makespan is smallest (ties: fewer), `whole` = every tile's K-steps.
static long long ksplit_balance(const std::vector<long long>& whole, std::vector<std::pair<int, int>> cand, int ncu,
                                int slots, int cost) {
  if (cand.empty() || (long long)whole.size() <= ncu) return 0;
  std::stable_sort(cand.begin(), cand.end(), [](auto& a, auto& b) { return a.first > b.first; });
  long long best_m = lpt_makespan(whole, ncu, slots);
  if (best_m < 0) return 0;
  long long best_k = 0;
  std::vector<long long> costs = whole;
  // remove one whole tile of each split candidate as it is split: keep a multiset by value
  for (long long k = 1; k <= (long long)cand.size(); ++k) {
    const int nk = cand[k - 1].first, np = cand[k - 1].second;
    auto it = std::find(costs.begin(), costs.end(), (long long)nk);
    if (it == costs.end()) break;
    costs.erase(it);
    for (int pc = 0; pc < np; ++pc) costs.push_back((pc + 1) * nk / np - pc * nk / np + cost);
    const long long m = lpt_makespan(costs, ncu, slots);
    if (m < 0) break;
    if (m < best_m) { best_m = m; best_k = k; }
  }
  return best_k;
}

static int ksplit_pieces(int I, int R) {
  if (I <= 32) return 1;   // 32 x 64 tiles
  const int nk = rup(R, 32) / 32;
  const long long tiles = (long long)((I + 63) / 64) * ((rup(R, 32) + 63) / 64);
  if (tiles >= kKsplitChipCUs) return 1;
  int best = 1;
  long long best_cost = nk;
  for (int np = 2; np <= kKsplitMax; ++np) {
    const int len = (nk + np - 1) / np;
    if (len < kKsplitMinSteps) break;
    const long long cost = (tiles * np + kKsplitChipCUs - 1) / kKsplitChipCUs * len + kKsplitCost;
    if (cost < best_cost) { best = np; best_cost = cost; }
  }
  return best;
}

// CUs of the current device (looked up once per device)
static int device_cus() {
  constexpr int kMaxDev = 64;
  static std::once_flag once[kMaxDev];
  static int cus[kMaxDev];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 256;
  std::call_once(once[dev], [dev]() {
    int n = 0;
    cus[dev] = (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) ? n : 256;
  });
  return cus[dev];
}

// Persistent fp32 solve lists: every tile goes, largest MFMA work first, to the CU with the
// least work so far (ties: the CU whose XCD already holds tiles of the same M column / P row
// panel, which then come from that XCD's L2), then each CU's tiles are split over its
// kF32Slots workgroups (LPT again). Workgroup b runs on CU b mod ncu (round-robin dispatch;
// a different placement only costs speed). Fills `tiles` in list order and `off`.
static void plan_f32_lists(std::vector<GemmTile>& tiles, std::vector<int>& off, int ncu) {
  std::vector<GemmTile> sorted = tiles;
  auto work = [](const GemmTile& t) { return (long long)t.bm * t.nk; };
  std::stable_sort(sorted.begin(), sorted.end(), [&](const GemmTile& a, const GemmTile& b) { return work(a) > work(b); });
  constexpr int kXcd = 8;
  std::vector<std::vector<GemmTile>> bins(ncu);
  std::vector<long long> load(ncu, 0);
  std::map<std::pair<int, int>, std::array<int, kXcd>> col_on, row_on;
  for (const GemmTile& t : sorted) {
    auto& cx = col_on[{t.prob, t.tn}];
    auto& rx = row_on[{t.prob, t.tm * t.bm}];
    int best = 0;
    long long best_key = 0;
    for (int b = 0; b < ncu; ++b) {
      const long long key = load[b] * 1000000LL - cx[b % kXcd] * 1000LL - rx[b % kXcd];
      if (b == 0 || key < best_key) { best = b; best_key = key; }
    }
    bins[best].push_back(t);
    load[best] += work(t);
    cx[best % kXcd] += 1;
    rx[best % kXcd] += 1;
  }
  const int nslots = ncu * kF32Slots;
  std::vector<std::vector<GemmTile>> lists(nslots);
  for (int c = 0; c < ncu; ++c) {
    long long sl[kF32Slots] = {};
    for (const GemmTile& t : bins[c]) {   // already largest first
      int k = 0;
      for (int j = 1; j < kF32Slots; ++j)
        if (sl[j] < sl[k]) k = j;
      lists[c + (size_t)k * ncu].push_back(t);
      sl[k] += work(t);
    }
  }
  tiles.clear();
  off.assign(nslots + 1, 0);
  for (int b = 0; b < nslots; ++b) {
    off[b] = (int)tiles.size();
    tiles.insert(tiles.end(), lists[b].begin(), lists[b].end());
  }
  off[nslots] = (int)tiles.size();
}

// What each prepare recorded for its workspace: the solve mode (the run must use the operand
// planes its prepare wrote) and a fingerprint of the carve - the problem shapes, the byte
// count and every process switch that moves buffers (tile rows, stage-1 unit sizing,
// K-split) - so a run whose plan would carve the workspace differently is refused instead of
// reading another layout. Keyed by address: a workspace freed and reallocated at the same
// address for the same problems still needs its own prepare (include/admmq.h).
struct WsRecord { int mode; unsigned long long fp; };
static std::mutex g_ws_mu;
static std::unordered_map<const void*, WsRecord> g_ws_rec;
static void record_ws(const void* ws, int mode, unsigned long long fp) {
  std::lock_guard<std::mutex> g(g_ws_mu);
  g_ws_rec[ws] = {mode, fp};
}
static bool recorded_ws(const void* ws, WsRecord& out) {
  std::lock_guard<std::mutex> g(g_ws_mu);
  auto it = g_ws_rec.find(ws);
  if (it == g_ws_rec.end()) return false;
  out = it->second;
  return true;
}
static int recorded_ws_mode(const void* ws) {
  WsRecord r;
  return recorded_ws(ws, r) ? r.mode : -1;
}

// The two-stage search needs the per-block threshold table in LDS; otherwise exhaustive.
static bool two_stage_ok(int ncand, int bits) {
  return !g_exhaustive && ncand <= kMaxStage1 && bits <= kMaxStage1Bits && hist_lds_bytes(ncand, bits) <= 64 * 1024;
}

// Exact merged order of the level thresholds for (n, qmax) (k_mse_hist3): thr[k][c] is
// within a few ulps of (2k-1) ((n-1) + 5c) times a constant, so the integer keys give
// the order; rank0[e] for e = (k-1) n + c, and the groups of equal keys as
// {first rank, size, element indices...} padded to 6 entries. false: a tie group larger
// than 4 (the per-level stage 1 is used instead).
// rank0 is returned padded to kMaxMerged entries and followed by the coarse cell index
// lower bound lo[g], g = 0..kCells (see h3_setup): the number of thresholds whose cell
// (floor of threshold * kCells / largest threshold) is below g for EVERY mx. A
// threshold's cell is floor(z (1 + d)) with z = kCells key / key_max and |d| a few ulps
// (the float thresholds and the cell scale each within ~10 ulps of the key proportion),
// so counting the keys with z (1 + 1e-4) < g can only undercount.
static bool merged_tables(int n, int qmax, std::vector<unsigned short>& rank0, std::vector<unsigned short>& groups) {
  const int M = qmax * n;
  std::vector<std::pair<long long, int>> key(M);
  for (int k = 1; k <= qmax; ++k)
    for (int c = 0; c < n; ++c) key[(k - 1) * n + c] = {(long long)(2 * k - 1) * ((n - 1) + 5LL * c), (k - 1) * n + c};
  std::sort(key.begin(), key.end());
  rank0.assign(kMaxMerged + kCells + 2, 0);
  groups.clear();
  for (int r = 0; r < M;) {
    int r1 = r + 1;
    while (r1 < M && key[r1].first == key[r].first) ++r1;
    for (int j = r; j < r1; ++j) rank0[key[j].second] = (unsigned short)j;
    if (r1 - r > 1) {
      if (r1 - r > 4) return false;
      unsigned short g[6] = {(unsigned short)r, (unsigned short)(r1 - r), 0, 0, 0, 0};
      for (int j = r; j < r1; ++j) g[2 + j - r] = (unsigned short)key[j].second;
      groups.insert(groups.end(), g, g + 6);
    }
    r = r1;
  }
  const double kmax = (double)key[M - 1].first;
  int cnt = 0;
  for (int g = 0; g <= kCells; ++g) {
    while (cnt < M && (double)kCells * (double)key[cnt].first / kmax * (1.0 + 1e-4) < (double)g) ++cnt;
    rank0[kMaxMerged + g] = (unsigned short)cnt;
  }
  return true;
}

static inline void prof_mark(hipStream_t s) {
  if (!g_prof.on || !g_prof.sampled || g_prof.next >= g_prof.ev.size()) return;
  (void)hipEventRecord(g_prof.ev[g_prof.next++], s);
}
static inline void prof_class(int c) {
  if (g_prof.on && g_prof.sampled && g_prof.next < g_prof.ev.size()) g_prof.cls.push_back(c);
}
// The event pair of one sampled launch of class c, for a launcher that has its dispatches
// record them (hipExtLaunchKernelGGL: start of the kernel, end of the kernel), so the
// measured time is the kernel's own, as rocprofv3 reports it, without the dispatch gap an
// event packet between two kernels opens. Null events when not sampled.
static inline void prof_pair(int c, hipEvent_t* e0, hipEvent_t* e1) {
  *e0 = *e1 = nullptr;
  if (!g_prof.on || !g_prof.sampled || g_prof.next + 2 > g_prof.ev.size()) return;
  g_prof.cls.push_back(c);
  *e0 = g_prof.ev[g_prof.next++];
  *e1 = g_prof.ev[g_prof.next++];
}

// Carves the workspace in a fixed order so that size and run agree exactly.
struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base(static_cast<char*>(b)) {}
  template <class T>
  T* take(size_t n) {
    off = align_up(off, 256);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += n * sizeof(T);
    return p;
  }
};

// Per-slot quantizer search state of one job.
static void carve_view(Carver& cv, MseView& v, int nslot, int ncand) {
  v.stat = cv.take<unsigned>(4 * (size_t)nslot);
  v.sse = cv.take<unsigned long long>((size_t)nslot * ncand);
  v.h1 = cv.take<unsigned long long>((size_t)nslot * kHistRep * (ncand + 1));
  v.h2 = cv.take<unsigned long long>((size_t)nslot * kHistRep * (ncand + 1));
  v.s2 = cv.take<double>((size_t)nslot);
  v.sel = cv.take<int>((size_t)nslot * (2 + kMaxSel));
  v.ticket = cv.take<unsigned>((size_t)nslot);
  v.ready = cv.take<unsigned long long>((size_t)nslot);

}

struct AdmmPlan {
  std::vector<ProbDesc> desc;
  std::vector<GemmTile> tiles;
  std::vector<Chunk> sse_chunks, fin_chunks, hist_chunks;
  std::vector<Chunk> hist_multi;   // the same units, several per block (launches without the fused finalize)
  Chunk* d_hist_multi = nullptr;
  int nhm_big = 0;                 // hist_multi blocks of the big jobs (listed first)
  ProbDesc* d_desc = nullptr;
  GemmTile* d_tiles = nullptr;
  Chunk* d_sse = nullptr;
  Chunk* d_fin = nullptr;
  Chunk* d_hist = nullptr;
  bool split = false;            // per-iteration solve on the split fp16 planes (kSolveSplit)
  std::vector<ThinLoopUnit> thin;   // solve workgroups (32 columns each) of the thin (I <= kThinRows) factors
  ThinLoopUnit* d_thin = nullptr;
  int thin_nr = 0, thin_maxld = 0;
  unsigned short* d_rank0 = nullptr;    // merged stage-1 order (kMaxMerged), then the cell index (kCells + 2)
  unsigned short* d_groups = nullptr;   // merged stage-1 tie groups (3 kMaxMerged)
  size_t bytes = 0;
  int maxIp = 0, maxld = 0, maxldm = 0, maxnbk = 0, maxI = 0, maxR = 0;
  int ntiles_wide = 0, ntiles_big = 0, ntiles_small = 0;   // 256x128, 64x64, 32x64 tiles (in that order)
  // persistent fp32 solve (k_gemm_f32p): tiles in list order, workgroup b's list [off[b], off[b+1])
  bool f32p = false;
  bool f32t = false;   // one tile per workgroup, tile rows per problem (k_gemm_f32t)
  std::vector<int> list_off;
  int* d_list_off = nullptr;
  int nslots = 0;
  int ntiles_f32t = 0;
  bool wide = false;                                       // I > 64 factors take 256x128 tiles (k_gemm<8, 1, 3, *, 2>)
  int fin_groups = 1;             // float4 groups per thread of the finalize units
  int hist_nv = 1;
  std::vector<int> small;         // jobs with I <= kThinRows (one-block fused search + finalize)
  int* d_small = nullptr;
  int nfin_big = 0, nhist_big = 0;   // finalize / stage-1 units of the other jobs (listed first)
  bool rows_aligned = true;          // every big job's stage-1 units are whole rows (fused finalize possible)
  unsigned long long* d_ready = nullptr;   // [nprob][2] fused-finalize ready words (zeroed per run)
  unsigned* d_kctr = nullptr;        // K-split arrival counters (zeroed per run)
  size_t nkctr = 0;
  bool ksplit_par = false;           // this launch runs the K-split pieces in parallel (else serially)
  int small_groups = 0;              // float4 groups per thread of the fused kernel (0: too large)
  // persistent thin-factor loop (k_thin_loop, one team of workgroups per problem): possible
  // when every problem is thin, ld <= 1152 and the workgroups fit the CUs (64-column
  // workgroups for some ld <= 512 problems where 32-column ones would not)
  std::vector<ThinLoopUnit> tl_units;
  ThinLoopUnit* d_tl_units = nullptr;
  ThinSync* d_tl_sync = nullptr;
  bool tl_ok = false;
};

static GemmTile mk_tile(int prob, int tm, int tn, int first, int nk) {
  GemmTile t;
  std::memset(&t, 0, sizeof(t));
  t.prob = prob; t.tm = tm; t.tn = tn; t.first = first; t.nk = nk; t.bm = 0;
  t.k0 = 0; t.np = 1; t.pc = 0; t.ser = 1;
  t.P = nullptr; t.M = nullptr; t.U = nullptr; t.eP = nullptr; t.eM = nullptr; t.ld = 0; t.ldm = 0;   // set at upload
  return t;
}

// CU-balanced order of the big GEMM tiles. When every tile of a launch is resident at
// once (at most `slots` workgroups per CU), workgroup b lands on CU b mod ncu (round
// robin over the XCDs, then over each XCD's CUs; tools/gemm_timeline.py checks it), so
// the tiles at positions b, b + ncu, b + 2 ncu share one CU's MFMA pipes. Longest-first
// order alone gives some CUs three long tiles and others two; instead every tile, longest
// first, goes to the CU with the fewest K-steps that still has a free slot.
// The grid is padded with empty tiles (nk = 0: the workgroup returns at once) to a whole
// number of rounds, so every CU may take up to `slots` tiles, not only the CUs whose
// positions exist in a partial last round (C3 mode 1: 645 tiles, max CU load 90 -> 84).
static void order_tiles_for_cus(std::vector<GemmTile>& tiles, int ncu, int slots) {
  const int n = (int)tiles.size();
  if (n <= ncu || n > ncu * slots) return;
  std::vector<GemmTile> sorted = tiles;
  auto cost = [](const GemmTile& t) { return (long long)t.nk * ((t.bm > 0 ? t.bm : 64) / 32); };   // 32-row K-steps
  std::stable_sort(sorted.begin(), sorted.end(), [&](const GemmTile& a, const GemmTile& b) { return cost(a) > cost(b); });
  std::vector<std::vector<GemmTile>> bins(ncu);
  std::vector<long long> load(ncu, 0);
  // Among the least-loaded CUs, prefer the XCD (CU b mod 8) that already holds tiles of
  // the same column tile of M (they share its B panel through that XCD's L2), then of
  // the same row tile of P.
  constexpr int kXcd = 8;
  std::map<std::pair<int, int>, std::array<int, kXcd>> col_on, row_on;
  for (const GemmTile& t : sorted) {
    auto& cx = col_on[{t.prob, t.tn}];
    auto& rx = row_on[{t.prob, t.tm}];
    int best = -1;
    long long best_key = 0;
    for (int b = 0; b < ncu; ++b) {
      if ((int)bins[b].size() >= slots) continue;
      // smaller is better: load first, then affinity (column, row)
      const long long key = load[b] * 1000000LL - cx[b % kXcd] * 1000LL - rx[b % kXcd];
      if (best < 0 || key < best_key) { best = b; best_key = key; }
    }
    bins[best].push_back(t);
    load[best] += cost(t);
    cx[best % kXcd] += 1;
    rx[best % kXcd] += 1;
  }
  size_t rounds = 0;
  for (int b = 0; b < ncu; ++b) rounds = std::max(rounds, bins[b].size());
  GemmTile empty = mk_tile(0, 0, 0, 0, 0);
  tiles.assign(rounds * ncu, empty);
  for (int b = 0; b < ncu; ++b)
    for (int r = 0; r < (int)bins[b].size(); ++r) tiles[b + (size_t)r * ncu] = bins[b][r];
}

// Finalize units hold whole rows (the split solve needs each row's exponent in one pass):
// at most 1024 G elements, G in {1, 2, 4, 8}. Returns G.
static int fin_groups_for(const std::vector<ProbDesc>& desc, const std::vector<int>& jobs) {
  long long units4k = 0;
  int maxld = 0;
  for (int i : jobs) {
    units4k += ((long long)desc[i].I * desc[i].ld + kFinElems - 1) / kFinElems;
    maxld = std::max(maxld, desc[i].ld);
  }
  int g = units4k >= kFinMinUnits ? 4 : 1;   // small problem sets keep their parallelism
  while (g < 8 && 1024 * g < maxld) g *= 2;
  return g;
}

// Teams of the persistent thin-factor loop: 32-column workgroups, and while they would
// not all fit on the CUs at once, the shortest problems with ld <= 512 take 64-column ones
// (two k classes per thread, the same chains and sums: thin_loop.hip), whose per-iteration
// work (64 ld) stays below the largest team's (32 x 1152).
static bool plan_thin_teams(AdmmPlan& pl, int ncu) {
  pl.tl_units.clear();
  const int nprob = (int)pl.desc.size();
  if ((int)pl.small.size() != nprob || nprob == 0 || pl.thin_maxld > 1152) return false;
  std::vector<int> cw(nprob, 32);
  auto nwg = [&](int i) { const int ld = pl.desc[i].ld; return cw[i] == 64 ? ld / 64 + (ld % 64 ? 1 : 0) : ld / 32; };
  long long total = 0;
  for (int i = 0; i < nprob; ++i) total += nwg(i);
  const bool wide_all = g_thin_loop.load() == 2;
  while (total > ncu || wide_all) {
    int best = -1;
    for (int i = 0; i < nprob; ++i)
      if (cw[i] == 32 && pl.desc[i].ld <= 512 && pl.desc[i].ld >= 64 && (best < 0 || pl.desc[i].ld < pl.desc[best].ld))
        best = i;
    if (best < 0) {
      if (total > ncu) return false;
      break;
    }
    total -= nwg(best);
    cw[best] = 64;
    total += nwg(best);
  }
  for (const ThinLoopUnit& u0 : pl.thin) {   // the problems in the planner's order
    if (u0.col0 != 0) continue;
    const int i = u0.job, ld = pl.desc[i].ld;
    const int n = nwg(i);
    for (int c = 0, r = 0; c < ld; ++r) {
      const int w = std::min(cw[i], ld - c);
      ThinLoopUnit u;
      std::memset(&u, 0, sizeof(u));
      u.job = i; u.col0 = c; u.cw = w; u.rank = r; u.nteam = n;
      pl.tl_units.push_back(u);
      c += w;
    }
  }
  return true;
}

// The fp32 64 x 64 tile list of a plan (pl.desc, pl.split set; not f32p / f32t): whole
// tiles in problem order (XCD-aware within each problem), K-split pieces in parallel or
// folded serially, then the CU-level LPT order. part / ctr are left for the caller.
template <class WideFn>
static void build_big_tiles(AdmmPlan& pl, const std::vector<int>& order, WideFn wide_prob) {
  pl.tiles.clear();
  // The K-split pieces of a factor (fixed by its shape) run in parallel, np workgroups per
  // tile, only in a launch whose whole tiles leave CUs idle (a lone large factor, as in a
  // multi-GPU shard); otherwise one workgroup folds them serially (same bits, no hand-off).
  long long whole64 = 0;
  for (int i : order) {
    const ProbDesc& d = pl.desc[i];
    if (d.I <= kThinRows || d.Ip == 32 || wide_prob(d)) continue;
    whole64 += (long long)(d.Ip / 64) * ((d.ld + 63) / 64);
  }
  pl.ksplit_par = g_ksplit_par.load() == 2 || (g_ksplit_par.load() == 1 && whole64 <= kKsplitChipCUs);
  // A launch that fills the chip runs the pieces serially, except the `npar` longest split
  // tiles (balance): their pieces in parallel fill the gaps a CU-level LPT of whole tiles
  // leaves (C3 mode 0: 36-K-step tiles, max CU load 90 against a mean of 80).
  long long npar = pl.ksplit_par ? (1LL << 40) : 0;
  if (!pl.ksplit_par && g_ksplit_par.load() == 1 && g_ksplit_bal.load()) {
    std::vector<long long> whole;   // K-steps of every 64 x 64 tile of the launch
    std::vector<std::pair<int, int>> cand;   // (nk, np) of the split tiles, longest first
    for (int i : order) {
      const ProbDesc& d = pl.desc[i];
      if (d.I <= kThinRows || d.Ip == 32 || wide_prob(d)) continue;
      const long long nt = (long long)(d.Ip / 64) * ((d.ld + 63) / 64);
      for (long long t = 0; t < nt; ++t) whole.push_back(d.ld / 32);
      if (d.ksplit > 1)
        for (long long t = 0; t < nt; ++t) cand.push_back({d.ld / 32, d.ksplit});
    }
    npar = ksplit_balance(whole, cand, 256, f32_slots(), g_ksplit_cost.load());
  }
  long long nsplit = 0;   // split tiles emitted so far (the first npar of them run in parallel)
  for (int i : order) {
    const ProbDesc& d = pl.desc[i];
    if (d.I <= kThinRows || d.Ip == 32 || wide_prob(d)) continue;   // thin / 32-row / wide: elsewhere
    const int TM = d.Ip / 64, TN = (d.ld + 63) / 64;
    const int nk = d.ld / 32;
    for (int g0 = 0; g0 < TN; g0 += 8)
      for (int tm = 0; tm < TM; ++tm)
        for (int tn = g0; tn < std::min(TN, g0 + 8); ++tn) {
          const int np = (d.ksplit > 1 && nsplit++ < npar) ? d.ksplit : 1;
          for (int pc = 0; pc < np; ++pc) {   // parallel K-split pieces: [pc nk / np, (pc + 1) nk / np)
            const int k0 = pc * nk / np, k1 = (pc + 1) * nk / np;
            GemmTile t = mk_tile(i, tm, tn, (tm == 0 && tn == 0 && pc == 0) ? 1 : 0, k1 - k0);
            if (np > 1) {
              t.k0 = k0; t.np = np; t.pc = pc;   // (part / ctr: filled per call)
            } else {
              t.ser = d.ksplit;   // serial form (1: no K-split)
            }
            pl.tiles.push_back(t);
          }
        }
  }
  {
    // a launch of more tiles than resident slots (K-split pieces, C4) is dispatched in
    // order as slots free up: longest first (a no-op without pieces: problems are in ld order)
    if (pl.tiles.size() > 256 * 3)
      std::stable_sort(pl.tiles.begin(), pl.tiles.end(), [](const GemmTile& a, const GemmTile& b) { return a.nk > b.nk; });
    order_tiles_for_cus(pl.tiles, 256, f32_slots());
  }
}

// Memo of build_big_tiles by a hash of its inputs (bounded; cleared when full)
static std::mutex g_tile_mu;
static std::unordered_map<unsigned long long, std::pair<std::vector<GemmTile>, bool>> g_tile_cache;
static bool tile_cache_get(unsigned long long key, std::vector<GemmTile>& tiles, bool& par) {
  std::lock_guard<std::mutex> g(g_tile_mu);
  auto it = g_tile_cache.find(key);
  if (it == g_tile_cache.end()) return false;
  tiles.insert(tiles.end(), it->second.first.begin(), it->second.first.end());
  par = it->second.second;
  return true;
}
static void tile_cache_put(unsigned long long key, const std::vector<GemmTile>& tiles, bool par) {
  std::lock_guard<std::mutex> g(g_tile_mu);
  if (g_tile_cache.size() >= 64) g_tile_cache.clear();
  g_tile_cache[key] = {tiles, par};
}

static int plan_admm(const admmq_problem* probs, int nprob, int ncand, void* ws, AdmmPlan& pl, int solve_mode) {
  if (nprob <= 0 || !probs) return fail(ADMMQ_ERR_ARG, "no problems");
  if (ncand < 1) return fail(ADMMQ_ERR_ARG, "num_attempts must be >= 1");
  Carver cv(ws);
  pl.desc.resize(nprob);
  pl.thin_nr = 0;
  for (int i = 0; i < nprob; ++i)
    if (probs[i].I > 0 && probs[i].I <= kThinRows) pl.thin_nr = std::max(pl.thin_nr, probs[i].I);
  pl.split = solve_mode == kSolveSplit;
  // Wide tiles when the 64x64 tiles would take many rounds of the resident slots
  // (256 CUs x 3): then a CU's bytes per MAC matter more than the number of tiles, and
  // 256x128 tiles read 3/8 of the operand bytes per MAC (the Llama shapes of C5). The
  // element results do not depend on the tile shape (same K order per element).
  {
    long long t64 = 0;
    for (int i = 0; i < nprob; ++i)
      if (probs[i].I > 32) t64 += (long long)((probs[i].I + 63) / 64) * ((rup(std::max(probs[i].R, 1), 32) + 63) / 64);
    pl.wide = t64 >= g_wide_min_tiles.load();
  }
  auto wide_prob = [&](const ProbDesc& d) { return pl.wide && d.I > 64 && d.ksplit == 1; };
  for (int i = 0; i < nprob; ++i)   // the split finalize needs whole rows in one unit
    if (probs[i].I > kThinRows && rup(std::max(probs[i].R, 1), 32) > 8192) pl.split = false;
  for (int i = 0; i < nprob; ++i) {
    const admmq_problem& a = probs[i];
    if (a.I <= 0 || a.R <= 0) return fail(ADMMQ_ERR_ARG, "I and R must be positive");
    if ((long long)a.I * a.R > (1LL << 30)) return fail(ADMMQ_ERR_ARG, "factor too large");
    ProbDesc& d = pl.desc[i];
    std::memset(&d, 0, sizeof(d));
    d.F_user = a.F; d.G_user = a.G; d.H0_user = a.H0; d.H_out = a.H_out; d.U_user = a.U;
    d.HT_dbg = a.HT_out; d.X_dbg = a.X_out;
    d.I = a.I; d.R = a.R;
    d.ld = rup(a.R, 32);
    // K-split pieces (fp32 64 x 64 tiles only; by shape alone): such a factor never takes
    // the wide tiles, whatever its launch, so its bits stay those of its own shape
    d.ksplit = (!pl.split && g_ksplit.load() != 0 && g_f32_kernel.load() == 0 && g_gemm_ks_f32 == 1 &&
                a.I > kThinRows) ? ksplit_pieces(a.I, a.R) : 1;
    const bool f32p_prob = !pl.split && g_f32_kernel.load() != 0 && !wide_prob(d) && a.I > kThinRows;
    d.Ip = a.I <= 32 ? 32 : rup(a.I, wide_prob(d) ? kWideRows : (f32p_prob ? std::max(64, f32_tile_rows(a.I, rup(a.R, 32))) : 64));
    d.ldm = rup(a.R, 64);
    d.nbk = d.ldm / 32;
    d.nq = a.I * ((a.R + 3) / 4);
    // 32-bit element offsets inside a problem's padded buffers (admm_finalize_block)
    if ((long long)d.Ip * d.ld >= (1LL << 31)) return fail(ADMMQ_ERR_ARG, "factor too large");
    const bool thin = a.I <= kThinRows;
    d.split = (pl.split && !thin) ? 1 : 0;
    const size_t fe = (size_t)d.Ip * d.ld;
    d.Fp = cv.take<float>(fe); d.H = cv.take<float>(fe); d.U = cv.take<float>(fe);
    d.P = cv.take<float>(fe); d.X = cv.take<float>(fe); d.HT = cv.take<float>(fe);
    d.M = cv.take<float>((size_t)d.ldm * d.ldm);
    d.A64 = cv.take<double>((size_t)d.ldm * d.ldm);
    d.L64 = cv.take<double>((size_t)d.ldm * d.ldm);
    d.D64 = cv.take<double>((size_t)d.ldm * 32);
    if (d.split) {
      d.P2 = cv.take<_Float16>(2 * fe);
      d.eP = cv.take<int>(d.Ip);
      d.M2 = cv.take<_Float16>(2 * (size_t)d.ldm * d.ldm);
      d.eM = cv.take<int>(d.ldm);
    }
    if (d.ksplit > 1) {   // the partial images of every 64 x 64 tile (the counters are carved below)
      const long long nt = (long long)(d.Ip / 64) * ((d.ld + 63) / 64);
      d.kpart = cv.take<float>((size_t)nt * d.ksplit * 4096);
    }
    d.res = cv.take<double>(2 * kResRep * 4);
    d.flags = cv.take<int>(4);
    d.rho = cv.take<float>(4);
    carve_view(cv, d.mv, 2, ncand);
    d.mv.X = d.HT; d.mv.U = d.U; d.mv.rows = d.I; d.mv.cols = d.R; d.mv.ld = d.ld; d.mv.qpr = (d.R + 3) / 4;
    d.mv.nq = d.nq; d.mv.nelem = d.I * d.R; d.mv.done = d.flags;
    pl.maxIp = std::max(pl.maxIp, d.Ip); pl.maxld = std::max(pl.maxld, d.ld);
    pl.maxldm = std::max(pl.maxldm, d.ldm); pl.maxnbk = std::max(pl.maxnbk, d.nbk);
    pl.maxI = std::max(pl.maxI, d.I); pl.maxR = std::max(pl.maxR, d.R);
  }
  // GEMM tiles, longest K first (LPT over the grid); `first` marks tile (0,0).
  // 64x64 tiles (Ip > 32) first, then the 32x64 tiles of the 17..32-row factors.
  // XCD-aware order: workgroups b and b+8 share an XCD (round-robin dispatch), so the
  // row tiles that read the same B tile (one column tile tn of M) are laid out 8 apart:
  // within each group of up to 8 column tiles, positions run tm-major, tn-minor.
  pl.tiles.clear();
  std::vector<int> order(nprob);
  for (int i = 0; i < nprob; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return pl.desc[a].ld > pl.desc[b].ld; });
  // Wide tiles (kWideRows x 128, pl.wide, I > 64), placed by XCD: workgroup b runs on XCD
  // b mod 8, in order of b within the XCD. These launches have I >> R (the Llama shapes),
  // so the P row panel (kWideRows x ld) is the big operand: every row panel goes to ONE
  // XCD (least K-step load first), which runs all of its column tiles back to back, so P is
  // fetched once into that XCD's L2 instead of once per XCD (the column-major order kept
  // a column tile of M per XCD and made all 8 XCDs fetch every P panel: 3.5x the
  // algorithmic bytes at C5). Queue x fills positions x, x + 8, ...; a queue that runs
  // out early takes tiles from the tail of the longest one.
  std::vector<GemmTile> wide;
  {
    constexpr int kXcd = 8;
    std::vector<std::vector<GemmTile>> q(kXcd);
    std::vector<long long> qload(kXcd, 0);
    for (int i : order) {
      const ProbDesc& d = pl.desc[i];
      if (!wide_prob(d)) continue;
      const int TM = d.Ip / kWideRows, TN = (d.ld + 127) / 128;
      for (int tm = 0; tm < TM; ++tm) {
        const int x = (int)(std::min_element(qload.begin(), qload.end()) - qload.begin());
        for (int tn = 0; tn < TN; ++tn) q[x].push_back(mk_tile(i, tm, tn, (tm == 0 && tn == 0) ? 1 : 0, d.ld / 32));
        qload[x] += (long long)TN * (d.ld / 32);
      }
    }
    std::vector<size_t> head(kXcd, 0);
    size_t left = 0;
    for (auto& v : q) left += v.size();
    for (size_t b = 0; left > 0; ++b, --left) {
      int x = (int)(b % kXcd);
      if (head[x] >= q[x].size()) {   // exhausted: the longest remaining queue donates its last tile
        int y = 0;
        for (int z = 1; z < kXcd; ++z)
          if (q[z].size() - head[z] > q[y].size() - head[y]) y = z;
        wide.push_back(q[y].back());
        q[y].pop_back();
        continue;
      }
      wide.push_back(q[x][head[x]++]);
    }
  }
  // persistent fp32 solve: every non-thin, non-wide factor in per-workgroup lists
  pl.f32p = !pl.split && g_f32_kernel.load() == 1;
  pl.f32t = !pl.split && g_f32_kernel.load() == 2;
  pl.list_off.clear();
  pl.nslots = 0;
  if (pl.f32p) {
    std::vector<GemmTile> ft;
    for (int i : order) {
      const ProbDesc& d = pl.desc[i];
      if (d.I <= kThinRows || wide_prob(d)) continue;
      const int bm = f32_tile_rows(d.I, d.ld);
      const int TM = (d.I + bm - 1) / bm, TN = (d.ld + 63) / 64;
      for (int tm = 0; tm < TM; ++tm)
        for (int tn = 0; tn < TN; ++tn) {
          GemmTile t = mk_tile(i, tm, tn, (tm == 0 && tn == 0) ? 1 : 0, d.ld / 32);
          t.bm = bm;
          ft.push_back(t);
        }
    }
    if (!ft.empty()) {
      const int ncu = device_cus();
      plan_f32_lists(ft, pl.list_off, ncu);
      pl.nslots = ncu * kF32Slots;
    }
    pl.tiles = ft;   // the wide tiles (if any) are inserted in front below
  }
  if (pl.f32t) {
    for (int i : order) {
      const ProbDesc& d = pl.desc[i];
      if (d.I <= kThinRows || wide_prob(d)) continue;
      const int bm = f32_tile_rows(d.I, d.ld);
      const int TM = (d.I + bm - 1) / bm, TN = (d.ld + 63) / 64;
      for (int tm = 0; tm < TM; ++tm)
        for (int tn = 0; tn < TN; ++tn) {
          GemmTile t = mk_tile(i, tm, tn, (tm == 0 && tn == 0) ? 1 : 0, d.ld / 32);
          t.bm = bm;
          pl.tiles.push_back(t);
        }
    }
    order_tiles_for_cus(pl.tiles, 256, 3);
    pl.ntiles_f32t = (int)pl.tiles.size();
  }
  // K-split arrival counters: one per split tile, contiguous (zeroed at the start of every run)
  pl.nkctr = 0;
  for (int i = 0; i < nprob; ++i)
    if (pl.desc[i].ksplit > 1) pl.nkctr += (size_t)(pl.desc[i].Ip / 64) * ((pl.desc[i].ld + 63) / 64);
  pl.d_kctr = cv.take<unsigned>(std::max<size_t>(pl.nkctr, 1));
  // The 64 x 64 tile list (pieces, serial folds, CU order) is a pure function of the
  // problems' shapes and the switches: memoised, so repeated calls (prepare and run of one
  // call, every ALS sweep) skip the LPT placement; the per-call pointers are filled after.
  std::vector<size_t> ctrbase(nprob, 0);
  {
    size_t n = 0;
    for (int i : order) {
      const ProbDesc& d = pl.desc[i];
      if (d.I <= kThinRows || d.Ip == 32 || wide_prob(d) || d.ksplit <= 1) continue;
      ctrbase[i] = n;
      n += (size_t)(d.Ip / 64) * ((d.ld + 63) / 64);
    }
  }
  if (!pl.f32p && !pl.f32t) {
    unsigned long long key = 1469598103934665603ull;
    auto mix = [&](long long v) {
      for (int b = 0; b < 8; ++b) { key ^= (unsigned long long)((v >> (8 * b)) & 0xFF); key *= 1099511628211ull; }
    };
    mix(g_ksplit_par.load()); mix(g_ksplit_bal.load()); mix(g_ksplit_cost.load()); mix(f32_slots());
    for (int i : order) {
      const ProbDesc& d = pl.desc[i];
      mix(i); mix(d.I); mix(d.Ip); mix(d.ld); mix(d.ksplit); mix(wide_prob(d) ? 1 : 0);
    }
    if (!tile_cache_get(key, pl.tiles, pl.ksplit_par)) {
      build_big_tiles(pl, order, wide_prob);
      tile_cache_put(key, pl.tiles, pl.ksplit_par);
    }
    for (GemmTile& t : pl.tiles)   // this call's partial images and counters
      if (t.np > 1) {
        const ProbDesc& d = pl.desc[t.prob];
        const int TN = (d.ld + 63) / 64;
        t.part = d.kpart + (size_t)(t.tm * TN + t.tn) * t.np * 4096;
        t.ctr = pl.d_kctr + ctrbase[t.prob] + (size_t)(t.tm * TN + t.tn);
      }
  }
  std::vector<GemmTile> small;
  for (int i : order) {   // 32 x 64 tiles of the 17..32-row factors
    const ProbDesc& d = pl.desc[i];
    if (pl.f32p || pl.f32t) break;
    if (d.I <= kThinRows || d.Ip != 32) continue;
    const int TN = (d.ld + 63) / 64;
    for (int tn = 0; tn < TN; ++tn) small.push_back(mk_tile(i, 0, tn, tn == 0 ? 1 : 0, d.ld / 32));
  }
  pl.ntiles_big = (pl.f32p || pl.f32t) ? 0 : (int)pl.tiles.size();   // f32p / f32t: their own launches
  pl.ntiles_small = (int)small.size();
  pl.ntiles_wide = (int)wide.size();
  pl.tiles.insert(pl.tiles.end(), small.begin(), small.end());
  pl.tiles.insert(pl.tiles.begin(), wide.begin(), wide.end());
  // thin factors: one solve workgroup per 32 columns (thin_loop.hip), longest rows first;
  // the same list is the persistent loop's teams (rank = column block)
  pl.thin.clear();
  pl.thin_maxld = 0;
  for (int i : order) {
    const ProbDesc& d = pl.desc[i];
    if (d.I > kThinRows) continue;
    pl.thin_maxld = std::max(pl.thin_maxld, d.ld);
    for (int c = 0; c < d.ld; c += 32) {
      ThinLoopUnit u;
      std::memset(&u, 0, sizeof(u));
      u.job = i; u.col0 = c; u.cw = 32; u.rank = c / 32; u.nteam = d.ld / 32;
      pl.thin.push_back(u);
    }
  }
  pl.sse_chunks.clear();
  pl.fin_chunks.clear();
  pl.hist_chunks.clear();
  long long hist_units = 0;
  std::vector<int> big_jobs;
  for (int i = 0; i < nprob; ++i) {
    hist_units += ((long long)pl.desc[i].I * pl.desc[i].ld + kHistElems - 1) / kHistElems;
    if (pl.desc[i].I > kThinRows) big_jobs.push_back(i);
  }
  pl.fin_groups = fin_groups_for(pl.desc, big_jobs.empty() ? order : big_jobs);
  pl.hist_nv = hist_units > kHistMaxUnits ? 2 : 1;   // one round of resident stage-1 blocks
  // Stage-1 unit size of the big jobs: kHistElems x hist_nv, or smaller when that would
  // leave the one round of resident blocks (2 per CU) partly filled: C3 mode 0 had 371
  // units of ~8 k elements, so 115 CUs ran two blocks (16 k elements) and 141 one; units
  // of about total / (2 x CUs) elements give every CU the same share (unit boundaries move
  // only the order of the fp64 residual partial sums, never an element's result)
  long long big_elems = 0;
  for (int i : big_jobs) big_elems += (long long)pl.desc[i].I * pl.desc[i].ld;
  // whole-row units of at most t elements of the big jobs
  auto big_units = [&](long long t) {
    long long units = 0;
    for (int i : big_jobs) {
      const ProbDesc& d = pl.desc[i];
      const long long st = d.ld <= t ? (t / d.ld) * d.ld : t;
      units += ((long long)d.I * d.ld + st - 1) / st;
    }
    return units;
  };
  // three float4 groups per thread (k_mse_hist3<.., 3, ..>) when the units at two would
  // outnumber the fused search's resident blocks (2 per CU) and at three would not: the
  // finalize then stays in the search launch (C4: 5.7 M elements per mode, 722 units of
  // 8 k against 512 slots; without this, the separate k_finalize_admm launch)
  if (pl.hist_nv == 2 && g_fin_nv3.load() && big_units((long long)kHistElems * 2) > 2LL * device_cus() &&
      big_units((long long)kHistElems * 3) <= 2LL * device_cus())
    pl.hist_nv = 3;
  // (not with hist_nv = 1: a lone layer4 factor's 589 k elements in 512 one-row units
  // instead of 171 three-row ones made its search 22 -> 27 us - the flush atomics and the
  // ticket chain grow with the block count faster than the per-block phases shrink)
  long long hu_big = (long long)kHistElems * pl.hist_nv;
  if (pl.hist_nv >= 2 && g_even_units.load()) {
    const long long slots = 2LL * device_cus();
    int big_maxld = 0;
    for (int i : big_jobs) big_maxld = std::max(big_maxld, pl.desc[i].ld);
    for (long long t = std::max<long long>(big_maxld, (big_elems + slots - 1) / slots); t < hu_big; t += 256)
      if (big_units(t) <= slots) { hu_big = t; break; }
  }
  // stage-1 / finalize units of the small jobs (I <= kThinRows) go last: when their
  // fused one-block path runs (k_mse_small_admm), the launches take only the others
  pl.small.clear();
  pl.rows_aligned = true;
  const long long fin_cap = 1024LL * pl.fin_groups;
  for (int pass = 0; pass < 2; ++pass) {
    for (int i : order) {
      ProbDesc& d = pl.desc[i];
      if ((d.I <= kThinRows) != (pass == 1)) continue;
      if (pass == 1) pl.small.push_back(i);
      for (int q = 0; q < d.nq; q += kSseQuads) pl.sse_chunks.push_back({i, q});
      const long long tot = (long long)d.I * d.ld;
      // whole rows per unit (rows longer than a unit: plain chunks; never a split problem)
      const long long step = d.ld <= fin_cap ? (fin_cap / d.ld) * d.ld : fin_cap;
      d.fin_rows = d.ld <= fin_cap ? (int)(fin_cap / d.ld) : 0;
      for (long long e = 0; e < tot; e += step)
        pl.fin_chunks.push_back({i, (int)e, d.mv.stat, d.flags, d.HT, d.U, std::min(tot, e + step), d.H, d.Fp, d.mv.sel});
      // stage-1 units: whole rows where a row fits (the fused finalize needs them), each
      // with the job's finalize inputs; `total` is the unit's end
      const long long hu = pass == 0 ? hu_big : (long long)kHistElems * pl.hist_nv;
      const long long hstep = d.ld <= hu ? (hu / d.ld) * d.ld : hu;
      if (pass == 0 && d.ld > hu) pl.rows_aligned = false;
      int nh = 0;
      for (long long e = 0; e < tot; e += hstep, ++nh)
        pl.hist_chunks.push_back({i, (int)e, d.mv.stat, d.flags, d.HT, d.U, std::min(tot, e + hstep), d.H, d.Fp, d.mv.sel});
      d.mv.nhist = nh;
    }
    if (pass == 0) { pl.nfin_big = (int)pl.fin_chunks.size(); pl.nhist_big = (int)pl.hist_chunks.size(); }
  }
  // Without the fused finalize (the search launch cannot hold every unit at once, e.g.
  // C5: ~6800 units) every block repeats the table setup (~6 us) and the histogram flush
  // for one 8192-element unit; instead a block takes `reps` consecutive units of its job,
  // sized for about kHistMultiRounds rounds of resident blocks.
  pl.hist_multi.clear();
  pl.nhm_big = 0;
  {
    const long long nu_all = (long long)pl.hist_chunks.size();
    const int forced = g_hist_reps.load();
    const int reps = forced > 0 ? forced
                                : (int)std::max(1LL, std::min<long long>(kHistMultiMaxReps,
                                                                         nu_all / (kHistMultiRounds * kHistMaxUnits)));
    for (size_t a = 0; a < pl.hist_chunks.size();) {
      size_t b = a;   // the job's units are contiguous
      while (b < pl.hist_chunks.size() && pl.hist_chunks[b].job == pl.hist_chunks[a].job) ++b;
      const int nblk = (int)((b - a + reps - 1) / reps);
      for (size_t c = a; c < b; c += reps) {
        const size_t e = std::min(b, c + reps) - 1;
        Chunk k = pl.hist_chunks[c];
        k.reps = (int)(e - c + 1);
        k.step = (int)(pl.hist_chunks[c].total - pl.hist_chunks[c].start);   // a full unit unless it is the last
        k.total = pl.hist_chunks[e].total;
        k.nblk = nblk;
        pl.hist_multi.push_back(k);
      }
      if ((int)a < pl.nhist_big) pl.nhm_big = (int)pl.hist_multi.size();
      a = b;
    }
  }
  long long small_max = 0;
  for (int i : pl.small) small_max = std::max(small_max, (long long)pl.desc[i].I * pl.desc[i].ld);
  pl.small_groups = small_admm_groups(small_max);
  pl.d_ready = cv.take<unsigned long long>(2 * (size_t)nprob);
  for (int i = 0; i < nprob; ++i) pl.desc[i].mv.ready = pl.d_ready ? pl.d_ready + 2 * i : nullptr;
  pl.d_desc = cv.take<ProbDesc>(nprob);
  pl.d_tiles = cv.take<GemmTile>(pl.tiles.size());
  pl.d_list_off = cv.take<int>(pl.list_off.size() + 1);
  pl.d_sse = cv.take<Chunk>(pl.sse_chunks.size());
  pl.d_fin = cv.take<Chunk>(pl.fin_chunks.size());
  pl.d_hist = cv.take<Chunk>(pl.hist_chunks.size());
  pl.d_hist_multi = cv.take<Chunk>(pl.hist_multi.size());
  pl.d_small = cv.take<int>(std::max<size_t>(pl.small.size(), 1));
  pl.d_thin = cv.take<ThinLoopUnit>(pl.thin.size());
  if ((int)pl.small.size() == nprob) {   // sized by the problems alone (not by the device's CUs)
    pl.d_tl_sync = cv.take<ThinSync>(nprob);
    pl.d_tl_units = cv.take<ThinLoopUnit>(pl.thin.size());   // >= the loop's workgroups
    pl.tl_ok = plan_thin_teams(pl, device_cus());
  }
  pl.d_rank0 = cv.take<unsigned short>(kMaxMerged + kCells + 2);
  pl.d_groups = cv.take<unsigned short>(3 * kMaxMerged);
  pl.bytes = align_up(cv.off, 256);
  return ADMMQ_OK;
}

// Fingerprint of a plan's carve (FNV-1a over the byte count, the shapes and the offsets of
// each problem's buffers from the workspace base): equal iff prepare and run lay it out alike
static unsigned long long plan_fingerprint(const AdmmPlan& pl, const void* ws) {
  unsigned long long h = 1469598103934665603ull;
  auto mix = [&](long long v) {
    for (int b = 0; b < 8; ++b) { h ^= (unsigned long long)((v >> (8 * b)) & 0xFF); h *= 1099511628211ull; }
  };
  const char* base = static_cast<const char*>(ws);
  auto off = [&](const void* p) { return p ? (long long)(static_cast<const char*>(p) - base) : -1LL; };
  mix((long long)pl.bytes);
  mix((long long)pl.desc.size());
  for (const ProbDesc& d : pl.desc) {
    mix(d.I); mix(d.R); mix(d.Ip); mix(d.ld); mix(d.ldm); mix(d.split); mix(d.ksplit);
    mix(off(d.Fp)); mix(off(d.M)); mix(off(d.P2)); mix(off(d.kpart)); mix(off(d.mv.h1)); mix(off(d.flags));
  }
  mix(off(pl.d_desc)); mix(off(pl.d_tiles)); mix(off(pl.d_kctr)); mix(off(pl.d_rank0)); mix(pl.hist_nv);
  return h;
}

static int upload_admm(AdmmPlan& pl, hipStream_t s) {
  int rc;
  if ((rc = h2d(pl.d_desc, pl.desc.data(), pl.desc.size() * sizeof(ProbDesc), s))) return rc;
  for (GemmTile& t : pl.tiles) {
    const ProbDesc& d = pl.desc[t.prob];
    t.U = d.U; t.ld = d.ld; t.ldm = d.ldm;
    if (d.split) {   // the fp16 planes keep the fp32 rows' strides (in floats)
      t.P = reinterpret_cast<const float*>(d.P2); t.M = reinterpret_cast<const float*>(d.M2);
      t.eP = d.eP; t.eM = d.eM;
    } else {
      t.P = d.P; t.M = d.M;
    }
  }
  if ((rc = h2d(pl.d_tiles, pl.tiles.data(), pl.tiles.size() * sizeof(GemmTile), s))) return rc;
  if (!pl.list_off.empty() && (rc = h2d(pl.d_list_off, pl.list_off.data(), pl.list_off.size() * sizeof(int), s)))
    return rc;
  if ((rc = h2d(pl.d_sse, pl.sse_chunks.data(), pl.sse_chunks.size() * sizeof(Chunk), s))) return rc;
  if ((rc = h2d(pl.d_fin, pl.fin_chunks.data(), pl.fin_chunks.size() * sizeof(Chunk), s))) return rc;
  if ((rc = h2d(pl.d_hist, pl.hist_chunks.data(), pl.hist_chunks.size() * sizeof(Chunk), s))) return rc;
  if ((rc = h2d(pl.d_hist_multi, pl.hist_multi.data(), pl.hist_multi.size() * sizeof(Chunk), s))) return rc;
  if (!pl.thin.empty() && (rc = h2d(pl.d_thin, pl.thin.data(), pl.thin.size() * sizeof(ThinLoopUnit), s))) return rc;
  if (!pl.small.empty() && (rc = h2d(pl.d_small, pl.small.data(), pl.small.size() * sizeof(int), s))) return rc;
  return check_hip("upload");
}

__global__ void k_export_info(const ProbDesc* __restrict__ d, int n, int32_t* info) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    info[4 * i + 0] = d[i].flags[1];
    info[4 * i + 1] = d[i].flags[0];
    info[4 * i + 2] = d[i].flags[2];
    info[4 * i + 3] = d[i].flags[3];   // internal fault (fused-finalize wait timed out)
  }
}

// ---------------------------------------------------------------------------
// Standalone quantization
struct QPlan {
  std::vector<QJob> jobs;
  std::vector<Chunk> pack_chunks, stat_chunks, sse_chunks, hist_chunks;
  QJob* d_jobs = nullptr;
  Chunk* d_pack = nullptr;
  Chunk* d_stat = nullptr;
  Chunk* d_sse = nullptr;
  Chunk* d_hist = nullptr;
  unsigned short* d_rank0 = nullptr;    // merged stage-1 order (kMaxMerged), then the cell index (kCells + 2)
  unsigned short* d_groups = nullptr;   // merged stage-1 tie groups (3 kMaxMerged)
  size_t bytes = 0;
};

static int plan_quant(const admmq_qtensor* t, int n, int ncand, void* ws, QPlan& pl) {
  if (n <= 0 || !t) return fail(ADMMQ_ERR_ARG, "no tensors");
  if (ncand < 1) return fail(ADMMQ_ERR_ARG, "num_attempts must be >= 1");
  Carver cv(ws);
  pl.jobs.resize(n);
  for (int i = 0; i < n; ++i) {
    QJob& j = pl.jobs[i];
    std::memset(&j, 0, sizeof(j));
    if (t[i].rows <= 0 || t[i].cols <= 0) return fail(ADMMQ_ERR_ARG, "empty tensor");
    j.src = t[i].x; j.dst = t[i].y;
    j.rows = (int)t[i].rows; j.cols = (int)t[i].cols;
    j.ld = rup(j.cols, 4);
    if ((long long)j.rows * j.ld >= (1LL << 31)) return fail(ADMMQ_ERR_ARG, "tensor too large");
    j.nq = j.rows * (j.ld / 4);
    j.has_kw = t[i].has_minmax; j.tmin_kw = t[i].tmin; j.tmax_kw = t[i].tmax;
    j.Xp = cv.take<float>((size_t)j.rows * j.ld);   // (carved either way: the size does not depend on src)
    j.copy = !(j.cols % 4 == 0 && (reinterpret_cast<uintptr_t>(j.src) & 15) == 0);
    if (!j.copy) j.Xp = const_cast<float*>(j.src);   // read in place (only k_qpack's copy writes Xp)
    carve_view(cv, j.mv, 1, ncand);
    j.mv.X = j.Xp; j.mv.rows = j.rows; j.mv.cols = j.cols; j.mv.ld = j.ld; j.mv.qpr = j.ld / 4;
    j.mv.nq = j.nq; j.mv.nelem = j.rows * j.cols; j.mv.done = nullptr;
  }
  pl.pack_chunks.clear();
  pl.stat_chunks.clear();
  pl.sse_chunks.clear();
  pl.hist_chunks.clear();
  for (int i = 0; i < n; ++i) {
    const QJob& j = pl.jobs[i];
    const long long tot = (long long)j.rows * j.ld;
    for (long long e = 0; e < tot; e += kElemChunk) pl.pack_chunks.push_back({i, (int)e});
    pl.jobs[i].pu0 = (int)pl.stat_chunks.size();
    for (long long e = 0; e < tot; e += kPackElems) pl.stat_chunks.push_back({i, (int)e});
    pl.jobs[i].pun = (int)pl.stat_chunks.size() - pl.jobs[i].pu0;
    for (int q = 0; q < j.nq; q += kSseQuads) pl.sse_chunks.push_back({i, q});
    for (long long e = 0; e < tot; e += kHistElems) pl.hist_chunks.push_back({i, (int)e, j.mv.stat, nullptr, j.Xp, nullptr, tot});
    pl.jobs[i].mv.nhist = (int)((tot + kHistElems - 1) / kHistElems);
  }
  pl.d_jobs = cv.take<QJob>(n);
  pl.d_pack = cv.take<Chunk>(pl.pack_chunks.size());
  pl.d_stat = cv.take<Chunk>(pl.stat_chunks.size());
  for (int i = 0; i < n; ++i) pl.jobs[i].pstat = cv.take<unsigned>(3 * (size_t)pl.jobs[i].pun);
  pl.d_sse = cv.take<Chunk>(pl.sse_chunks.size());
  pl.d_hist = cv.take<Chunk>(pl.hist_chunks.size());
  pl.d_rank0 = cv.take<unsigned short>(kMaxMerged + kCells + 2);
  pl.d_groups = cv.take<unsigned short>(3 * kMaxMerged);
  pl.bytes = align_up(cv.off, 256);
  return ADMMQ_OK;
}

__global__ void k_qinit(QJob* jobs, int n, int ncand) {
  const MseView& v = jobs[blockIdx.x].mv;
  for (int c = threadIdx.x; c < ncand; c += blockDim.x) v.sse[c] = 0ull;
  for (int c = threadIdx.x; c < kHistRep * (ncand + 1); c += blockDim.x) { v.h1[c] = 0ull; v.h2[c] = 0ull; }
  if (threadIdx.x == 0) {
    v.stat[0] = 0u; v.stat[1] = 0xFFFFFFFFu; v.stat[2] = 0u; v.stat[3] = 0u;
    v.s2[0] = 0.0;
    v.ticket[0] = 0u;
  }
}

__global__ void k_copy_sse(const QJob* jobs, int ncand, unsigned long long* out) {
  for (int c = threadIdx.x; c < ncand; c += blockDim.x) out[c] = jobs[0].mv.sse[c];
}

// exhaustive: evaluate every candidate's canonical SSE (debug table / forced mode)
static int run_quant(QPlan& pl, int n, int bits, int qscheme, int ncand, hipStream_t s, bool final_pass,
                     bool exhaustive) {
  int rc;
  if ((rc = h2d(pl.d_jobs, pl.jobs.data(), n * sizeof(QJob), s))) return rc;
  if ((rc = h2d(pl.d_pack, pl.pack_chunks.data(), pl.pack_chunks.size() * sizeof(Chunk), s))) return rc;
  if ((rc = h2d(pl.d_stat, pl.stat_chunks.data(), pl.stat_chunks.size() * sizeof(Chunk), s))) return rc;
  if ((rc = h2d(pl.d_sse, pl.sse_chunks.data(), pl.sse_chunks.size() * sizeof(Chunk), s))) return rc;
  if ((rc = h2d(pl.d_hist, pl.hist_chunks.data(), pl.hist_chunks.size() * sizeof(Chunk), s))) return rc;
  hipLaunchKernelGGL(k_qinit, dim3(n), dim3(256), 0, s, pl.d_jobs, n, ncand);
  launch_qpack(pl.d_jobs, n, pl.d_stat, (int)pl.stat_chunks.size(), s);
  if (qscheme == kMse) {
    const bool all = exhaustive || !two_stage_ok(ncand, bits);
    std::vector<unsigned short> rank0, groups;
    const bool merged = !all && merged_ok(ncand, bits) && !g_legacy_stage1 &&
                        merged_tables(ncand, 1 << (bits - 1), rank0, groups);
    if (merged) {
      if ((rc = h2d(pl.d_rank0, rank0.data(), rank0.size() * 2, s))) return rc;
      if (!groups.empty() && (rc = h2d(pl.d_groups, groups.data(), groups.size() * 2, s))) return rc;
      launch_mse_hist3(nullptr, pl.d_jobs, pl.d_hist, (int)pl.hist_chunks.size(), ncand, bits, 0, pl.d_rank0,
                       pl.d_groups, (int)groups.size() / 6, 1, false, 0, 0u, s);
    } else if (!all) {
      launch_mse_hist(nullptr, pl.d_jobs, pl.d_hist, (int)pl.hist_chunks.size(), ncand, bits, 0, 1, s);
    } else {   // exhaustive: every candidate's canonical SSE over all chunks
      launch_mse_select_all(nullptr, pl.d_jobs, n, ncand, 0, s);
      launch_mse_sse(nullptr, pl.d_jobs, pl.d_sse, (int)pl.sse_chunks.size(), ncand, bits, 0, s);
    }
  }
  if (final_pass) launch_qfinal(pl.d_jobs, pl.d_pack, (int)pl.pack_chunks.size(), ncand, bits, qscheme, s);
  return check_hip("quantize");
}

}  // namespace admmq

using namespace admmq;

static int valid_scheme(int q) { return q >= 0 && q <= 3; }
static int valid_bits(int b) { return b >= 1 && b <= 16; }

static const int g_gemm_stage_env = [] {
  const char* e = std::getenv("ADMMQ_GEMM_F32_STAGE");
  if (e && *e >= '0' && *e <= '4' && e[1] == 0) g_gemm_f32_stage = *e - '0';
  const char* u = std::getenv("ADMMQ_EVEN_UNITS");   // diagnostics: 0 = kHistElems x nv stage-1 units
  if (u && u[0] == '0' && u[1] == 0) g_even_units = 0;
  const char* fc = std::getenv("ADMMQ_FIN_CAPACITY");   // diagnostics: admmq_debug_set_fin_capacity
  if (fc) g_fin_cap_override = std::atoi(fc);
  return 0;
}();

extern "C" {

int32_t admmq_version(void) { return 100; }

int32_t admmq_set_exhaustive_search(int32_t enable) {
  g_exhaustive = enable != 0;
  return ADMMQ_OK;
}

int32_t admmq_set_solve_mode(int32_t mode) {
  if (mode != kSolveF32 && mode != kSolveSplit) return fail(ADMMQ_ERR_ARG, "solve mode must be 0 (fp32) or 1 (split)");
  g_solve_mode = mode;
  return ADMMQ_OK;
}

int32_t admmq_get_solve_mode(void) { return g_solve_mode.load(); }

// diagnostics (not in include/admmq.h): 1 (default) = finalize fused into the search
// launch where its blocks are all resident, 0 = the separate finalize launch
// diagnostics: stage-1 units per block of the non-fused search launch (0 = planner's choice)
int32_t admmq_debug_set_search_units_per_block(int32_t reps) {
  if (reps < 0 || reps > 64) return fail(ADMMQ_ERR_ARG, "units per block out of range");
  g_hist_reps = reps;
  return ADMMQ_OK;
}

int32_t admmq_debug_set_fused_finalize(int32_t enable) {
  g_fused_finalize = enable != 0;
  return ADMMQ_OK;
}

// diagnostics (not in include/admmq.h): workspace bytes of the plan carved against a
// non-null base (no memory is touched), so a test can check that sizing (null base)
// and the real carve agree
size_t admmq_debug_admm_plan_bytes(const admmq_problem* probs, int32_t nprob, int32_t num_attempts, void* base) {
  AdmmPlan pl;
  if (plan_admm(probs, nprob, num_attempts, base, pl, g_solve_mode.load()) != ADMMQ_OK) return 0;
  return pl.bytes;
}

// diagnostics (not in include/admmq.h): 1 (default) = the search takes three float4 groups
// per thread where that keeps the finalize fused (planned at prepare), 0 = at most two
int32_t admmq_debug_set_fin_nv3(int32_t on) {
  if (on < 0 || on > 1) return fail(ADMMQ_ERR_ARG, "fin_nv3 must be 0 or 1");
  g_fin_nv3 = on;
  return ADMMQ_OK;
}

// diagnostics (not in include/admmq.h): resident-block budget of the fused finalize (0: the device's)
int32_t admmq_debug_set_fin_capacity(int32_t blocks) {
  if (blocks < 0) return fail(ADMMQ_ERR_ARG, "blocks must be >= 0");
  g_fin_cap_override = blocks;
  return ADMMQ_OK;
}

// diagnostics (not in include/admmq.h): the persistent thin-factor loop on / off / on with
// 64-column workgroups wherever allowed
int32_t admmq_debug_set_thin_loop(int32_t on) {
  if (on < 0 || on > 2) return fail(ADMMQ_ERR_ARG, "thin_loop: 0, 1 or 2");
  g_thin_loop = on;
  return ADMMQ_OK;
}

// diagnostics (not in include/admmq.h): polls of the fused finalize's bounded wait
// (default kFinWaitPollsDefault; a test sets 1 to force the timeout / internal-fault path)
int32_t admmq_debug_set_fin_wait_polls(uint32_t polls) {
  g_fin_wait_polls = polls ? polls : kFinWaitPollsDefault;
  return ADMMQ_OK;
}

// diagnostics (not in include/admmq.h): persistent fp32 solve on/off and its tile rule
// (f32_tile_rows; changes the bits of the factors whose tile rows change between 64 and 32)
int32_t admmq_debug_set_gemm_ks(int32_t ks) {
  if (ks != 1 && ks != 2) return fail(ADMMQ_ERR_ARG, "ks must be 1 or 2");
  g_gemm_ks_f32 = ks;
  return ADMMQ_OK;
}

// diagnostics (not in include/admmq.h): staging form of the fp32 64 x 64 tiles (same bits):
// 0 = k_gemm's global_load_lds with per-lane 64-bit addresses, 1 = k_gemm_f32b (buffer
// loads with a scalar K offset, U prefetched), 2 = k_gemm_f32b with a 2-deep
// ring, 3 = k_gemm_f32b without the U prefetch (the default: C3 mode 0 0.655 -> 0.597 us per
// 64x64 K-step per CU against 0), 4 = 3 with the waves' MFMA bursts at raised issue
// priority (s_setprio). ADMMQ_GEMM_F32_STAGE sets it at load time.
int32_t admmq_debug_set_even_units(int32_t on) {
  g_even_units = on != 0;
  return ADMMQ_OK;
}

int32_t admmq_debug_set_gemm_stage(int32_t v) {
  if (v < 0 || v > 4) return fail(ADMMQ_ERR_ARG, "stage must be 0..4");
  g_gemm_f32_stage = v;
  return ADMMQ_OK;
}

// diagnostics (not in include/admmq.h): K-split of the fp32 64 x 64 solve tiles by the
// factor's shape (1, default) or never (0; changes the bits of the factors that split)
int32_t admmq_debug_set_ksplit(int32_t on) {
  if (on < 0 || on > 1) return fail(ADMMQ_ERR_ARG, "ksplit must be 0 or 1");
  g_ksplit = on;
  return ADMMQ_OK;
}
// diagnostics: execution form of the K-split pieces (same bits): 1 = parallel where the launch
// leaves CUs idle (default), 0 = always serial (one workgroup per tile), 2 = always parallel
int32_t admmq_debug_set_ksplit_form(int32_t form) {
  if (form < 0 || form > 2) return fail(ADMMQ_ERR_ARG, "ksplit form must be 0..2");
  g_ksplit_par = form;
  return ADMMQ_OK;
}
// diagnostics: parallel pieces for CU balance in launches that fill the chip (same bits):
// on / off, and the price of a parallel piece in K-steps
int32_t admmq_debug_set_ksplit_balance(int32_t on, int32_t cost) {
  if (on < 0 || on > 1 || cost < 0 || cost > 64) return fail(ADMMQ_ERR_ARG, "ksplit balance: on 0/1, cost 0..64");
  g_ksplit_bal = on;
  g_ksplit_cost = cost;
  return ADMMQ_OK;
}
// diagnostics: the parallel-piece count the balance picks for the 64 x 64 tiles of a batch
// of (I, R) factors (fp32 form, default switches), or -1 on bad arguments
int64_t admmq_debug_ksplit_balance_count(const int32_t* IR, int32_t nprob) {
  if (!IR || nprob <= 0) return -1;
  std::vector<long long> whole;
  std::vector<std::pair<int, int>> cand;
  for (int p = 0; p < nprob; ++p) {
    const int I = IR[2 * p], R = IR[2 * p + 1];
    if (I <= 32) continue;
    const int ld = rup(R, 32), np = ksplit_pieces(I, R);
    const long long nt = (long long)((I + 63) / 64) * ((ld + 63) / 64);
    for (long long t = 0; t < nt; ++t) {
      whole.push_back(ld / 32);
      if (np > 1) cand.push_back({ld / 32, np});
    }
  }
  return ksplit_balance(whole, cand, 256, f32_slots(), g_ksplit_cost.load());
}
// diagnostics: the wide-tile threshold (64x64 tiles per launch; default 4 x 768)
int32_t admmq_debug_set_wide_min_tiles(int64_t t) {
  if (t < 0) return fail(ADMMQ_ERR_ARG, "wide min tiles must be >= 0");
  g_wide_min_tiles = t;
  return ADMMQ_OK;
}
// diagnostics: keep every candidate in the selected set S (1) or the rigorous set (0, default):
// the multi-candidate paths run every time, with the same exact answer
int32_t admmq_debug_set_sel_widen(int32_t on) {
  if (on < 0 || on > 1) return fail(ADMMQ_ERR_ARG, "sel widen must be 0 or 1");
  if (set_sel_widen_search(on) != 0 || set_sel_widen_thin(on) != 0) return check_hip("sel widen");
  return ADMMQ_OK;
}
// diagnostics: the K-split pieces the planner gives an (I, R) factor (0 on bad arguments)
int32_t admmq_debug_ksplit_pieces(int32_t I, int32_t R) {
  if (I <= 0 || R <= 0) return 0;
  return ksplit_pieces(I, R);
}

int32_t admmq_debug_set_f32_persistent(int32_t kernel, int32_t rule) {
  if (rule < 0 || rule > 3) return fail(ADMMQ_ERR_ARG, "rule must be 0..3");
  if (kernel < 0 || kernel > 2) return fail(ADMMQ_ERR_ARG, "kernel must be 0..2");
  g_f32_kernel = kernel;
  g_f32_rule = rule;
  return ADMMQ_OK;
}

// diagnostics (not in include/admmq.h): 1 = per-level stage 1, 0 = merged thresholds
int32_t admmq_debug_set_legacy_stage1(int32_t enable) {
  g_legacy_stage1 = enable != 0;
  return ADMMQ_OK;
}

int32_t admmq_profile_begin(int32_t max_launches, int32_t sample_every) {
  if (g_prof.on) return fail(ADMMQ_ERR_ARG, "profiling already active");
  if (sample_every < 1) return fail(ADMMQ_ERR_ARG, "sample_every must be >= 1");
  g_prof.every = sample_every;
  g_prof.sampled = true;
  g_prof.ev.resize(2 * (size_t)std::max(max_launches, 1));
  for (auto& e : g_prof.ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(ADMMQ_ERR_HIP, "hipEventCreate");
  g_prof.cls.clear();
  g_prof.next = 0;
  g_prof.on = true;
  return ADMMQ_OK;
}

int32_t admmq_profile_end(double* ms_per_class, int64_t* launches_per_class) {
  if (!g_prof.on) return fail(ADMMQ_ERR_ARG, "profiling not active");
  g_prof.on = false;
  g_prof.sampled = true;
  for (int c = 0; c < ADMMQ_PROF_CLASSES; ++c) { ms_per_class[c] = 0.0; launches_per_class[c] = 0; }
  const size_t pairs = std::min(g_prof.next / 2, g_prof.cls.size());
  int rc = ADMMQ_OK;
  if (pairs > 0 && hipEventSynchronize(g_prof.ev[2 * pairs - 1]) != hipSuccess) rc = fail(ADMMQ_ERR_HIP, "sync");
  for (size_t i = 0; rc == ADMMQ_OK && i < pairs; ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]) != hipSuccess) { rc = ADMMQ_ERR_HIP; break; }
    ms_per_class[g_prof.cls[i]] += ms;
    launches_per_class[g_prof.cls[i]] += 1;
  }
  for (auto& e : g_prof.ev) (void)hipEventDestroy(e);
  g_prof.ev.clear();
  g_prof.cls.clear();
  return rc;
}

const char* admmq_last_error(void) { return g_err.c_str(); }

static int check_opts(const admmq_admm_options* o) {
  if (!o) return fail(ADMMQ_ERR_ARG, "options must not be NULL");
  if (o->solve_mode != kSolveF32 && o->solve_mode != kSolveSplit)
    return fail(ADMMQ_ERR_ARG, "solve_mode must be ADMMQ_SOLVE_FP32 or ADMMQ_SOLVE_SPLIT");
  if (o->fused_finalize != 0 && o->fused_finalize != 1) return fail(ADMMQ_ERR_ARG, "fused_finalize must be 0 or 1");
  for (int r : o->reserved)
    if (r != 0) return fail(ADMMQ_ERR_ARG, "reserved option fields must be zero");
  return ADMMQ_OK;
}
static admmq_admm_options default_opts() {
  admmq_admm_options o;
  std::memset(&o, 0, sizeof(o));
  o.solve_mode = g_solve_mode.load();
  o.fused_finalize = g_fused_finalize.load() ? 1 : 0;
  return o;
}

int32_t admmq_admm_default_options(admmq_admm_options* out) {
  if (!out) return fail(ADMMQ_ERR_ARG, "options must not be NULL");
  *out = default_opts();
  return ADMMQ_OK;
}

size_t admmq_admm_workspace_size_ex(const admmq_problem* probs, int32_t nprob, int32_t num_attempts,
                                    const admmq_admm_options* opt) {
  if (check_opts(opt)) return 0;
  AdmmPlan pl;
  if (plan_admm(probs, nprob, num_attempts, nullptr, pl, opt->solve_mode) != ADMMQ_OK) return 0;
  return pl.bytes;
}

size_t admmq_admm_workspace_size(const admmq_problem* probs, int32_t nprob, int32_t num_attempts) {
  const admmq_admm_options o = default_opts();
  return admmq_admm_workspace_size_ex(probs, nprob, num_attempts, &o);
}

int32_t admmq_admm_prepare_ex(const admmq_problem* probs, int32_t nprob, int32_t num_attempts,
                              const admmq_admm_options* opt, void* workspace, size_t workspace_bytes, void* stream) {
  int rc = check_opts(opt);
  if (rc) return rc;
  AdmmPlan pl;
  rc = plan_admm(probs, nprob, num_attempts, workspace, pl, opt->solve_mode);
  if (rc) return rc;
  if (!workspace || workspace_bytes < pl.bytes) return fail(ADMMQ_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if ((rc = upload_admm(pl, s))) return rc;
  prof_class(ADMMQ_PROF_PREPARE); prof_mark(s);
  launch_rho(pl.d_desc, nprob, s);
  launch_pack(pl.d_desc, nprob, pl.maxIp, pl.maxld, s);
  launch_fill_a64(pl.d_desc, nprob, pl.maxldm, s);
  launch_spd_inverse(pl.d_desc, nprob, pl.maxnbk, s);
  if (pl.split) {   // fp16 planes of M and of the first right-hand side P
    launch_split_rows(pl.d_desc, nprob, pl.maxldm, 1, s);
    launch_split_rows(pl.d_desc, nprob, pl.maxIp, 0, s);
  }
  prof_mark(s);
  if ((rc = check_hip("admm_prepare"))) return rc;
  record_ws(workspace, opt->solve_mode, plan_fingerprint(pl, workspace));
  return ADMMQ_OK;
}

int32_t admmq_admm_prepare(const admmq_problem* probs, int32_t nprob, int32_t num_attempts, void* workspace,
                           size_t workspace_bytes, void* stream) {
  const admmq_admm_options o = default_opts();
  return admmq_admm_prepare_ex(probs, nprob, num_attempts, &o, workspace, workspace_bytes, stream);
}

int32_t admmq_admm_run_ex(const admmq_problem* probs, int32_t nprob, int32_t max_iter, float eps, int32_t bits,
                          int32_t qscheme, int32_t num_attempts, const admmq_admm_options* opt, void* workspace,
                          size_t workspace_bytes, int32_t* info, void* stream) {
  int rc = check_opts(opt);
  if (rc) return rc;
  if (!valid_scheme(qscheme)) return fail(ADMMQ_ERR_SCHEME, "unknown qscheme");
  if (!valid_bits(bits)) return fail(ADMMQ_ERR_ARG, "bits out of range");
  WsRecord wr;
  if (!recorded_ws(workspace, wr))
    return fail(ADMMQ_ERR_ARG, "admm_run: the workspace has not been prepared (admmq_admm_prepare)");
  const int rec = wr.mode;
  if (rec != opt->solve_mode) return fail(ADMMQ_ERR_ARG, "admm_run: solve_mode differs from the one its prepare used");
  AdmmPlan pl;
  rc = plan_admm(probs, nprob, num_attempts, workspace, pl, rec);
  if (rc) return rc;
  if (!workspace || workspace_bytes < pl.bytes) return fail(ADMMQ_ERR_WORKSPACE, "workspace too small");
  if (plan_fingerprint(pl, workspace) != wr.fp)
    return fail(ADMMQ_ERR_ARG, "admm_run: the problems or layout switches differ from the workspace's prepare");
  hipStream_t s = static_cast<hipStream_t>(stream);
  // descriptors carry this call's output pointers (H_out may differ from prepare's)
  if ((rc = upload_admm(pl, s))) return rc;
  if (pl.nkctr > 0 && hipMemsetAsync(pl.d_kctr, 0, pl.nkctr * sizeof(unsigned), s) != hipSuccess)
    return check_hip("K-split counter reset");
  const int nsse = (int)pl.sse_chunks.size(), nfin = (int)pl.fin_chunks.size();
  const int nhist = (int)pl.hist_chunks.size();
  const bool exhaustive = !two_stage_ok(num_attempts, bits);
  std::vector<unsigned short> rank0, groups;
  const bool merged = !exhaustive && merged_ok(num_attempts, bits) && !g_legacy_stage1 && qscheme == kMse &&
                      merged_tables(num_attempts, 1 << (bits - 1), rank0, groups);
  const int ngroups = (int)groups.size() / 6;
  if (merged) {
    if ((rc = h2d(pl.d_rank0, rank0.data(), rank0.size() * 2, s))) return rc;
    if (ngroups && (rc = h2d(pl.d_groups, groups.data(), groups.size() * 2, s))) return rc;
  }
  const bool fuse_small = qscheme == kMse && !exhaustive && merged && !pl.small.empty() &&
                          pl.small_groups > 0 && num_attempts <= 1024;
  // the big jobs' finalize inside the search launch when all its blocks fit at once
  // (with a margin of one resident block per CU: see hist3_fin_capacity)
  const int nh_big = fuse_small ? pl.nhist_big : nhist;
  // the fused paths report a broken residency assumption only through info: without it
  // they never run (include/admmq.h)
  const bool fused_allowed = opt->fused_finalize != 0 && info != nullptr;
  const bool fin_ok = fused_allowed && qscheme == kMse && !exhaustive && merged && pl.rows_aligned && nh_big > 0;
  const int cap_over = g_fin_cap_override.load();
  const int fin_cap = fin_ok ? (cap_over > 0 ? std::min(cap_over, hist3_fin_capacity(num_attempts, bits, pl.hist_nv))
                                             : hist3_fin_capacity(num_attempts, bits, pl.hist_nv))
                             : 0;
  // one whole-row unit per block, all blocks resident; a launch with more units than that
  // takes the separate finalize launch (round 3 measured blocks taking several units each
  // with the finalize fused: no faster at C4, 324 vs 318 ms per sweep, and that path held
  // the fused kernel at 40 spilled VGPRs)
  const int nfin_blocks = nh_big;
  const bool fuse_fin = fin_ok && fin_cap > 0 && nfin_blocks <= fin_cap;
  const unsigned polls = g_fin_wait_polls.load();
  if (fuse_fin && hipMemsetAsync(pl.d_ready, 0, 2 * (size_t)nprob * sizeof(unsigned long long), s) != hipSuccess)
    return check_hip("ready reset");
  // every problem thin: all iterations in one persistent launch (k_thin_loop) when the
  // fused paths are allowed (the op's fault retry turns them off) and it fits the device
  bool loop_done = false;
  if (pl.tl_ok && g_thin_loop.load() != 0 && fused_allowed && qscheme == kMse && !exhaustive && max_iter > 1 &&
      num_attempts >= 2 && num_attempts <= kTLMaxCand && bits >= 2 && bits <= 5) {
    if ((rc = h2d(pl.d_tl_units, pl.tl_units.data(), pl.tl_units.size() * sizeof(ThinLoopUnit), s))) return rc;
    if (hipMemsetAsync(pl.d_tl_sync, 0, (size_t)nprob * sizeof(ThinSync), s) != hipSuccess)
      return check_hip("thin loop reset");
    g_prof.sampled = true;
    prof_class(ADMMQ_PROF_THIN_LOOP); prof_mark(s);
    loop_done = launch_thin_loop(pl.d_desc, pl.d_tl_units, (int)pl.tl_units.size(), pl.d_tl_sync, pl.thin_nr, pl.thin_maxld,
                                 max_iter - 1, eps, num_attempts, bits, polls, device_cus(), s) == 0;
    prof_mark(s);
  }
  for (int it = 0; !loop_done && it + 1 < max_iter; ++it) {
    const int slot = it & 1;
    g_prof.sampled = it % g_prof.every == 0;
    // one event pair per launch (classes: include/admmq.h, admmq_profile_end)
    if (pl.ntiles_wide + pl.ntiles_small + pl.ntiles_big + pl.nslots + pl.ntiles_f32t > 0) {
      const bool diag = pl.nslots + pl.ntiles_f32t > 0;   // the diagnostic fp32 kernels: event packets
      hipEvent_t g0 = nullptr, g1 = nullptr;
      if (diag) { prof_class(ADMMQ_PROF_GEMM); prof_mark(s); } else { prof_pair(ADMMQ_PROF_GEMM, &g0, &g1); }
      if (pl.ntiles_wide + pl.ntiles_small + pl.ntiles_big > 0)
        launch_gemm(pl.d_desc, pl.d_tiles, pl.ntiles_wide, pl.ntiles_small, pl.ntiles_big, pl.split, slot, it, eps,
                    num_attempts, s, g0, g1, pl.ksplit_par);
      if (pl.nslots > 0)
        launch_gemm_f32p(pl.d_desc, pl.d_tiles + pl.ntiles_wide, pl.d_list_off, pl.nslots, slot, it, eps, num_attempts,
                         s);
      if (pl.ntiles_f32t > 0)
        launch_gemm_f32t(pl.d_desc, pl.d_tiles + pl.ntiles_wide, pl.ntiles_f32t, slot, it, eps, num_attempts, s);
      if (diag) prof_mark(s);
    }
    if (!pl.thin.empty()) {
      prof_class(ADMMQ_PROF_GEMM_THIN); prof_mark(s);
      launch_thin_solve(pl.d_desc, pl.d_thin, (int)pl.thin.size(), pl.thin_nr, pl.thin_maxld, slot, it, eps,
                        num_attempts, s);
      prof_mark(s);
    }
    if (qscheme == kMse) {
      // two-stage: stage 1, the selection and (when |S| > 1) stage 2 all in the hist launch
      if (!exhaustive && merged) {
        // fused finalize: one whole-row unit per block; otherwise possibly several units per block
        const int nh = fuse_fin ? nfin_blocks : (fuse_small ? pl.nhm_big : (int)pl.hist_multi.size());
        if (nh > 0) {
          hipEvent_t h0, h1;
          prof_pair(ADMMQ_PROF_SEARCH, &h0, &h1);
          launch_mse_hist3(pl.d_desc, nullptr,
                           fuse_fin ? pl.d_hist : pl.d_hist_multi, nh, num_attempts,
                           bits, slot, pl.d_rank0, pl.d_groups, ngroups, pl.hist_nv, fuse_fin, it, polls, s, h0, h1);
        }
        if (fuse_small) {   // the small jobs' search and finalize in one block each
          prof_class(ADMMQ_PROF_SMALL); prof_mark(s);
          launch_mse_small_admm(pl.d_desc, pl.d_small, (int)pl.small.size(), pl.small_groups, num_attempts, bits,
                                slot, it, pl.d_rank0, pl.d_groups, ngroups, s);
          prof_mark(s);
        }
      } else {
        prof_class(ADMMQ_PROF_SEARCH); prof_mark(s);
        if (!exhaustive) {
          launch_mse_hist(pl.d_desc, nullptr, pl.d_hist, nhist, num_attempts, bits, slot, pl.hist_nv, s);
        } else {
          launch_mse_select_all(pl.d_desc, nullptr, nprob, num_attempts, slot, s);
          launch_mse_sse(pl.d_desc, nullptr, pl.d_sse, nsse, num_attempts, bits, slot, s);
        }
        prof_mark(s);
      }
    }
    // fused: every job's finalize ran in the search launch (big jobs) or the small-job kernel
    const int nf = fuse_fin ? 0 : (fuse_small ? pl.nfin_big : nfin);
    if (nf > 0) {
      prof_class(ADMMQ_PROF_FINALIZE); prof_mark(s);
      launch_finalize_admm(pl.d_desc, pl.d_fin, nf, pl.fin_groups, num_attempts, bits, qscheme, slot, it, s);
      prof_mark(s);
    }
  }
  g_prof.sampled = true;
  if (max_iter > 1) launch_unpack(pl.d_desc, nprob, pl.maxI, pl.maxR, s);
  if (info) hipLaunchKernelGGL(k_export_info, dim3((nprob + 63) / 64), dim3(64), 0, s, pl.d_desc, nprob, info);
  return check_hip("admm_run");
}

int32_t admmq_admm_run(const admmq_problem* probs, int32_t nprob, int32_t max_iter, float eps, int32_t bits,
                       int32_t qscheme, int32_t num_attempts, void* workspace, size_t workspace_bytes,
                       int32_t* info, void* stream) {
  admmq_admm_options o = default_opts();
  const int rec = recorded_ws_mode(workspace);   // the mode this workspace was prepared with
  if (rec >= 0) o.solve_mode = rec;
  return admmq_admm_run_ex(probs, nprob, max_iter, eps, bits, qscheme, num_attempts, &o, workspace, workspace_bytes,
                           info, stream);
}

// diagnostics (not in include/admmq.h): per-block timelines of the last launches (make TRACE=1)
int32_t admmq_debug_hist_trace(unsigned long long* host, int32_t n) { return copy_hist_trace(host, n); }
int32_t admmq_debug_gemm_trace(unsigned long long* host, int32_t n) { return copy_gemm_trace(host, n); }
int32_t admmq_debug_gemm_trace2(unsigned long long* host, int32_t n) { return copy_gemm_trace2(host, n); }
int32_t admmq_debug_gemm_simd(unsigned* host, int32_t n) { return copy_gemm_simd(host, n); }
int32_t admmq_debug_setup_trace(unsigned long long* host, int32_t n) { return copy_setup_trace(host, n); }
int32_t admmq_debug_fin_trace(unsigned long long* host, int32_t n) { return copy_fin_trace(host, n); }
int32_t admmq_debug_hist_cu(unsigned long long* host, int32_t n) { return copy_hist_cu(host, n); }
int32_t admmq_debug_small_trace(unsigned long long* host, int32_t n) { return copy_small_trace(host, n); }
int32_t admmq_debug_thin_loop_trace(unsigned long long* host, int32_t n) { return copy_thin_loop_trace(host, n); }
int32_t admmq_debug_sel_stats(unsigned long long* host, int32_t reset) { return copy_sel_stats(host, reset); }
int32_t admmq_debug_check_thresholds(uint32_t seed, int32_t nsamp) { return check_thresholds(seed, nsamp); }
int32_t admmq_debug_check_cells(int32_t n, int32_t bits, uint32_t seed, int32_t nsamp, uint32_t* maxdev) {
  return check_cells(n, bits, seed, nsamp, maxdev);
}

int32_t admmq_admm_iteration_batched(const admmq_problem* probs, int32_t nprob, int32_t max_iter, float eps,
                                     int32_t bits, int32_t qscheme, int32_t num_attempts, void* workspace,
                                     size_t workspace_bytes, int32_t* info, void* stream) {
  int rc = admmq_admm_prepare(probs, nprob, num_attempts, workspace, workspace_bytes, stream);
  if (rc) return rc;
  return admmq_admm_run(probs, nprob, max_iter, eps, bits, qscheme, num_attempts, workspace, workspace_bytes, info,
                        stream);
}

// (A, C, B) around the channel dim and the broadcast output shape (outer x Lo); false:
// invalid arguments (error recorded)
static bool channel_geometry(const int64_t* shape, int32_t ndim, int32_t dim, long long& A, int& C, long long& B,
                             long long& outer, int& L, int& Lo) {
  if (!shape || ndim < 1 || ndim > 16) { fail(ADMMQ_ERR_ARG, "channel quantization needs 1 <= ndim <= 16"); return false; }
  if (dim < -ndim || dim >= ndim) { fail(ADMMQ_ERR_ARG, "dim out of range"); return false; }
  const int d = dim < 0 ? dim + ndim : dim;
  A = 1; B = 1;
  for (int k = 0; k < ndim; ++k) {
    if (shape[k] <= 0) { fail(ADMMQ_ERR_ARG, "empty tensor"); return false; }
    if (k < d) A *= shape[k];
    if (k > d) B *= shape[k];
  }
  if (shape[d] > (1 << 30) || A * B * shape[d] > (1LL << 40)) { fail(ADMMQ_ERR_ARG, "tensor too large"); return false; }
  C = (int)shape[d];
  L = (int)shape[ndim - 1];
  if (L != C && L != 1 && C != 1) {
    fail(ADMMQ_ERR_ARG, "the channel statistics do not broadcast against the last dimension");
    return false;
  }
  Lo = std::max(L, C);
  outer = A * B * C / L;
  return true;
}

size_t admmq_quantize_channel_workspace_size(const int64_t* shape, int32_t ndim, int32_t dim) {
  long long A, B, outer;
  int C, L, Lo;
  if (!channel_geometry(shape, ndim, dim, A, C, B, outer, L, Lo)) return 0;
  return align_up((size_t)3 * C * sizeof(unsigned), 256);
}

int32_t admmq_quantize_channel(const float* x, float* y, const int64_t* shape, int32_t ndim, int32_t dim, int32_t bits,
                               int32_t qscheme, void* workspace, size_t workspace_bytes, void* stream) {
  if (qscheme != ADMMQ_CHANNEL_SYMMETRIC && qscheme != ADMMQ_CHANNEL_AFFINE)
    return fail(ADMMQ_ERR_SCHEME, "qscheme must be ADMMQ_CHANNEL_SYMMETRIC or ADMMQ_CHANNEL_AFFINE");
  if (!valid_bits(bits) || bits > 31) return fail(ADMMQ_ERR_ARG, "bits out of range");
  if (!x || !y) return fail(ADMMQ_ERR_ARG, "null tensor");
  long long A, B, outer;
  int C, L, Lo;
  if (!channel_geometry(shape, ndim, dim, A, C, B, outer, L, Lo)) return ADMMQ_ERR_ARG;
  if (!workspace || workspace_bytes < (size_t)3 * C * sizeof(unsigned)) return fail(ADMMQ_ERR_WORKSPACE, "workspace too small");
  launch_channel_quant(x, y, A, C, B, outer, L, Lo, static_cast<unsigned*>(workspace), bits,
                       qscheme == ADMMQ_CHANNEL_SYMMETRIC ? kSymmetric : kAffine, static_cast<hipStream_t>(stream));
  return check_hip("quantize_channel");
}

size_t admmq_quantize_workspace_size(const admmq_qtensor* t, int32_t n, int32_t num_attempts) {
  QPlan pl;
  if (plan_quant(t, n, num_attempts, nullptr, pl) != ADMMQ_OK) return 0;
  return pl.bytes;
}

int32_t admmq_quantize_batched(const admmq_qtensor* t, int32_t n, int32_t bits, int32_t qscheme, int32_t num_attempts,
                               void* workspace, size_t workspace_bytes, void* stream) {
  if (!valid_scheme(qscheme)) return fail(ADMMQ_ERR_SCHEME, "unknown qscheme");
  if (!valid_bits(bits)) return fail(ADMMQ_ERR_ARG, "bits out of range");
  QPlan pl;
  int rc = plan_quant(t, n, num_attempts, workspace, pl);
  if (rc) return rc;
  if (!workspace || workspace_bytes < pl.bytes) return fail(ADMMQ_ERR_WORKSPACE, "workspace too small");
  return run_quant(pl, n, bits, qscheme, num_attempts, static_cast<hipStream_t>(stream), true, g_exhaustive.load());
}

int32_t admmq_mse_sse_table(const float* x, int64_t rows, int64_t cols, int32_t bits, int32_t num_attempts,
                            uint64_t* sse_out, void* workspace, size_t workspace_bytes, void* stream) {
  if (!valid_bits(bits)) return fail(ADMMQ_ERR_ARG, "bits out of range");
  admmq_qtensor t;
  std::memset(&t, 0, sizeof(t));
  t.x = x; t.y = nullptr; t.rows = rows; t.cols = cols;
  QPlan pl;
  int rc = plan_quant(&t, 1, num_attempts, workspace, pl);
  if (rc) return rc;
  if (!workspace || workspace_bytes < pl.bytes) return fail(ADMMQ_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if ((rc = run_quant(pl, 1, bits, kMse, num_attempts, s, false, true))) return rc;
  hipLaunchKernelGGL(k_copy_sse, dim3(1), dim3(256), 0, s, pl.d_jobs, num_attempts,
                     reinterpret_cast<unsigned long long*>(sse_out));
  return check_hip("mse_sse_table");
}

}  // extern "C"

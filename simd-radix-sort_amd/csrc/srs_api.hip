// srs_api.hip — C ABI (include/srs_c_api.h) and the host-side level driver.
//
// Drop-in for simd_sort::radix_sort::sort (radixSort.hpp:1761-1783): the
// caller's arrays are sorted in place; the host-pointer entry points stage
// through HBM. The driver walks the MSB levels breadth-first:
//
//   big segments (> kLocalCap keys):  plan -> scan -> tile map -> count ->
//       scan -> children -> scatter     (one launch each per level)
//   small segments:                    local LDS sort (one launch at the end)
//   finished, not in OUT:              D2D copy
//
// Two small control read-backs per level (tile/histogram totals, list
// counters) size the next launches. Everything else stays on the device.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "../../include/srs_c_api.h"
#include "srs_common.h"
#include "srs_kernels.h"

namespace srs {
namespace {

static_assert(SRS_MAX_COLS >= SRS_MAX_PAYLOADS + 1, "descriptor columns: key + payloads");
static_assert(sizeof(SortDesc) <= 4096, "SortDesc is a kernel argument (start_kernel)");

thread_local std::string g_err = "no error";
unsigned long long* g_stamp_acc = nullptr;  // srs_debug_set_stamp_buffer
uint32_t* g_lb_status = nullptr;             // srs_debug_set_lookback
unsigned long long* g_lb_err = nullptr;

// SRS_TRACE_LEVELS=1: one stderr line per global level and per local stage
// (segment counts; diagnostics only, costs one extra read-back per sort)
bool trace_levels() {
  static const bool on = [] {
    const char* e = getenv("SRS_TRACE_LEVELS");
    return e && *e && *e != '0';
  }();
  return on;
}

// SRS_NO_DIRECT_LOCAL=1: the small local class always takes the fast kernel
// (A/B runs of the direct kernel in one build)
bool direct_local_enabled() {
  static const bool on = [] {
    const char* e = getenv("SRS_NO_DIRECT_LOCAL");
    return !(e && *e && *e != '0');
  }();
  return on;
}

// the large-class direct kernel (SRS_NO_DIRECT_LOCAL2=1: the fast kernel
// takes the large class, for A/B runs)
bool direct_local2_enabled() {
  static const bool on = [] {
    const char* e = getenv("SRS_NO_DIRECT_LOCAL2");
    return !(e && *e && *e != '0');
  }();
  return on;
}

// Fewest small-class segments for which the direct kernel runs. Below it the
// fast kernel alone is cheaper: the direct kernel's hand-over list costs one
// more launch (~5-9 us) per sort, and mid-size sorts of 8-byte keys keep more
// than 52 varying bits per segment after one global level (handed over after
// one key read). tools/perf_dat.py, u64 + u64 (ns per record, fast only vs
// with the direct kernel): 2^18 0.373 / 0.427, 2^22 0.068 / 0.079, 2^24
// 0.0441 / 0.0447; at 1e9 (262144 segments) the direct kernel saves ~0.9 ms.
// Read on every call (tests lower it to reach the kernel at small sizes).
int64_t direct_min_segs() {
  const char* e = getenv("SRS_DIRECT_MIN_SEGS");
  return (e && *e) ? atoll(e) : 8192;
}

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                            \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess)                                                        \
      return fail(e_ == hipErrorOutOfMemory ? SRS_ERR_OUT_OF_MEMORY : SRS_ERR_HIP, \
                  std::string(#expr " -> ") + hipGetErrorString(e_));            \
  } while (0)

#define SRS_TRY(expr)          \
  do {                         \
    int r_ = (expr);           \
    if (r_ != SRS_OK) return r_; \
  } while (0)

int key_size_of(int kind) {
  switch (kind) {
    case SRS_KEY_U8: case SRS_KEY_I8: return 1;
    case SRS_KEY_U16: case SRS_KEY_I16: return 2;
    case SRS_KEY_U32: case SRS_KEY_I32: case SRS_KEY_F32: return 4;
    case SRS_KEY_U64: case SRS_KEY_I64: case SRS_KEY_F64: return 8;
    default: return 0;
  }
}

// ---------------------------------------------------------------------------
// kernel timing (optional; HIP events around every launch on its stream)
// ---------------------------------------------------------------------------
struct TimingRec {
  std::string name;
  std::string name2;  // optional second family (per-level names: "scatter.L1")
  hipEvent_t a, b;
  double elems;
};
struct KStat {
  int64_t launches = 0;
  double ms = 0;
  double elems = 0;
};
std::mutex g_tmu;
// 0 off, 1 every launch scope, 2 only the scatter's (bench.py's timed
// region: the roofline needs the dominant kernel's durations, and markers
// around every launch cost the step 0.05-0.2 ms)
int g_timing = 0;
bool timing_wants(const char* name) {
  return g_timing == 1 || (g_timing == 2 && strcmp(name, "scatter") == 0);
}
std::vector<TimingRec> g_pending;
std::vector<hipEvent_t> g_event_pool;
std::map<std::string, KStat> g_stats;

hipEvent_t get_event() {
  if (!g_event_pool.empty()) {
    hipEvent_t e = g_event_pool.back();
    g_event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

struct TimedScope {
  bool on = false;
  TimingRec rec;
  hipStream_t st;
  TimedScope(const char* name, double elems, hipStream_t s, int level = 0) : st(s) {
    std::lock_guard<std::mutex> lk(g_tmu);
    if (!timing_wants(name)) return;
    rec.name = name;
    if (level > 0) rec.name2 = std::string(name) + ".L" + std::to_string(level);
    rec.elems = elems;
    rec.a = get_event();
    rec.b = get_event();
    if (!rec.a || !rec.b) return;
    on = hipEventRecord(rec.a, st) == hipSuccess;
  }
  ~TimedScope() {
    if (!on) return;
    std::lock_guard<std::mutex> lk(g_tmu);
    if (hipEventRecord(rec.b, st) == hipSuccess) g_pending.push_back(rec);
  }
};

bool timing_enabled() {
  std::lock_guard<std::mutex> lk(g_tmu);
  return g_timing != 0;
}

void note_elems(const char* name, double elems, int level = 0) {
  std::lock_guard<std::mutex> lk(g_tmu);
  if (!timing_wants(name)) return;
  g_stats[name].elems += elems;
  if (level > 0) g_stats[std::string(name) + ".L" + std::to_string(level)].elems += elems;
}

void drain_timing_locked() {
  for (auto& r : g_pending) {
    float ms = 0;
    if (hipEventSynchronize(r.b) == hipSuccess &&
        hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
      KStat& k = g_stats[r.name];
      k.launches++;
      k.ms += ms;
      k.elems += r.elems;
      if (!r.name2.empty()) {
        KStat& k2 = g_stats[r.name2];
        k2.launches++;
        k2.ms += ms;
        k2.elems += r.elems;
      }
    }
    g_event_pool.push_back(r.a);
    g_event_pool.push_back(r.b);
  }
  g_pending.clear();
}

// ---------------------------------------------------------------------------
// per-device workspace (grown on demand, reused across calls)
// ---------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int mode = 0;  // how p was allocated (BigAlloc); 0 = hipMalloc
};

// ---- large-buffer allocation (the O(n) workspace: TMP, TMP2, staging) ------
// SRS_WS_ALLOC selects how the big workspace buffers are backed (diagnostics
// of the placement-dependent write rate): "malloc" (default,
// hipMalloc), "contig" (hipExtMallocWithFlags(hipDeviceMallocContiguous):
// one physically contiguous range), "vmm" (one hipMemCreate handle mapped
// into a range reserved at 1 GiB alignment), "vmm2m" / "vmmshuf" (2 MB
// handles mapped in order / in a shuffled order).
enum BigAlloc {
  ALLOC_MALLOC = 0,
  ALLOC_CONTIG = 1,
  ALLOC_VMM = 2,
  ALLOC_VMM_SHUF = 3,
  ALLOC_VMM_2M = 4,
  ALLOC_MODES = 5
};
struct VmmRec {
  std::vector<hipMemGenericAllocationHandle_t> h;
  size_t size;
};
std::mutex g_vmu;
std::map<void*, VmmRec> g_vmm;

int ws_alloc_mode() {
  const char* e = getenv("SRS_WS_ALLOC");
  if (!e || !*e || !strcmp(e, "malloc")) return ALLOC_MALLOC;
  if (!strcmp(e, "contig")) return ALLOC_CONTIG;
  if (!strcmp(e, "vmm")) return ALLOC_VMM;
  if (!strcmp(e, "vmmshuf")) return ALLOC_VMM_SHUF;
  if (!strcmp(e, "vmm2m")) return ALLOC_VMM_2M;
  return ALLOC_MALLOC;
}

bool is_vmm(int mode) { return mode == ALLOC_VMM || mode == ALLOC_VMM_SHUF || mode == ALLOC_VMM_2M; }

hipError_t big_alloc(void** p, size_t bytes, int mode) {
  *p = nullptr;
  if (mode == ALLOC_CONTIG) return hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous);
  if (!is_vmm(mode)) return hipMalloc(p, bytes);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended);
  if (e != hipSuccess) return e;
  if (gran == 0) gran = size_t(2) << 20;
  const size_t chunk_min = std::max<size_t>(gran, size_t(2) << 20);
  size_t sz = (bytes + gran - 1) / gran * gran;
  const size_t chunk = mode == ALLOC_VMM ? sz : chunk_min;
  sz = (sz + chunk - 1) / chunk * chunk;
  const size_t nch = sz / chunk;
  void* va = nullptr;
  e = hipMemAddressReserve(&va, sz, size_t(1) << 30, nullptr, 0);
  if (e != hipSuccess) return e;
  std::vector<size_t> slot(nch);
  for (size_t k = 0; k < nch; k++) slot[k] = k;
  if (mode == ALLOC_VMM_SHUF) {  // (a fixed permutation: reproducible placement)
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t k = nch; k > 1; k--) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      std::swap(slot[k - 1], slot[x % k]);
    }
  }
  VmmRec rec;
  rec.size = sz;
  for (size_t k = 0; k < nch && e == hipSuccess; k++) {
    hipMemGenericAllocationHandle_t h;
    e = hipMemCreate(&h, chunk, &prop, 0);
    if (e != hipSuccess) break;
    rec.h.push_back(h);
    e = hipMemMap((char*)va + slot[k] * chunk, chunk, 0, h, 0);
  }
  if (e == hipSuccess) {
    hipMemAccessDesc a = {};
    a.location = prop.location;
    a.flags = hipMemAccessFlagsProtReadWrite;
    e = hipMemSetAccess(va, sz, &a, 1);
  }
  if (e != hipSuccess) {
    for (size_t k = 0; k < rec.h.size(); k++) {
      (void)hipMemUnmap((char*)va + slot[k] * chunk, chunk);
      (void)hipMemRelease(rec.h[k]);
    }
    (void)hipMemAddressFree(va, sz);
    return e;
  }
  std::lock_guard<std::mutex> g(g_vmu);
  g_vmm[va] = std::move(rec);
  *p = va;
  return hipSuccess;
}

hipError_t big_free(void* p, int mode) {
  if (!p) return hipSuccess;
  if (!is_vmm(mode)) return hipFree(p);
  VmmRec r;
  {
    std::lock_guard<std::mutex> g(g_vmu);
    auto it = g_vmm.find(p);
    if (it == g_vmm.end()) return hipErrorInvalidValue;
    r = std::move(it->second);
    g_vmm.erase(it);
  }
  (void)hipDeviceSynchronize();  // (unmapping does not wait for queued kernels)
  hipError_t e = hipMemUnmap(p, r.size);
  hipError_t e2 = hipSuccess;
  for (auto& h : r.h) {
    const hipError_t x = hipMemRelease(h);
    if (x != hipSuccess) e2 = x;
  }
  hipError_t e3 = hipMemAddressFree(p, r.size);
  return e != hipSuccess ? e : e2 != hipSuccess ? e2 : e3;
}

// ---- placed allocation ------------------------------------------------------
// The scatter's and the local pass's write rate depends on where in HBM the
// written buffer sits: the same 8 GB column written by the same kernel takes
// ~6.2 or ~7.0 ms per scatter launch depending on the allocation (a probe of
// the write pattern over the buffer separates the two at ~1.5 vs ~2.1 ms per
// 8 GB). placed_alloc allocates a buffer, probes it, and while
// its probe is slower than kPlaceSlack x the fastest rate seen in this process
// takes another allocation (up to kPlaceTries, while free memory allows; the
// rejected ones are held until the choice is made, so that each try gets
// other memory), keeping the fastest. Small buffers are not probed.
constexpr size_t kPlaceMinBytes = size_t(256) << 20;
// (round 5, tools/ab_outputs.py: output columns probing at 0.19-0.20 ms per
// GB gave C1 steps of 20.9-21.0 ms, at 0.22 21.5-21.9 in the same process;
// round 4's 1.12 let the latter through)
constexpr int kPlaceTries = 6;
constexpr double kPlaceSlack = 1.04;
// before any buffer of the process has been probed: the fast class's probe
// rate on MI355X (0.187-0.202 ms per GB in round 5's runs; the slow class
// 0.22-0.25), so that the first buffer is held to the same bar
constexpr double kPlaceFirstRef = 0.200;
// One placement at a time per device (probes of two buffers on one device
// would time each other). The probe waits for the device to be idle (work
// still running would time the probe, not the placement: a probe beside the
// bench's input fill picked slow buffers, 22.4 vs 21.2 ms per C1 step) and
// runs on a private stream; the lock is per device, so a thread placing a
// buffer on its GPU never blocks another GPU's thread (a global
// lock held across that wait could deadlock one-process multi-GPU sorts
// whose peers' receives were queued behind it), and the shard reserves its
// buffers before its first message.
std::mutex g_plmu_map;                       // the map below
std::map<int, std::unique_ptr<std::mutex>> g_plmu;
std::mutex g_place_ref_mu;
double g_place_ref = 0;  // fastest probe seen, ms per GB (0: none yet)

bool placement_enabled() {
  const char* e = getenv("SRS_PLACE");  // SRS_PLACE=0: plain allocations (A/B runs)
  return !(e && *e == '0');
}

std::mutex& device_place_mutex(int dev) {
  std::lock_guard<std::mutex> g(g_plmu_map);
  auto& m = g_plmu[dev];
  if (!m) m.reset(new std::mutex());
  return *m;
}

hipError_t placed_alloc(void** p, size_t bytes, int mode) {
  if (bytes < kPlaceMinBytes || !placement_enabled()) return big_alloc(p, bytes, mode);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(device_place_mutex(dev));
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return e;
  hipStream_t ps = nullptr;
  e = hipStreamCreateWithFlags(&ps, hipStreamNonBlocking);
  if (e != hipSuccess) return e;
  void* best = nullptr;
  double best_rate = 0;
  double ref = 0;  // the fastest placement of earlier buffers
  {
    std::lock_guard<std::mutex> r(g_place_ref_mu);
    ref = g_place_ref;
  }
  double seen = ref;  // the fastest placement seen so far, this one included
  std::vector<void*> rejected;
  for (int k = 0; k < kPlaceTries; k++) {
    if (k > 0) {
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < bytes + bytes / 8) break;
    }
    void* c = nullptr;
    e = big_alloc(&c, bytes, mode);
    if (e != hipSuccess) {
      if (best) break;  // (keep what we have)
      (void)hipStreamDestroy(ps);
      return e;
    }
    const float ms = probe_write_ms(c, bytes, ps);
    const double rate = ms > 0 ? ms / ((double)bytes / 1e9) : 0;  // ms per GB
    if (rate > 0 && (seen == 0 || rate < seen)) seen = rate;
    if (!best || (rate > 0 && rate < best_rate)) {
      if (best) rejected.push_back(best);
      best = c;
      best_rate = rate;
    } else {
      rejected.push_back(c);
    }
    if (best_rate <= 0) break;  // (no probe possible: keep it)
    if (best_rate <= kPlaceSlack * (ref > 0 ? ref : kPlaceFirstRef)) break;
  }
  {
    std::lock_guard<std::mutex> r(g_place_ref_mu);
    if (seen > 0 && (g_place_ref == 0 || seen < g_place_ref)) g_place_ref = seen;
  }
  for (void* r : rejected) (void)big_free(r, mode);
  (void)hipStreamDestroy(ps);
  (void)hipGetLastError();
  *p = best;
  return hipSuccess;
}

void free_buf(DevBuf& b) {
  if (b.p) (void)big_free(b.p, b.mode);
  b = DevBuf();
}

std::mutex g_pub_amu;
std::map<void*, size_t> g_pub_allocs;  // srs_alloc_device: base -> bytes

// [p, p + bytes) lies inside one srs_alloc_device buffer (placement-probed)
bool placed_memory(const void* p, size_t bytes) {
  std::lock_guard<std::mutex> g(g_pub_amu);
  auto it = g_pub_allocs.upper_bound(const_cast<void*>(p));
  if (it == g_pub_allocs.begin()) return false;
  --it;
  const char* a = (const char*)it->first;
  return (const char*)p >= a && (const char*)p + bytes <= a + it->second;
}

// While this thread runs the multi-GPU shard's exchange (srs_shard.hip),
// workspace buffers that grow keep their old memory until the exchange is
// over: hipFree waits for the whole device, i.e. for every receive already
// queued on the communication stream -- without the transport's time limit,
// and it would serialise the round sorts behind the exchange.
thread_local bool t_defer = false;
thread_local std::vector<std::pair<void*, int>> t_deferred;

hipError_t ws_free(void* p, int mode) {
  if (!p) return hipSuccess;
  if (t_defer) {
    t_deferred.push_back({p, mode});
    return hipSuccess;
  }
  return big_free(p, mode);
}

int ensure(DevBuf& b, size_t bytes, int mode = ALLOC_MALLOC, bool placed = false) {
  if (b.bytes >= bytes && b.p) return SRS_OK;
  if (b.p) {
    HIP_TRY(ws_free(b.p, b.mode));
    b.p = nullptr;
    b.bytes = 0;
  }
  size_t want = std::max<size_t>(bytes, 256);
  if (placed) HIP_TRY(placed_alloc(&b.p, want, mode));
  else HIP_TRY(big_alloc(&b.p, want, mode));
  b.bytes = want;
  b.mode = mode;
  return SRS_OK;
}

// Growing a list that already holds live entries (copy then swap).
int ensure_keep(DevBuf& b, size_t bytes, size_t live_bytes, hipStream_t st) {
  if (b.bytes >= bytes && b.p) return SRS_OK;
  DevBuf nb;
  size_t want = std::max<size_t>(bytes, b.bytes * 2);
  HIP_TRY(hipMalloc(&nb.p, want));
  nb.bytes = want;
  if (b.p && live_bytes) HIP_TRY(hipMemcpyAsync(nb.p, b.p, live_bytes, hipMemcpyDeviceToDevice, st));
  if (b.p) {
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(ws_free(b.p, ALLOC_MALLOC));
  }
  b = nb;
  return SRS_OK;
}

// A short host wait on the sort's stream (a control read-back): polled for
// up to 20 ms, then waited for. hipStreamSynchronize's blocking wake-up
// costs ~30 us per call (the mid-size measurements), several
// times per sort; a level's kernels take a few ms at most, so the poll ends
// the wait in ~1 us.
// a spin-wait hint (x86 `pause`; elsewhere a yield)
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}

int sync_poll(hipStream_t st) {
  // (spinning for the first 200 us, then yielding the core: the shard's rank
  // threads, one per GPU, each poll their own read-backs)
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(st);
    if (q == hipSuccess) return SRS_OK;
    if (q != hipErrorNotReady) HIP_TRY(q);
    const auto dt = std::chrono::steady_clock::now() - t0;
    if (dt > std::chrono::milliseconds(20)) break;
    if (dt < std::chrono::microseconds(200)) cpu_relax();
    else std::this_thread::yield();
  }
  HIP_TRY(hipStreamSynchronize(st));
  return SRS_OK;
}

struct Workspace {
  DevBuf tmp;         // TMP data buffer (same footprint as the input)
  DevBuf tmp2;        // TMP2: AoS records as SoA slice columns (SortDesc::tmp2)
  DevBuf stage;       // device copy of host arrays (host-pointer API)
  DevBuf desc;        // SortDesc
  DevBuf big[2], local, local2, copy, fallback, fallback2, redo, redo2;
  DevBuf plan, tcount, gcount, tbase, gbase, var, sbase;
  DevBuf tile_seg, group_seg, hist, offs, gsum, gofs, scan_tmp, totals, ctr;
  DevBuf shist, lut, lut_rbits;  // balanced first level (sampled histogram, digit table)
  // stripe first level: piece sizes and tile prefixes, bucket totals, the
  // second level's tile counts and gathered tile table (GTile)
  DevBuf prun, ptile, btot, bnt, btile, nt_over, gtile, gorder;
  int64_t gorder_cap = 0;
  DevBuf mid;  // mid-size single launch: the tiles' key OR / AND, their digit counts
  DevBuf midbar;  // and its grid barrier's words (zeroed once)
  hipStream_t side = nullptr;  // medium sorts: the large local class's stream
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  ListCounters* h_ctr = nullptr;
  uint64_t* h_totals = nullptr;
  MidFlag* h_mid = nullptr;        // the mid-size launch's early answer
  unsigned long long mid_seq = 0;  // (its sequence numbers)
  // Stream order of the workspace: the last call's kernels may still be
  // queued on its stream when the call returns. `idle` is recorded on that
  // stream at the end of every call; the next call's stream waits for it
  // before its first workspace write (WsUse).
  hipEvent_t idle = nullptr;
  bool idle_pending = false;
  // single-launch small sorts (run_small): which fallback bodies ran, for
  // srs_debug_last_fallbacks. One slot per stream: small sorts skip the
  // workspace's stream-order wait, so sorts on different streams must not
  // share a slot (the map is only touched under `mu`).
  std::map<hipStream_t, DevBuf> small_taken;
  bool last_small = false;
  hipStream_t last_small_stream = nullptr;
  // one call at a time per device (calls on different devices run in
  // parallel: the multi-GPU host split sorts its shards from several threads)
  std::mutex mu;
  // Freed when the last holder lets go (srs_release_workspace only drops the
  // registry's reference, so a call that has looked the workspace up keeps
  // it alive until it returns).
  ~Workspace() {
    if (idle) {  // the last call's kernels may still read the buffers
      (void)hipEventSynchronize(idle);
      (void)hipEventDestroy(idle);
    }
    DevBuf* bufs[] = {&tmp, &tmp2, &stage, &desc, &big[0], &big[1], &local, &local2, &fallback,
                      &fallback2, &redo, &redo2, &shist, &lut, &lut_rbits, &copy, &plan, &tcount,
                      &gcount, &tbase, &gbase, &var, &sbase, &tile_seg, &group_seg, &hist, &offs,
                      &gsum, &gofs, &scan_tmp, &totals, &ctr, &prun, &ptile, &btot, &bnt, &btile,
                      &nt_over, &gtile, &gorder, &mid, &midbar};
    for (DevBuf* b : bufs) free_buf(*b);
    for (auto& t : small_taken) free_buf(t.second);
    if (h_ctr) (void)hipHostFree(h_ctr);
    if (h_totals) (void)hipHostFree(h_totals);
    if (h_mid) (void)hipHostFree(h_mid);
    if (side) (void)hipStreamDestroy(side);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    (void)hipGetLastError();  // (release-time failures leave no sticky error behind)
  }
};

std::mutex g_wmu;  // the map below
// (never destroyed: at process exit the HIP runtime -- or a profiler's tool
// library -- may already be torn down, and ~Workspace would call into it;
// a segfault after rocprofv3's finalisation. srs_release_workspace frees.)
std::map<int, std::shared_ptr<Workspace>>& g_ws = *new std::map<int, std::shared_ptr<Workspace>>;

// A workspace held for one call: the reference keeps it alive, the lock
// (taken after the lookup, released first) makes the call its only user.
struct WsLock {
  std::shared_ptr<Workspace> ref;
  std::unique_lock<std::mutex> lk;
};

int get_ws_locked(std::shared_ptr<Workspace>* out) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  auto it = g_ws.find(dev);
  if (it != g_ws.end()) {
    *out = it->second;
    return SRS_OK;
  }
  auto w = std::make_shared<Workspace>();
  HIP_TRY(hipHostMalloc((void**)&w->h_ctr, sizeof(ListCounters), hipHostMallocDefault));
  HIP_TRY(hipHostMalloc((void**)&w->h_totals, 4 * sizeof(uint64_t), hipHostMallocDefault));
  // (coherent: the mid-size kernel stores into it while the host polls)
  HIP_TRY(hipHostMalloc((void**)&w->h_mid, sizeof(MidFlag), hipHostMallocCoherent));
  memset(w->h_mid, 0, sizeof(MidFlag));
  g_ws[dev] = w;
  *out = w;
  return SRS_OK;
}

// The current device's workspace, locked for this call (lk holds a reference
// and W->mu).
int acquire_ws(Workspace** out, WsLock* lk) {
  std::shared_ptr<Workspace> w;
  {
    std::lock_guard<std::mutex> g(g_wmu);
    SRS_TRY(get_ws_locked(&w));
  }
  lk->lk = std::unique_lock<std::mutex>(w->mu);
  lk->ref = std::move(w);
  *out = lk->ref.get();
  return SRS_OK;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Holds the workspace for one call on stream `st` (under W->mu): waits on the
// device for the previous call's work on the workspace (any stream), and
// marks the end of this call's work when it goes out of scope, also on error.
struct WsUse {
  Workspace* W = nullptr;
  hipStream_t st = nullptr;
  int begin(Workspace* w, hipStream_t s) {
    W = w;
    st = s;
    if (!W->idle) HIP_TRY(hipEventCreateWithFlags(&W->idle, hipEventDisableTiming));
    if (W->idle_pending) HIP_TRY(hipStreamWaitEvent(st, W->idle, 0));
    return SRS_OK;
  }
  ~WsUse() {
    if (W && W->idle) W->idle_pending = hipEventRecord(W->idle, st) == hipSuccess;
  }
};


// ---------------------------------------------------------------------------
// the sort driver (device pointers)
// ---------------------------------------------------------------------------
struct Request {
  int64_t num;
  int kind;
  int up;
  int64_t thresh;
  bool aos;
  uint32_t elem_size;                // AoS record size
  void* in_cols[SRS_MAX_PAYLOADS + 1];
  void* out_cols[SRS_MAX_PAYLOADS + 1];
  uint32_t widths[SRS_MAX_PAYLOADS + 1];
  int ncols;                         // SoA: 1 + payloads; AoS: 1
  const int64_t* seg_bounds = nullptr;  // optional: sort [b[i], b[i+1]) independently
  int64_t nsegs = 0;
  int known_top_bits = 0;               // every segment's keys agree on these top bits
  int leaf_mode = SRS_LEAF_SORTED;      // SRS_LEAF_UNSORTED: CmpSorterNoSort
};

// SortDesc::leaf_skip of a request: CmpSorterNoSort leaves every leaf of
// <= cmpSortThreshold keys in partition order (src/cmp_sorters.hpp:66-78)
int32_t leaf_skip_of(const Request& R) {
  if (R.leaf_mode != SRS_LEAF_UNSORTED || R.thresh <= 1) return 0;
  return (int32_t)std::min<int64_t>(R.thresh, 65535);
}

void key_masks(int kind, int up, SortDesc& d) {
  const int kb = 8 * key_size_of(kind);
  const uint64_t all = kb == 64 ? ~0ull : ((1ull << kb) - 1);
  const uint64_t sb = 1ull << (kb - 1);
  uint64_t mpos = 0, mneg = 0;
  switch (kind) {
    case SRS_KEY_U8: case SRS_KEY_U16: case SRS_KEY_U32: case SRS_KEY_U64:
      mpos = mneg = 0;
      break;
    case SRS_KEY_F32: case SRS_KEY_F64:
      mpos = sb;   // non-negative: flip sign bit
      mneg = all;  // negative: flip everything
      break;
    default:       // signed
      mpos = mneg = sb;
      break;
  }
  if (!up) {
    mpos ^= all;
    mneg ^= all;
  }
  d.mpos = mpos;
  d.mneg = mneg;
  d.signbit = sb;
  d.negzero = sb;  // bit pattern of -0.0
  d.key_bits = kb;
}

// ---- balanced first level ---------------------------------------------------
// A plain first digit (the top bits) is fine for uniform keys but wastes a
// level on skewed ones: uniform floats in [-1, 1) put a quarter of all keys
// under one exponent, so three levels are needed instead of two. For large
// inputs a sampled 16-bit histogram (a few million keys in contiguous chunks)
// decides; if some top-9-bit bucket would hold more than kSkew times its
// share, the first level instead sends the keys to 512 key-range groups of
// ~equal size through a 16-bit digit table (the multi-GPU partition's LUT
// digit). Each group's children start below the key prefix its bins share.
constexpr int64_t kBalancedMinN = int64_t(1) << 24;
constexpr int kBalancedSkew = 4;
constexpr int kGroups = kMaxBins;

// *spread (also without a table): the sample's top 9 bits spread the keys
// (no bucket above kBalancedSkew times its share), so a plain first digit
// partitions them well.
// The digit table of a balanced first level, planned from the sampled
// 16-bit histogram h of the transformed keys (n input keys): mode 0 (no
// table: it would not beat the plain digit), 1 (16-bit bins -> groups,
// lut16) or 3 (split table, tab3), each group's rbits, and the predicted
// keys the next level leaves above the LDS capacity (over; over_other for
// the table not taken). Host only; srs_debug_plan_table exposes it.
struct TablePlan {
  int mode = 0;
  std::vector<int32_t> lut16, tab3, rbits;
  int groups = 0;
  double over = 0, over_other = 0;
};

void plan_table(const std::vector<uint32_t>& h, int64_t n, int key_bits, TablePlan* P) {
  *P = TablePlan();


  // (host time here is GPU idle time: every pass below looks only at the
  // non-empty bins or is a plain integer sweep)
  std::vector<uint64_t> ct(512, 0);
  std::vector<int32_t> nz;  // the non-empty bins
  nz.reserve(8192);
  for (int b0 = 0; b0 < 65536; b0 += 16) {  // (skips empty runs 16 bins at a time)
    uint64_t any = 0;
    for (int j = 0; j < 16; j++) any |= h[b0 + j];
    if (!any) continue;
    for (int b = b0; b < b0 + 16; b++)
      if (h[b]) {
        nz.push_back(b);
        ct[b >> 7] += h[b];
      }
  }
  uint64_t total = 0;
  for (uint64_t c : ct) total += c;
  if (total == 0) return;
  // Bins -> groups. Candidate groupings of the 16-bit bins into 512 key-range
  // groups; the one whose next level is predicted to leave the fewest keys in
  // buckets above the LDS capacity wins (a group's next digit splits its key
  // range evenly, so a group that mixes bins of different key density, e.g.
  // two float exponents, overfills the buckets of the denser one: C2 had 2101
  // such buckets, 5 % of its keys, taking a third and fourth level):
  //  * cumulative: group of bin b = floor(G * (keys before b + half of b) / total);
  //  * bin-aligned: a top-9-bit bin worth at least one group gets groups of its
  //    own, cut at 16-bit bins by key counts; bins worth less share groups of
  //    at most one share.
  const double to_n = (double)n / (double)total;  // sample -> input keys
  // predicted keys the next level leaves in buckets above kLocalCap (keys
  // uniform inside a 16-bit bin), or that need two more levels
  std::vector<double> qsum(kMaxBins, 0.0);
  auto overflow = [&](const std::vector<int32_t>& L) -> double {
    // a group's bins are one run of the (monotone) table
    std::vector<int32_t> fst(kGroups, -1), lst(kGroups, -1), nz0(kGroups, 0), nz1(kGroups, 0);
    std::vector<uint64_t> cnt(kGroups, 0);
    // each group's run of the (monotone) table: one forward sweep that
    // gallops over each run instead of stepping through 65,536 entries
    for (int b = 0; b < 65536;) {
      const int g = L[b];
      int step = 1;
      while (b + step < 65536 && L[b + step] == g) step <<= 1;
      int lo = b + (step >> 1), hi = std::min(b + step, 65536);  // last g in [lo, hi)
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (L[mid] == g) lo = mid;
        else hi = mid;
      }
      fst[g] = b;
      lst[g] = lo;
      b = lo + 1;
    }
    for (size_t i = 0; i < nz.size(); i++) {  // the group's non-empty bins: nz[nz0, nz1)
      const int g = L[nz[i]];
      if (!cnt[g]) nz0[g] = (int32_t)i;
      nz1[g] = (int32_t)i + 1;
      cnt[g] += h[nz[i]];
    }
    double over = 0;
    for (int g = 0; g < kGroups; g++) {
      const double len = (double)cnt[g] * to_n;
      if (len <= kLocalCap) continue;
      int bl = 0;
      while ((1 << bl) <= (fst[g] ^ lst[g])) bl++;
      int need;
      if (levels_for((int64_t)len, kLocalCapTarget, &need) > 1) {
        over += len;
        continue;
      }
      const int bits = choose_bits((int64_t)len, key_bits - (16 - bl));
      if (bits >= bl) {  // each bin splits into 2^(bits - bl) buckets
        const double lim = (double)kLocalCap * (double)(1 << (bits - bl)) / to_n;
        const double lim3 = lim + 3.0 * std::sqrt(lim);  // (sample noise)
        for (int i = nz0[g]; i < nz1[g]; i++)
          if ((double)h[nz[i]] > lim3) over += h[nz[i]] * to_n;
      } else {  // each bucket spans 2^(bl - bits) bins of the aligned range
        const int sh = bl - bits, b0 = fst[g] & ~((1 << bl) - 1);
        int qlo = kMaxBins, qhi = -1;
        for (int i = nz0[g]; i < nz1[g]; i++) {
          const int q = (nz[i] - b0) >> sh;
          qsum[q] += h[nz[i]];
          qlo = std::min(qlo, q);
          qhi = std::max(qhi, q);
        }
        const double lim = (double)kLocalCap / to_n, lim3 = lim + 3.0 * std::sqrt(lim);
        for (int q = qlo; q <= qhi; q++) {
          if (qsum[q] > lim3) over += qsum[q] * to_n;
          qsum[q] = 0;
        }
      }
    }
    return over;
  };
  // The 16-bit-table candidates (DigitLut mode 1, below) are planned only
  // when the split table's predicted overflow is not already zero (they cost
  // ~0.3 ms of host time, during which the GPU waits).
  std::vector<int32_t> lut(65536), first(kGroups, -1), last(kGroups, -1), rbits(kGroups);
  double over_best = -1;  // (-1: not evaluated)
  int buckets_used = 0, groups_used = 0;
  for (int t = 0; t < 512; t++) buckets_used += ct[t] != 0;
  // false: no table pays
  auto plan_mode1 = [&]() -> bool {
    {  // (an empty bin takes the group before it)
      double before = 0;
      int g = 0, at = 0;
      for (int b : nz) {
        std::fill(lut.begin() + at, lut.begin() + b, g);
        const int x = (int)((before + 0.5 * h[b]) * kGroups / (double)total);
        g = std::min(std::max(x, g), kGroups - 1);
        lut[b] = g;
        at = b + 1;
        before += h[b];
      }
      std::fill(lut.begin() + at, lut.end(), g);
    }
    over_best = overflow(lut);
    {
      std::vector<int32_t> la(65536, 0);
      std::vector<double> x(512);
      for (int t = 0; t < 512; t++) x[t] = (double)kGroups * (double)ct[t] / (double)total;
      for (double sc = 1.0; sc > 0.5; sc -= 0.005) {
        std::vector<int> nt(512, 0);
        int S = 0;
        double acc = 0;
        bool open = false;
        for (int t = 0; t < 512; t++) {
          if (!ct[t]) continue;
          if (x[t] < 1.0) {
            if (!open || acc + x[t] > 1.0) {
              S++;
              open = true;
              acc = 0;
            }
            acc += x[t];
            continue;
          }
          open = false;
          nt[t] = std::min(128, std::max(1, (int)std::lround(x[t] * sc)));
          S += nt[t];
        }
        if (S > kGroups) continue;
        int g = -1;
        acc = 0;
        open = false;
        for (int t = 0; t < 512; t++) {
          if (!ct[t] || x[t] < 1.0) {
            if (ct[t] && (!open || acc + x[t] > 1.0)) {
              g++;
              open = true;
              acc = 0;
            }
            acc += x[t];
            for (int j = 0; j < 128; j++) la[t * 128 + j] = std::max(g, 0);
            continue;
          }
          open = false;
          const int base = g + 1;
          double before = 0;
          int prev = 0;
          for (int j = 0; j < 128; j++) {
            const double hj = h[t * 128 + j];
            int k = (int)((before + 0.5 * hj) * nt[t] / (double)ct[t]);
            k = std::min(std::max(k, prev), nt[t] - 1);
            prev = k;
            la[t * 128 + j] = base + k;
            before += hj;
          }
          g = base + nt[t] - 1;
        }
        const double o = overflow(la);
        if (o <= over_best) {
          over_best = o;
          lut.swap(la);
        }
        break;
      }
    }
    for (int b = 0; b < 65536; b++) {
      const int g = lut[b];
      if (first[g] < 0) first[g] = b;
      last[g] = b;
    }
    // the table only pays when its groups outnumber the plain digit's
    // non-empty buckets (Gaussian int64 keys fill two 16-bit bins: both ways
    // give two buckets, and the table pass is the slower one)
    {
      std::vector<uint8_t> has(kGroups, 0);
      for (int b : nz) has[lut[b]] = 1;
      for (int g = 0; g < kGroups; g++) groups_used += has[g];
    }
    if (groups_used < 2 * buckets_used) return false;
    for (int g = 0; g < kGroups; g++) {
      const int diff = first[g] < 0 ? 0xFFFF : (first[g] ^ last[g]);
      int bl = 0;
      while ((1 << bl) <= diff) bl++;
      rbits[g] = key_bits - (16 - bl);  // the group's keys share 16 - bl top bits
    }
    return true;
  };
  // Split table (DigitLut mode 3), when its next level overflows no more:
  // each top-9-bit bin t gets 2^lg_t consecutive groups, the next lg_t key
  // bits (no group spans two bins unless both are worth less than a group).
  // One 2 KB table and one lookup per key instead of the two-level 16-bit
  // table (up to 24 KB staged per tile, two dependent lookups).
  {
    const int kb = key_bits;
    // A group's rbits bounds every key code the table sends it, so a group
    // that takes a run of empty bins, or bins of different key density (two
    // float exponents), gets a next digit that splits the keys it holds
    // badly: C2's first group took the 128 empty bins below -1.0 (rbits 31)
    // and left 1.95 M keys in one bucket, its shared tail group put one
    // exponent's keys into a sixteenth of its buckets. When they fit, every
    // non-empty bin gets groups of its own and every run of empty bins one
    // group (which stays empty unless the sample missed keys). Otherwise bins
    // worth less than one group share groups (consecutive, at most one share
    // each) and empty bins join the group before them.
    std::vector<int> lg(512, -1);     // own groups 2^lg; -1: none
    std::vector<int> share(512, -1);  // >= 0: index of the shared group it joins
    int S = 0;
    int nonempty = 0, empty_runs = 0;
    for (int t = 0; t < 512; t++) {
      nonempty += ct[t] != 0;
      empty_runs += !ct[t] && (t == 0 || ct[t - 1]);
    }
    const bool own = nonempty + empty_runs <= 512;
    if (own) {
      S = empty_runs;
      for (int t = 0; t < 512; t++) {
        if (!ct[t]) continue;
        const double x = 512.0 * (double)ct[t] / (double)total;
        int l = 0;
        while (l < 9 && (double)(2 << l) <= x * 1.4142) l++;  // (nearest power of two)
        lg[t] = l;
        S += 1 << l;
      }
    } else {
      double acc = 0;
      int nsh = 0;
      bool open = false;
      for (int t = 0; t < 512; t++) {
        if (!ct[t]) continue;
        const double x = 512.0 * (double)ct[t] / (double)total;
        if (x < 1.0) {
          if (!open || acc + x > 1.0) {
            nsh++;
            S++;
            open = true;
            acc = 0;
          }
          share[t] = nsh - 1;
          acc += x;
          continue;
        }
        open = false;
        int l = 0;
        while (l < 9 && (double)(2 << l) <= x * 1.4142) l++;  // (nearest power of two)
        lg[t] = l;
        S += 1 << l;
      }
    }
    auto gsize = [&](int t, int l) { return (double)ct[t] / (double)(1 << l); };
    {  // over budget: halve where the resulting groups stay smallest (min-heap)
      std::priority_queue<std::pair<double, int>, std::vector<std::pair<double, int>>,
                          std::greater<std::pair<double, int>>> q;
      for (int t = 0; t < 512; t++)
        if (lg[t] > 0) q.push({gsize(t, lg[t] - 1), t});
      while (S > 512 && !q.empty()) {
        const int t = q.top().second;
        q.pop();
        S -= 1 << (lg[t] - 1);
        lg[t]--;
        if (lg[t] > 0) q.push({gsize(t, lg[t] - 1), t});
      }
    }
    {  // spare budget: split the largest groups that still fit (max-heap; a
       // bin whose doubling does not fit now never will: the budget only shrinks)
      std::priority_queue<std::pair<double, int>> q;
      for (int t = 0; t < 512; t++)
        if (lg[t] >= 0 && lg[t] < 9) q.push({gsize(t, lg[t]), t});
      while (!q.empty()) {
        const int t = q.top().second;
        q.pop();
        if (S + (1 << lg[t]) > 512) continue;
        S += 1 << lg[t];
        lg[t]++;
        if (lg[t] < 9) q.push({gsize(t, lg[t]), t});
      }
    }
    // the same grouping at 16-bit resolution (representable while lg <= 7)
    bool repr = S <= 512;
    std::vector<int32_t> l3(65536, 0);
    {
      int run = 0, cur_share = -1;
      for (int t = 0; t < 512 && repr; t++) {
        if (lg[t] < 0) {
          int g;
          if (own) {  // (an empty bin: its run's group)
            g = (t == 0 || ct[t - 1]) ? run++ : run - 1;
          } else if (share[t] >= 0 && share[t] != cur_share) {
            cur_share = share[t];
            g = run++;
          } else {
            g = run > 0 ? run - 1 : 0;
          }
          for (int j = 0; j < 128; j++) l3[t * 128 + j] = g;
          continue;
        }
        if (lg[t] > 7) {
          repr = false;
          break;
        }
        for (int j = 0; j < 128; j++) l3[t * 128 + j] = run + (j >> (7 - lg[t]));
        run += 1 << lg[t];
      }
    }
    const double over3 = repr ? overflow(l3) : 1e300;
    const char* force = getenv("SRS_TABLE");  // (A/B runs: "1" or "3" forces the table kind)
    const bool forced = force && *force;
    const bool early = !forced && repr && over3 == 0 &&
                       S - (own ? empty_runs : 0) >= 2 * buckets_used;
    if (!early && !plan_mode1()) return;
    const bool take3 = forced ? (*force == '3' && repr) : (early || (repr && over3 <= over_best));
    if (take3) {
      // entry t: first group (bits 0..15) | lg (16..23); shared and empty
      // bins: the group (lg 0)
      std::vector<int32_t> tab(512);
      std::vector<uint64_t> glo(kGroups, ~0ull), ghi(kGroups, 0);
      const int unit = kb - 9;  // key bits below the top 9
      for (int t = 0; t < 512; t++) {
        const uint64_t t0 = (uint64_t)t << unit;
        const int l = lg[t] < 0 ? 0 : lg[t];
        const int g0 = l3[t * 128];
        tab[t] = g0 | (l << 16);
        const int sub = unit - l;
        for (int j = 0; j < (1 << l); j++) {
          const uint64_t a0 = t0 + ((uint64_t)j << sub);
          glo[g0 + j] = std::min(glo[g0 + j], a0);
          ghi[g0 + j] = std::max(ghi[g0 + j], a0 + ((uint64_t(1) << sub) - 1));
        }
      }
      for (int g = 0; g < kGroups; g++) {
        if (glo[g] > ghi[g]) {
          rbits[g] = kb;  // (no keys)
          continue;
        }
        const uint64_t x = glo[g] ^ ghi[g];
        rbits[g] = x ? 64 - __builtin_clzll(x) : 0;
      }
      P->mode = 3;
      P->tab3 = tab;
      P->rbits = rbits;
      P->groups = S;
      P->over = over3;
      P->over_other = over_best;
      return;
    }
    P->over_other = over3;
  }
  P->mode = 1;
  P->lut16 = lut;
  P->rbits = rbits;
  P->groups = groups_used;
  P->over = over_best;
}

// *clusters (SoA only): the sampled keys form at most kMaxRanges clusters of
// at most kClusterSpan adjacent 16-bit bins each (e.g. the reference's
// Gaussian keys: one cluster around 0 for signed keys, two at both ends of
// the range for unsigned ones): a range level decides (plan_range_level), no
// digit table. Empty otherwise.
struct KeyCluster {
  int b0, b1;    // first and last sampled 16-bit bin
  uint64_t cnt;  // sampled keys
};
constexpr int kClusterGap = 4096;  // bins between two clusters
constexpr int kClusterSpan = 256;  // bins a cluster may cover

int plan_balanced_level(Workspace* W, const Request& R, const SortDesc& d, bool* use,
                        int* lut_entries, int* lut_mode, hipStream_t st, bool* spread,
                        std::vector<KeyCluster>* clusters) {
  *use = false;
  *lut_mode = 1;
  *spread = false;
  clusters->clear();
  const int ks = key_size_of(R.kind);
  const int64_t n = R.num;
  if (R.nsegs > 0 || n < kBalancedMinN || ks < 4) return SRS_OK;
  const int64_t blocks = std::min<int64_t>(kSampleMaxChunks, n / kSampleChunk);
  const int64_t stride = n / blocks;
  // shist: the 64K-bin histogram, then the workgroups' partial rows
  SRS_TRY(ensure(W->shist, 65536 * sizeof(uint32_t) + sample_partial_bytes()));
  // (AoS records: the key at offset 0 of each record)
  if (!launch_sample_hist16(R.in_cols[0], ks, R.aos ? (int)R.elem_size : ks, n, stride,
                            kSampleChunk, blocks, d.mpos, d.mneg,
                            (uint32_t*)W->shist.p + 65536, (uint32_t*)W->shist.p, st))
    return fail(SRS_ERR_INTERNAL, "sample histogram: too many keys per workgroup");
  std::vector<uint32_t> h(65536);
  HIP_TRY(hipMemcpyAsync(h.data(), W->shist.p, h.size() * 4, hipMemcpyDeviceToHost, st));
  SRS_TRY(sync_poll(st));
  uint64_t total = 0, top9max = 0;
  for (int b = 0; b < 512; b++) {
    uint64_t t = 0;
    for (int j = 0; j < 128; j++) t += h[b * 128 + j];
    total += t;
    top9max = std::max(top9max, t);
  }
  if (total == 0) return SRS_OK;
  // (not with canon_zero: the range level's exact min / max are taken over
  // the raw transformed keys, while its passes map -0.0 onto +0.0's code,
  // which can lie outside them)
  if (!R.aos && !d.canon_zero) {
    std::vector<KeyCluster> cl;
    bool ok = true;
    for (int b = 0; b < 65536 && ok; b++) {  // (stops at the first cluster too many or too wide)
      if (!h[b]) continue;
      if (cl.empty() || b - cl.back().b1 > kClusterGap) cl.push_back(KeyCluster{b, b, 0});
      cl.back().b1 = b;
      cl.back().cnt += h[b];
      ok = (int)cl.size() <= kMaxRanges && cl.back().b1 - cl.back().b0 < kClusterSpan;
    }
    if (ok) {
      *clusters = cl;
      return SRS_OK;
    }
  }
  if (top9max * 512 <= (uint64_t)kBalancedSkew * total) {
    *spread = true;
    return SRS_OK;
  }
  if (R.aos) return SRS_OK;  // (the digit table is not used for AoS records)
  TablePlan P;
  plan_table(h, n, d.key_bits, &P);
  if (trace_levels() && P.mode)
    fprintf(stderr, "[srs] digit table mode %d: %d groups, predicted overflow %.0f keys (other "
            "table %.0f)\n", P.mode, P.groups, P.over, P.over_other);
  if (P.mode == 0) return SRS_OK;
  std::vector<int32_t>& rbits = P.rbits;
  if (P.mode == 3) {
    SRS_TRY(ensure(W->lut, 512 * sizeof(int32_t)));
    SRS_TRY(ensure(W->lut_rbits, kGroups * sizeof(int32_t)));
    HIP_TRY(hipMemcpyAsync(W->lut.p, P.tab3.data(), 512 * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(W->lut_rbits.p, rbits.data(), rbits.size() * 4, hipMemcpyHostToDevice,
                           st));
    HIP_TRY(hipStreamSynchronize(st));  // the host vectors go out of scope
    *lut_entries = 1024;  // (u16 units)
    *lut_mode = 3;
    *use = true;
    return SRS_OK;
  }
  const std::vector<int32_t>& lut = P.lut16;
  // two-level u16 table (DigitLut mode 1): a 12-bit bin whose 16 sub-bins
  // fall into one group maps straight to it; a split bin points to 16 entries
  std::vector<uint16_t> t2(4096);
  for (int B = 0; B < 4096; B++) {
    bool same = true;
    for (int j = 1; j < 16; j++) same &= lut[B * 16 + j] == lut[B * 16];
    if (same) {
      t2[B] = (uint16_t)lut[B * 16];
    } else {
      const int idx = (int)(t2.size() - 4096) / 16;
      t2[B] = (uint16_t)(0x8000 | idx);
      for (int j = 0; j < 16; j++) t2.push_back((uint16_t)lut[B * 16 + j]);
    }
  }
  if ((int)t2.size() > kLdsLutEntries) return fail(SRS_ERR_INTERNAL, "digit table too large");
  *lut_entries = (int)t2.size();
  SRS_TRY(ensure(W->lut, align_up(t2.size() * sizeof(uint16_t), 16)));  // staged in 16-byte loads
  SRS_TRY(ensure(W->lut_rbits, kGroups * sizeof(int32_t)));
  HIP_TRY(hipMemcpyAsync(W->lut.p, t2.data(), t2.size() * 2, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(W->lut_rbits.p, rbits.data(), rbits.size() * 4, hipMemcpyHostToDevice,
                         st));
  HIP_TRY(hipStreamSynchronize(st));  // the host vectors go out of scope
  *use = true;
  return SRS_OK;
}

// The tile-pair scatter (scatter_pair_kernel): where it
// pays, as flags: 1 on plain-digit levels, 2 also on small-digit-table
// levels, 4 not on the first level. Measured in one process, arms
// alternated (tools/ab_inproc.py, profiles/r05/): C1 21.34 -> 20.94 ms per
// step (both levels), C2 17.60 -> 16.92 (both levels, with the 4-byte keys'
// digits staged: its digit-table first level 5.29 -> 4.99 ms per launch, the
// plain second 5.42 -> 5.06; before the staging the table level lost, 5.18
// -> 5.89), C3's second level 6.21 -> 5.98 but its first (whole 16-byte
// records read with a stride) 6.14 -> 6.31. Default: plain-digit levels,
// small digit tables with 4-byte keys, AoS records from the second level on.
// SRS_PAIR_TILES (A/B runs): 0 off, 1 every plain-digit level, 3 every
// supported level, 2 (or unset) the default.
int pair_tiles_mode(const SortDesc& d, int ks, bool aos_slices) {
  const char* e = getenv("SRS_PAIR_TILES");
  const int mode = e && *e ? atoi(e) : 2;
  if (mode == 0 || d.canon_zero || (ks != 4 && ks != 8)) return 0;
  // (the kernel holds column 0 in a register of the key's width: an AoS
  // record wider than its key, e.g. DataElement<float, uint32>, is not for it)
  const bool shape = d.cols[0].width == (uint32_t)ks &&
                     (d.pair ? ks == 4 && d.ncols == 3 : d.ncols <= 2);
  if (!shape) return 0;
  if (mode == 3) return 1 | 2;
  if (mode == 1) return 1;
  return aos_slices ? (1 | 4) : ks == 4 ? (1 | 2) : 1;
}

struct LevelState {
  int64_t nbig, n_local, n_local2, n_copy;
  int cur;
  int ncols;               // columns moved with the keys (SortDesc::ncols)
  int tmp2;                // SortDesc::tmp2
  int64_t known_len = -1;  // the length of the single big segment, when the host knows it
  int pair_tiles = 0;      // the scatter takes two count tiles per workgroup (pair_tiles_mode)
  int level = 0;           // global levels run so far (per-level timing names)
};

// One global MSB level over every large segment in W->big[S.cur]:
// plan -> bases -> count -> offsets + children -> scatter. Children go to
// W->big[S.cur ^ 1] / the local lists / the copy list; S is updated from the
// device counters. force_bits / lut: partition passes (srs_partition_device).
// How a level reads and hands on its segments: mode 0 plain; 1 a stripe
// level (its segments are stripes of the input, partitioned each on its own;
// the next level's segments are the buckets, read through a gathered tile
// table); 2 that gathered level. See GTile (srs_common.h).
struct LevelMode {
  int mode = 0;
  const GTile* gt = nullptr;        // mode 2
  const int32_t* nt_over = nullptr; // mode 2: tiles per segment
  const int32_t* torder = nullptr;  // mode 2: the count's tile order (stripe-major)
  int key_bits = 0;                 // mode 1
  bool home = false;                // every bucket of this level is final: scatter to OUT
};

// lut: 0 a plain digit, 1 a digit table of any kind, 2 a small kind (key
// ranges, split table: the kernels with the small LDS table)
int run_level(Workspace* W, int ks, const SortDesc* d_desc, LevelState& S, int force_bits,
              int lut, hipStream_t st, const int32_t* lut_rbits = nullptr,
              const LevelMode& M = LevelMode()) {
  const int64_t nbig = S.nbig;
  ListCounters* d_ctr = (ListCounters*)W->ctr.p;
  uint64_t* d_totals = (uint64_t*)W->totals.p;
  // ---- plan + tile / scan-group bases
  SRS_TRY(ensure(W->plan, nbig * sizeof(SegPlan)));
  SRS_TRY(ensure(W->tcount, nbig * 8));
  SRS_TRY(ensure(W->gcount, nbig * 8));
  SRS_TRY(ensure(W->tbase, nbig * 8));
  SRS_TRY(ensure(W->gbase, nbig * 8));
  SRS_TRY(ensure(W->var, nbig * 16));  // the segments' key OR, then their key AND
  SRS_TRY(ensure(W->sbase, (size_t)nbig * kMaxBins * 8));
  SRS_TRY(ensure(W->scan_tmp, scan_temp_elems(nbig) * 8));
  SegPlan* plan = (SegPlan*)W->plan.p;
  unsigned long long* var = (unsigned long long*)W->var.p;
  const bool small_plan = nbig <= kPlanSmallMax;
  if (small_plan) {
    TimedScope ts("plan", (double)nbig, st);
    launch_plan_small((Seg*)W->big[S.cur].p, nbig, plan, (int64_t*)W->tbase.p,
                      (int64_t*)W->gbase.p, var, d_totals, &d_ctr->n_big, force_bits,
                      S.tmp2 | (M.home ? 2 : 0), st, M.nt_over);
  } else {
    TimedScope ts("plan", (double)nbig, st);
    HIP_TRY(hipMemsetAsync(d_totals + 3, 0, sizeof(uint64_t), st));
    launch_plan((Seg*)W->big[S.cur].p, nbig, plan, (int64_t*)W->tcount.p,
                (int64_t*)W->gcount.p, var, d_totals + 3, force_bits, S.tmp2 | (M.home ? 2 : 0),
                st, M.nt_over);
    launch_excl_scan((uint64_t*)W->tcount.p, (uint64_t*)W->tbase.p, nbig,
                     (uint64_t*)W->scan_tmp.p, d_totals + 0, st);
    launch_excl_scan((uint64_t*)W->gcount.p, (uint64_t*)W->gbase.p, nbig,
                     (uint64_t*)W->scan_tmp.p, d_totals + 1, st);
    launch_plan_bases(plan, nbig, (int64_t*)W->tbase.p, (int64_t*)W->gbase.p, st);
  }
  int64_t ntiles, ngroups;
  uint64_t level_keys;
  if (nbig == 1 && S.known_len >= 0) {
    // the first level of a plain sort: the sizes follow from n (make_plan's
    // formulas), so no read-back and no host wait
    level_keys = (uint64_t)S.known_len;
    ntiles = (S.known_len + kTile - 1) / kTile;
    ngroups = (ntiles + kScanGroup - 1) / kScanGroup;
  } else {
    HIP_TRY(hipMemcpyAsync(W->h_totals, d_totals, 4 * sizeof(uint64_t),
                           hipMemcpyDeviceToHost, st));
    SRS_TRY(sync_poll(st));
    ntiles = (int64_t)W->h_totals[0];
    ngroups = (int64_t)W->h_totals[1];
    level_keys = W->h_totals[3];
  }
  S.known_len = -1;
  const int lv = ++S.level;
  const double level_elems = (double)level_keys;
  note_elems("count", level_elems, lv);
  note_elems("scatter", level_elems, lv);

  SRS_TRY(ensure(W->tile_seg, ntiles * 4));
  SRS_TRY(ensure(W->group_seg, ngroups * 4));
  SRS_TRY(ensure(W->hist, (size_t)ntiles * kMaxBins * 2));
  // u16 tile counts; u32 tile offsets when every segment of the level is
  // < 2^32 keys (all of them are when the level is), else u64
  const bool offs32 = level_keys < (1ull << 32);
  SRS_TRY(ensure(W->offs, (size_t)ntiles * kMaxBins * (offs32 ? 4 : 8)));
  // (+ the super-group rows of a one-segment level's scan, launch_offsets)
  const int64_t grows = ngroups + super_rows(ngroups);
  SRS_TRY(ensure(W->gsum, (size_t)grows * kMaxBins * 4));
  SRS_TRY(ensure(W->gofs, (size_t)grows * kMaxBins * 8));
  int32_t* tile_seg = (int32_t*)W->tile_seg.p;
  int32_t* group_seg = (int32_t*)W->group_seg.p;
  launch_seg_map2((int64_t*)W->tbase.p, ntiles, tile_seg, (int64_t*)W->gbase.p, ngroups,
                  group_seg, nbig, st);
  {
    TimedScope ts("count", (double)0, st, lv);
    launch_count(ks, d_desc, plan, tile_seg, ntiles, (uint16_t*)W->hist.p, var, var + nbig, lut, st,
                 M.gt, M.torder);
  }
  // ---- offsets + children (list capacity for the worst case: every bin non-empty)
  const size_t worst = (size_t)nbig * kMaxBins;
  const int nxt = S.cur ^ 1;
  SRS_TRY(ensure(W->big[nxt], worst * sizeof(Seg)));
  SRS_TRY(ensure_keep(W->local, (S.n_local + worst) * sizeof(Seg), S.n_local * sizeof(Seg), st));
  SRS_TRY(ensure_keep(W->local2, (S.n_local2 + worst) * sizeof(Seg), S.n_local2 * sizeof(Seg), st));
  SRS_TRY(ensure_keep(W->copy, (S.n_copy + worst) * sizeof(Seg), S.n_copy * sizeof(Seg), st));
  if (!small_plan)  // (plan_small_kernel zeroed it)
    HIP_TRY(hipMemsetAsync(&d_ctr->n_big, 0, sizeof(unsigned long long), st));
  {
    TimedScope ts("scan", (double)ntiles, st);
    launch_offsets(plan, nbig, group_seg, ngroups, (uint16_t*)W->hist.p,
                   (uint32_t*)W->gsum.p, (uint64_t*)W->gofs.p, (uint64_t*)W->sbase.p,
                   offs32 ? nullptr : (uint64_t*)W->offs.p, offs32 ? (uint32_t*)W->offs.p : nullptr,
                   var, (Seg*)W->big[nxt].p, (Seg*)W->local.p,
                   (Seg*)W->local2.p, (Seg*)W->copy.p, d_ctr, lut_rbits, st, M.mode,
                   (uint32_t*)W->prun.p);
  }
  if (g_lb_status)  // (diagnostic look-back: fresh status words per level)
    HIP_TRY(hipMemsetAsync(g_lb_status, 0, (size_t)ntiles * kMaxBins * 4, st));
  {
    TimedScope ts("scatter", (double)0, st, lv);
    const bool pairs = (S.pair_tiles & 1) && (lut == 0 || ((S.pair_tiles & 2) && lut == 2)) &&
                       !((S.pair_tiles & 4) && lv == 1);
    if (pairs)
      launch_scatter_pairs(ks, d_desc, plan, tile_seg, (uint64_t*)W->offs.p,
                           offs32 ? (const uint32_t*)W->offs.p : nullptr, ntiles, lut, st, M.gt);
    else
      launch_scatter(ks, d_desc, plan, tile_seg, (uint64_t*)W->offs.p,
                     offs32 ? (const uint32_t*)W->offs.p : nullptr, ntiles, lut, S.ncols, st,
                     M.gt);
  }
  if (M.mode == 1) {
    // the buckets become the next level's segments (logical starts: where
    // they end up), their tiles the pieces every stripe holds of them
    // (a digit-table level consumes no fixed bits: its groups' prefixes
    // come from lut_rbits)
    const int nb = 1 << std::abs(force_bits);
    const int rbits = lut ? M.key_bits : M.key_bits - std::abs(force_bits);
    launch_stripe_tables((const uint32_t*)W->prun.p, nbig, nb, (uint32_t*)W->ptile.p,
                         (uint64_t*)W->btot.p, (uint32_t*)W->bnt.p, rbits, BUF_TMP,
                         (Seg*)W->big[nxt].p, (int32_t*)W->nt_over.p, (uint32_t*)W->btile.p,
                         d_ctr, (const uint64_t*)W->sbase.p, plan, (GTile*)W->gtile.p,
                         lut_rbits, st, (int32_t*)W->gorder.p, W->gorder_cap);
  }
  HIP_TRY(hipMemcpyAsync(W->h_ctr, d_ctr, sizeof(ListCounters), hipMemcpyDeviceToHost, st));
  SRS_TRY(sync_poll(st));
  S.nbig = (int64_t)W->h_ctr->n_big;
  S.n_local = (int64_t)W->h_ctr->n_local;
  S.n_local2 = (int64_t)W->h_ctr->n_local2;
  S.n_copy = (int64_t)W->h_ctr->n_copy;
  S.cur = nxt;
  if (trace_levels()) {
    fprintf(stderr, "[srs] level: %lld segs, %.0f keys, %lld tiles%s -> big %lld, local %lld, "
            "local2 %lld, copy %lld\n", (long long)nbig, level_elems, (long long)ntiles,
            lut ? " (lut)" : "", (long long)S.nbig, (long long)S.n_local,
            (long long)S.n_local2, (long long)S.n_copy);
    if (S.nbig > 0) {  // the next level's segments: sizes and rbits
      std::vector<Seg> b(S.nbig);
      HIP_TRY(hipMemcpy(b.data(), W->big[nxt].p, S.nbig * sizeof(Seg), hipMemcpyDeviceToHost));
      int64_t sum = 0, mx = 0, under16k = 0;
      for (const Seg& s : b) {
        sum += s.len;
        mx = std::max<int64_t>(mx, s.len);
        under16k += s.len <= 16384;
      }
      fprintf(stderr, "[srs]   big: %lld keys, max %lld, <= 16K keys: %lld segs; first rbits %d\n",
              (long long)sum, (long long)mx, (long long)under16k, b[0].rbits);
    }
  }
  return SRS_OK;
}

// Descriptor columns of a request: IN / OUT are the caller's arrays, TMP /
// TMP2 the workspace (AoS records as one column, or as 8-byte slices that are
// dense SoA columns in the workspace when aos_cols).
void set_columns(const Request& R, SortDesc& d, char* tmp, char* tmp2, bool aos_cols,
                 size_t slice_bytes, const size_t* tmp_off, bool inplace, bool pair = false) {
  const int ks = key_size_of(R.kind);
  if (R.aos) {
    const uint32_t E = R.elem_size;
    char* in = (char*)R.in_cols[0];
    char* out = (char*)R.out_cols[0];
    const uint32_t slice = E < 8 ? E : 8;
    int nc = 0;
    for (uint32_t off = 0; off < E; off += slice, nc++) {
      if (aos_cols)  // slice nc: a dense 8-byte column in TMP / TMP2
        d.cols[nc] = Col{{in + off, out + off, tmp + nc * slice_bytes, tmp2 + nc * slice_bytes},
                         slice, {E, E, 8, 8}};
      else
        d.cols[nc] = Col{{in + off, out + off, tmp ? tmp + off : nullptr, nullptr}, slice,
                         {E, E, E, E}};
    }
    d.ncols = nc;
    d.key = d.cols[0];
    d.key.width = (uint32_t)ks;  // the key: low bytes of slice 0
  } else {
    for (int c = 0; c < R.ncols; c++) {
      const uint32_t w = R.widths[c];
      d.cols[c] = Col{{(char*)R.in_cols[c], (char*)R.out_cols[c], tmp ? tmp + tmp_off[c] : nullptr,
                       tmp2 ? tmp2 + tmp_off[c] : nullptr}, w, {w, w, w, w}};
    }
    if (pair) {  // payloads 1 and 2: one interleaved 8-byte word column in TMP / TMP2
      for (int c = 1; c <= 2; c++) {
        const size_t off = tmp_off[1] + 4 * (c - 1);
        d.cols[c].base[BUF_TMP] = tmp + off;
        d.cols[c].base[BUF_TMP2] = tmp2 + off;
        d.cols[c].stride[BUF_TMP] = d.cols[c].stride[BUF_TMP2] = 8;
      }
      d.pair = 1;
    }
    d.key = d.cols[0];
    d.ncols = R.ncols;
  }
  if (inplace)  // IN aliases OUT: a segment that never moved is already home
    for (int c = 0; c < d.ncols; c++) d.cols[c].base[BUF_IN] = d.cols[c].base[BUF_OUT];
}

bool is_inplace(const Request& R) {
  bool inplace = true;
  for (int c = 0; c < R.ncols; c++) inplace &= (R.in_cols[c] == R.out_cols[c]);
  return inplace;
}

// The stream's slot for the single-launch sorts' fallback flags
// (srs_debug_last_fallbacks). A caller that sorts on ever new streams would
// grow the map without bound: past 64 streams the slots are dropped after a
// device-wide wait (their kernels may still be writing them).
int taken_slot(Workspace* W, hipStream_t st, DevBuf** out) {
  if (W->small_taken.size() >= 64 && !W->small_taken.count(st)) {
    HIP_TRY(hipDeviceSynchronize());
    for (auto& t : W->small_taken) free_buf(t.second);
    W->small_taken.clear();
    W->last_small = false;
  }
  DevBuf& taken = W->small_taken[st];
  SRS_TRY(ensure(taken, 2 * sizeof(int64_t)));
  *out = &taken;
  return SRS_OK;
}

// n <= kLocalCap (and no segment list): the whole sort is one local segment,
// sorted by one single-workgroup launch that takes the descriptor as a kernel
// argument. No workspace memory is touched (the input and output arrays
// only), so no stream-order wait on the workspace either.
int run_small(Workspace* W, const Request& R, hipStream_t st) {
  const int ks = key_size_of(R.kind);
  const int64_t n = R.num;
  const bool inplace = is_inplace(R);
  SortDesc d;
  memset(&d, 0, sizeof d);
  key_masks(R.kind, R.up, d);
  const bool is_float = R.kind == SRS_KEY_F32 || R.kind == SRS_KEY_F64;
  d.canon_zero = (is_float && n <= R.thresh) ? 1 : 0;
  d.leaf_skip = leaf_skip_of(R);
  const int ksl = ks | (d.canon_zero ? SRS_KS_CANON : 0);
  set_columns(R, d, nullptr, nullptr, false, 0, nullptr, inplace);
  d.stamp_acc = g_stamp_acc;
  const Seg g{0, n, d.key_bits, inplace ? BUF_OUT : BUF_IN};
  DevBuf* tk = nullptr;
  SRS_TRY(taken_slot(W, st, &tk));
  DevBuf& taken = *tk;
  W->last_small = true;
  W->last_small_stream = st;
  note_elems("local", (double)n);
  {
    TimedScope ts("local", (double)0, st);
    launch_small_sort(ksl, d, g, (int64_t*)taken.p, st);
  }
  HIP_TRY(hipGetLastError());
  return SRS_OK;
}

// The column layout local_direct_kernel's mode pm writes without checking
// (it stores whole records / dense words): pm 0 a dense key column and one
// dense 8-byte payload column; pm 1 16-byte records of an 8-byte key, the two
// slices at +0 / +8 of each record in IN / OUT and dense 8-byte slice columns
// in TMP / TMP2; pm 2 a dense key column and the two 4-byte payloads as one
// interleaved 8-byte word column in TMP / TMP2 (SortDesc::pair).
bool direct_layout_ok(const SortDesc& d, int pm, int ks) {
  const Col& k = d.cols[0];
  const int bufs[] = {BUF_IN, BUF_OUT, BUF_TMP, BUF_TMP2};
  if (pm == 0) {  // (TMP2: the home-write layout, dense SoA columns too)
    if (d.ncols != 2 || d.pair || d.cols[1].width != 8 || k.width != (uint32_t)ks) return false;
    for (int b : {BUF_IN, BUF_OUT, BUF_TMP, BUF_TMP2}) {
      if (b == BUF_TMP2 && !d.tmp2) continue;
      if (k.stride[b] != k.width || d.cols[1].stride[b] != 8) return false;
    }
    return true;
  }
  if (pm == 1) {
    const Col& p = d.cols[1];
    if (d.ncols != 2 || !d.tmp2 || ks != 8 || k.width != 8 || p.width != 8) return false;
    for (int b : {BUF_IN, BUF_OUT})
      if (k.stride[b] != 16 || p.stride[b] != 16 || p.base[b] != k.base[b] + 8) return false;
    for (int b : {BUF_TMP, BUF_TMP2})
      if (k.stride[b] != 8 || p.stride[b] != 8) return false;
    return true;
  }
  if (pm == 2) {
    const Col& a = d.cols[1];
    const Col& c = d.cols[2];
    if (d.ncols != 3 || !d.pair || a.width != 4 || c.width != 4 || k.width != (uint32_t)ks)
      return false;
    for (int b : bufs)
      if (k.stride[b] != k.width) return false;
    for (int b : {BUF_IN, BUF_OUT})
      if (a.stride[b] != 4 || c.stride[b] != 4) return false;
    for (int b : {BUF_TMP, BUF_TMP2})
      if (a.stride[b] != 8 || c.stride[b] != 8 || c.base[b] != a.base[b] + 4) return false;
    return true;
  }
  return false;
}

constexpr int64_t kStripeMinN = int64_t(1) << 25;

bool stripes_enabled() {
  static const bool on = [] {
    const char* e = getenv("SRS_NO_STRIPES");
    return !(e && *e && *e != '0');
  }();
  return on;
}

// Range level: the keys form a few narrow clusters (the
// sample's KeyClusters). One exact pass finds each cluster's smallest and
// largest key (split points halfway between the sampled clusters); the first
// level then sends key u of cluster c to bucket base_c + ((u - lo_c) >>
// shift_c), lo_c = min_c rounded down to 2^shift_c, with the 512 buckets
// shared out by the clusters' sizes and shift_c the smallest that fits. A
// bucket's keys then share every bit above shift_c (its children's rbits):
// Gaussian keys (~1200 values) take two levels and end single-valued in OUT,
// instead of a level on the sign bit, count-only levels on shared bits and a
// copy home. *final: every bucket holds one key value (shift 0 everywhere).
// *one_value: all keys are equal.
int plan_range_level(Workspace* W, const Request& R, const std::vector<KeyCluster>& cl,
                     SortDesc& d, hipStream_t st, bool* use, bool* final_lvl, bool* one_value) {
  *use = *final_lvl = *one_value = false;
  const int ks = key_size_of(R.kind);
  const int kb = 8 * ks;
  const int K = (int)cl.size();
  uint64_t hi[kMaxRanges] = {~0ull, ~0ull, ~0ull, ~0ull};
  for (int k = 0; k + 1 < K; k++) {  // split halfway between the sampled clusters
    const uint64_t mid_bin = ((uint64_t)cl[k].b1 + (uint64_t)cl[k + 1].b0 + 1) / 2;
    hi[k] = (mid_bin << (kb - 16)) - 1;
  }
  SRS_TRY(ensure(W->totals, 2 * kMaxRanges * sizeof(uint64_t)));
  unsigned long long* mm = (unsigned long long*)W->totals.p;
  uint64_t init[2 * kMaxRanges];
  for (int c = 0; c < kMaxRanges; c++) {
    init[2 * c] = ~0ull;
    init[2 * c + 1] = 0;
  }
  std::vector<uint64_t> got(2 * kMaxRanges);
  HIP_TRY(hipMemcpyAsync(mm, init, sizeof init, hipMemcpyHostToDevice, st));
  launch_key_minmax(R.in_cols[0], ks, ks, R.num, d.mpos, d.mneg, hi, mm, st);
  HIP_TRY(hipMemcpyAsync(got.data(), mm, sizeof init, hipMemcpyDeviceToHost, st));
  SRS_TRY(sync_poll(st));
  // the non-empty ranges (a range's keys: u in (hi[c-1], hi[c]])
  struct Rg {
    uint64_t mn, mx, cnt, hi;
  };
  std::vector<Rg> rg;
  for (int c = 0; c < K; c++) {
    if (got[2 * c] > got[2 * c + 1]) continue;  // no key fell into this range
    rg.push_back(Rg{got[2 * c], got[2 * c + 1], std::max<uint64_t>(cl[c].cnt, 1), hi[c]});
  }
  if (rg.empty()) return SRS_OK;
  if (rg.size() == 1 && rg[0].mn == rg[0].mx) {
    *one_value = true;
    return SRS_OK;
  }
  // one shift for every range: the smallest that fits all of them into the
  // level's buckets (ranges keep their order: dense bucket bases)
  const int R_ = (int)rg.size();
  auto shr = [](uint64_t x, int s) { return s >= 64 ? 0 : x >> s; };
  auto span = [&](int s) {
    uint64_t t = 0;
    for (const Rg& r : rg) t += shr(r.mx, s) - shr(r.mn, s) + 1;
    return t;
  };
  int s = 0;
  while (s < kb && span(s) > (uint64_t)kMaxBins) s++;
  uint32_t used = 0;
  for (int c = 0; c < kMaxRanges; c++) {
    d.rng_hi[c] = ~0ull;
    d.rng_adj[c] = 0;
  }
  std::vector<int> base(R_);
  for (int c = 0; c < R_; c++) {
    d.rng_hi[c] = c + 1 < R_ ? rg[c].hi : ~0ull;
    base[c] = (int)used;
    d.rng_adj[c] = used - (uint32_t)shr(rg[c].mn, s);  // (wrapping)
    used += (uint32_t)(shr(rg[c].mx, s) - shr(rg[c].mn, s) + 1);
  }
  // children's rbits: the bits above the shift are shared in a bucket
  std::vector<int32_t> rbits(kMaxBins, s);
  SRS_TRY(ensure(W->lut_rbits, kMaxBins * sizeof(int32_t)));
  HIP_TRY(hipMemcpyAsync(W->lut_rbits.p, rbits.data(), kMaxBins * sizeof(int32_t),
                         hipMemcpyHostToDevice, st));
  HIP_TRY(hipStreamSynchronize(st));  // (rbits goes out of scope)
  d.digit_lut = nullptr;
  d.lut_mode = 2;
  d.lut_bits = kMaxDigitBits;
  d.lut_shift = s;
  d.lut_entries = 0;
  *use = true;
  *final_lvl = s == 0;
  if (trace_levels())
    for (int c = 0; c < R_; c++)
      fprintf(stderr, "[srs] range %d: keys [%llx, %llx] -> buckets from %d, shift %d\n", c,
              (unsigned long long)rg[c].mn, (unsigned long long)rg[c].mx, base[c], s);
  return SRS_OK;
}

int copy_through(const Request& R, hipStream_t st);

// Mid-size sorts (kLocalCap < n <= kMidMaxKeys) take one launch with grid barriers
// (launch_mid_sort); SRS_MID=0 sends them down the general path.
// (below this a sort's columns stay in the L2 / Infinity Cache and the
// placement of OUT does not matter)
constexpr int64_t kHomeTmp2MinN = int64_t(1) << 24;

bool home_tmp2_enabled() {
  static const bool on = [] {
    const char* e = getenv("SRS_HOME_TMP2");
    return !(e && *e == '0');
  }();
  return on;
}

// the shard's plain-digit partition on the tile-pair scatter (SRS_PARTITION_PAIRS=0: off)
bool partition_pairs_enabled() {
  static const bool on = [] {
    const char* e = getenv("SRS_PARTITION_PAIRS");
    return !(e && *e == '0');
  }();
  return on;
}

// medium sorts: both local classes at once (run_sort's local pass)
constexpr int64_t kLocalForkMaxN = int64_t(1) << 24;
bool local_fork_enabled() {
  static const bool on = [] {
    const char* e = getenv("SRS_LOCAL_FORK");
    return !(e && *e == '0');
  }();
  return on;
}

bool mid_enabled() {
  static const bool on = [] {
    const char* e = getenv("SRS_MID");
    return !(e && *e == '0');
  }();
  return on;
}

// the largest sort whose first level takes one launch (launch_mid_level);
// SRS_MID_LEVEL_MAX (records, <= kMidLevelMaxKeys) for A/B runs, 0 off
int64_t mid_level_max_n() {
  static const int64_t v = [] {
    const char* e = getenv("SRS_MID_LEVEL_MAX");
    const int64_t x = e && *e ? (int64_t)atof(e) : kMidLevelMaxKeys;
    return std::min<int64_t>(x, kMidLevelMaxKeys);
  }();
  return v;
}

// Waits for the mid-size kernel's MidFlag of call `seq`: a short poll, then
// the stream (which also surfaces a kernel failure).
int wait_mid_flag(const MidFlag* f, unsigned long long seq, hipStream_t st) {
  auto seen = [&] { return __atomic_load_n(&f->seq, __ATOMIC_ACQUIRE) == seq; };
  const auto t0 = std::chrono::steady_clock::now();
  while (!seen()) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(5)) {
      HIP_TRY(hipStreamSynchronize(st));
      if (!seen()) return fail(SRS_ERR_INTERNAL, "mid-size launch: no answer from the kernel");
      break;
    }
    cpu_relax();
  }
  return SRS_OK;
}

int run_sort(Workspace* W, const Request& R, hipStream_t st) {
  if (R.nsegs == 0 && R.num <= kLocalCap) return run_small(W, R, st);
  {
    const char* e = getenv("SRS_XCD_ROT");  // (placement diagnostics)
    set_xcd_rotation(e && *e ? atoi(e) : 0);
  }
  W->last_small = false;
  const int ks = key_size_of(R.kind);
  const int64_t n = R.num;
  const bool inplace = is_inplace(R);

  // ---- descriptor: key view + columns (AoS records as <= 8-byte slices) --
  SortDesc d;
  memset(&d, 0, sizeof d);
  key_masks(R.kind, R.up, d);
  const bool is_float = R.kind == SRS_KEY_F32 || R.kind == SRS_KEY_F64;
  d.canon_zero = (is_float && n <= R.thresh) ? 1 : 0;
  d.leaf_skip = leaf_skip_of(R);
  const int ksl = ks | (d.canon_zero ? SRS_KS_CANON : 0);  // kernel dispatch key
  // (the mid-size launch moves the columns as they are: no slices, no pairs)
  const bool mid = R.nsegs == 0 && n > kLocalCap && n <= kMidMaxKeys && mid_enabled();
  // (above it, the first level in one launch; the layout is the general path's
  // except C2's interleaved pair words, which that launch's scatter does not write)
  const bool mid1 = R.nsegs == 0 && n > kMidMaxKeys && n <= mid_level_max_n() && mid_enabled();

  // AoS records of 16+ bytes travel as SoA slice columns through the
  // workspace (TMP, TMP2) between the first scatter and the local pass: the
  // later count passes then read 8-byte keys instead of whole records and
  // the middle scatters move dense columns
  const bool aos_cols = R.aos && R.elem_size >= 16 && n > kLocalCap && R.nsegs == 0 && !mid;
  // A key and two 4-byte payload columns (C2) travel with the payloads
  // interleaved as one 8-byte word per record through TMP / TMP2: the
  // scatters then write 64-byte runs of words instead of two columns of
  // 32-byte runs (the same bytes as one 8-byte payload column measured
  // 23.6 -> 21.1 ms at 1e9)
  const bool pair_cols = !R.aos && R.ncols == 3 && R.widths[1] == 4 && R.widths[2] == 4 &&
                         n > kLocalCap && R.nsegs == 0 && !mid && !mid1;
  // Home write (round 6): when the output columns are not placement-probed
  // memory (srs_alloc_device) -- the reference's in-place contract
  // (radixSort.hpp:1780) on the caller's own array, or any array of the
  // caller's allocator -- the scatters stay in the workspace (IN -> TMP ->
  // TMP2, both placed) and only the local pass writes OUT, as one
  // contiguous run per segment. The scatter's partial 64-byte blocks are
  // what an unlucky placement slows down (6.2 vs 7.0 ms per
  // launch); a streaming write is far less exposed. (SRS_HOME_TMP2=0: off)
  bool home_tmp2 = false;
  if (!R.aos && !pair_cols && n >= kHomeTmp2MinN && R.nsegs == 0 && !mid && !mid1 &&
      home_tmp2_enabled()) {
    for (int c = 0; c < R.ncols && !home_tmp2; c++)
      home_tmp2 = !placed_memory(R.out_cols[c], (size_t)n * R.widths[c]);
  }
  size_t tmp_bytes = 0, slice_bytes = 0;
  std::vector<size_t> tmp_off;
  if (R.aos) {
    tmp_off.push_back(0);
    slice_bytes = align_up((size_t)n * 8, 256);
    tmp_bytes = aos_cols ? slice_bytes * (R.elem_size / 8) : align_up((size_t)n * R.elem_size, 256);
  } else {
    for (int c = 0; c < R.ncols; c++) {
      tmp_off.push_back(tmp_bytes);
      tmp_bytes += align_up((size_t)n * R.widths[c], 256);  // (a pair: 8n bytes at tmp_off[1])
    }
  }
  SRS_TRY(ensure(W->tmp, tmp_bytes, ws_alloc_mode(), true));
  char* tmp = (char*)W->tmp.p;
  char* tmp2 = nullptr;
  if (home_tmp2 && ensure(W->tmp2, tmp_bytes, ws_alloc_mode(), true) != SRS_OK) {
    home_tmp2 = false;  // (no room for TMP2: the scatter writes OUT as before)
    (void)hipGetLastError();
  }
  if (aos_cols || pair_cols || home_tmp2) {
    SRS_TRY(ensure(W->tmp2, tmp_bytes, ws_alloc_mode(), true));
    tmp2 = (char*)W->tmp2.p;
    d.tmp2 = 1;
  }

  set_columns(R, d, tmp, tmp2, aos_cols, slice_bytes, tmp_off.data(), inplace, pair_cols);

  d.stamp_acc = g_stamp_acc;
  d.lb_status = g_lb_status;
  d.lb_err = g_lb_err;
  bool balanced = false, spread = false, ranges = false, ranges_final = false;
  int lut_entries = 0, lut_mode = 1;
  std::vector<KeyCluster> clusters;
  SRS_TRY(plan_balanced_level(W, R, d, &balanced, &lut_entries, &lut_mode, st, &spread,
                              &clusters));
  if (!clusters.empty()) {
    bool one_value = false;
    SRS_TRY(plan_range_level(W, R, clusters, d, st, &ranges, &ranges_final, &one_value));
    if (one_value) return copy_through(R, st);  // (stable: nothing moves)
    balanced = ranges;  // (the range level runs where a digit-table level would)
  }
  if (balanced && !ranges) {
    d.digit_lut = (const int32_t*)W->lut.p;
    d.lut_shift = d.key_bits - (lut_mode == 3 ? 9 : 16);
    d.lut_bits = lut_mode == 3 ? 9 : 16;
    d.lut_mode = lut_mode;
    d.lut_entries = lut_entries;
  }
  SRS_TRY(ensure(W->desc, sizeof(SortDesc)));
  SortDesc* d_desc = (SortDesc*)W->desc.p;

  // ---- initial segments (the descriptor is written with them) --------------
  const int home = inplace ? BUF_OUT : BUF_IN;
  SRS_TRY(ensure(W->big[0], 1024 * sizeof(Seg)));
  SRS_TRY(ensure(W->big[1], 1024 * sizeof(Seg)));
  SRS_TRY(ensure(W->local, 1024 * sizeof(Seg)));
  SRS_TRY(ensure(W->local2, 1024 * sizeof(Seg)));
  SRS_TRY(ensure(W->copy, 1024 * sizeof(Seg)));
  SRS_TRY(ensure(W->ctr, sizeof(ListCounters)));
  SRS_TRY(ensure(W->totals, 4 * sizeof(uint64_t)));
  ListCounters* d_ctr = (ListCounters*)W->ctr.p;
  int64_t n_big = 0, n_local = 0, n_local2 = 0, n_copy = 0;
  bool mid_continued = false;  // (the big list came from the mid-size launch)
  int64_t one_seg_len = 0;     // (a segment sort of one large segment: its length)
  if (R.nsegs > 0) {
    // independent segments (multi-GPU receive groups): sorted as sub-ranges
    // of one sort, each starting at the full key width (the varying-bit
    // detection skips what a segment's keys share)
    std::vector<Seg> hb, hl, hl2;
    uint64_t lel = 0;
    for (int64_t i = 0; i < R.nsegs; i++) {
      const int64_t a = R.seg_bounds[i], len = R.seg_bounds[i + 1] - a;
      if (len < 2) continue;
      const Seg g{a, len, d.key_bits - R.known_top_bits, home};
      if (len <= kLocalCapSmall) hl.push_back(g);
      else if (len <= kLocalCap) hl2.push_back(g);
      else hb.push_back(g);
      if (len <= kLocalCap) lel += (uint64_t)len;
    }
    SRS_TRY(ensure(W->big[0], std::max<size_t>(1024, hb.size()) * sizeof(Seg)));
    SRS_TRY(ensure(W->local, std::max<size_t>(1024, hl.size()) * sizeof(Seg)));
    SRS_TRY(ensure(W->local2, std::max<size_t>(1024, hl2.size()) * sizeof(Seg)));
    if (hb.size() == 1 && hl.empty() && hl2.empty()) {
      // one large segment (the multi-GPU shard's rounds): the lists and the
      // descriptor in one launch, no host copies and no host wait, and its
      // first level sized from its length (no totals read-back): ~0.1 ms of
      // stalls per round sort less
      launch_start(d, d_desc, hb[0], 0, (Seg*)W->big[0].p, (Seg*)W->local.p, (Seg*)W->local2.p,
                   d_ctr, st);
      one_seg_len = hb[0].len;
    } else {
    if (!hb.empty())
      HIP_TRY(hipMemcpyAsync(W->big[0].p, hb.data(), hb.size() * sizeof(Seg),
                             hipMemcpyHostToDevice, st));
    if (!hl.empty())
      HIP_TRY(hipMemcpyAsync(W->local.p, hl.data(), hl.size() * sizeof(Seg),
                             hipMemcpyHostToDevice, st));
    if (!hl2.empty())
      HIP_TRY(hipMemcpyAsync(W->local2.p, hl2.data(), hl2.size() * sizeof(Seg),
                             hipMemcpyHostToDevice, st));
    launch_set_desc(d, d_desc, st);
    ListCounters c;
    memset(&c, 0, sizeof c);
    c.n_big = hb.size();
    c.n_local = hl.size();
    c.n_local2 = hl2.size();
    c.local_elems = lel;
    HIP_TRY(hipMemcpyAsync(d_ctr, &c, sizeof c, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));  // the host vectors go out of scope
    }
    n_big = (int64_t)hb.size();
    n_local = (int64_t)hl.size();
    n_local2 = (int64_t)hl2.size();
    W->h_ctr->local_elems = lel;
  } else {
    bool started = false;  // (by the mid-size launch)
    if (mid) {
      // one launch (grid barriers): the first level and every bucket's local
      // sort; buckets over kLocalCap (skewed keys) come back in the big list
      // and continue on the general levels below
      const int64_t T = (n + kTile - 1) / kTile;
      const int64_t part_bytes = mid_part_bytes(n);
      SRS_TRY(ensure(W->mid, part_bytes + T * kMaxBins * sizeof(uint32_t)));
      if (!W->midbar.p) {
        SRS_TRY(ensure(W->midbar, mid_bar_words() * sizeof(unsigned long long)));
        HIP_TRY(hipMemsetAsync(W->midbar.p, 0, mid_bar_words() * sizeof(unsigned long long), st));
      }
      auto barrier_failed = [&] { return __atomic_load_n(&W->h_mid->err, __ATOMIC_ACQUIRE) != 0; };
      if (barrier_failed())  // (an earlier call's barrier timed out: its output was wrong)
        return fail(SRS_ERR_INTERNAL, "mid-size launch: a grid barrier timed out");
      DevBuf* tk = nullptr;
      SRS_TRY(taken_slot(W, st, &tk));
      DevBuf& taken = *tk;
      hipError_t e;
      const unsigned long long seq = ++W->mid_seq;
      {
        note_elems("mid", (double)n);
        TimedScope ts("mid", (double)0, st);
        e = launch_mid_sort(ksl, d, n, home, (unsigned long long*)W->mid.p,
                            (uint32_t*)((char*)W->mid.p + part_bytes), d_ctr, (Seg*)W->big[0].p,
                            (unsigned long long*)taken.p, W->h_mid, seq,
                            (unsigned long long*)W->midbar.p, st);
      }
      if (e != hipSuccess) {
        // (a grid the device cannot hold resident: the general path, which
        // the column layout chosen for `mid` also serves)
        (void)hipGetLastError();
        if (trace_levels())
          fprintf(stderr, "[srs] mid-size launch refused (%s): general path\n", hipGetErrorString(e));
      } else {
        // The kernel's workgroup 0 posts the big-bucket count to host memory
        // once the first level's sizes are known (MidFlag): polled for a
        // while (a stream sync's wake-up cost ~30 us per call), then waited for
        SRS_TRY(wait_mid_flag(W->h_mid, seq, st));
        if (barrier_failed())
          return fail(SRS_ERR_INTERNAL, "mid-size launch: a grid barrier timed out");
        const unsigned long long nb_flag = __atomic_load_n(&W->h_mid->n_big, __ATOMIC_ACQUIRE);
        if (nb_flag >> 63)
          return fail(SRS_ERR_INTERNAL, "mid-size launch: more buckets than workgroups");
        n_big = (int64_t)nb_flag;
        if (n_big == 0) {
          W->last_small = true;  // (srs_debug_last_fallbacks reads `taken`)
          W->last_small_stream = st;
          return SRS_OK;
        }
        launch_set_desc(d, d_desc, st);
        W->h_ctr->local_elems = 0;
        started = true;
      }
    }
    if (mid1) {
      // the first level in one launch (grid barriers); the work lists and
      // their lengths come back as after a general first level
      const int64_t T = (n + kTile - 1) / kTile;
      const int64_t part_bytes = mid_level_part_bytes();
      SRS_TRY(ensure(W->mid, part_bytes + T * kMaxBins * sizeof(uint32_t)));
      if (!W->midbar.p) {
        SRS_TRY(ensure(W->midbar, mid_bar_words() * sizeof(unsigned long long)));
        HIP_TRY(hipMemsetAsync(W->midbar.p, 0, mid_bar_words() * sizeof(unsigned long long), st));
      }
      auto barrier_failed = [&] { return __atomic_load_n(&W->h_mid->err, __ATOMIC_ACQUIRE) != 0; };
      if (barrier_failed())
        return fail(SRS_ERR_INTERNAL, "mid-size launch: a grid barrier timed out");
      hipError_t e;
      const unsigned long long seq = ++W->mid_seq;
      {
        note_elems("mid_level", (double)n);
        TimedScope ts("mid_level", (double)0, st);
        e = launch_mid_level(ksl, d, n, home, (unsigned long long*)W->mid.p,
                             (uint32_t*)((char*)W->mid.p + part_bytes), d_ctr, (Seg*)W->big[0].p,
                             (Seg*)W->local.p, (Seg*)W->local2.p, (Seg*)W->copy.p, d_desc,
                             W->h_mid, seq, (unsigned long long*)W->midbar.p, st);
      }
      if (e != hipSuccess) {
        (void)hipGetLastError();
        if (trace_levels())
          fprintf(stderr, "[srs] mid-level launch refused (%s): general path\n", hipGetErrorString(e));
      } else {
        SRS_TRY(wait_mid_flag(W->h_mid, seq, st));
        if (barrier_failed())
          return fail(SRS_ERR_INTERNAL, "mid-size launch: a grid barrier timed out");
        n_big = (int64_t)__atomic_load_n(&W->h_mid->n_big, __ATOMIC_ACQUIRE);
        n_local = (int64_t)__atomic_load_n(&W->h_mid->n_local, __ATOMIC_ACQUIRE);
        n_local2 = (int64_t)__atomic_load_n(&W->h_mid->n_local2, __ATOMIC_ACQUIRE);
        n_copy = (int64_t)__atomic_load_n(&W->h_mid->n_copy, __ATOMIC_ACQUIRE);
        W->h_ctr->local_elems = __atomic_load_n(&W->h_mid->local_elems, __ATOMIC_ACQUIRE);
        if (trace_levels())
          fprintf(stderr, "[srs] mid-level: big %lld, local %lld, local2 %lld, copy %lld\n",
                  (long long)n_big, (long long)n_local, (long long)n_local2, (long long)n_copy);
        if (n_big + n_local + n_local2 + n_copy == 0) return SRS_OK;  // (keys all equal: copied)
        started = true;
      }
    }
    if (!started) {
      Seg seg0{0, n, d.key_bits, home};
      const bool to_local = n <= kLocalCap;
      launch_start(d, d_desc, seg0, to_local ? 1 : 0, (Seg*)W->big[0].p, (Seg*)W->local.p,
                   (Seg*)W->local2.p, d_ctr, st);
      n_big = to_local ? 0 : 1;
      n_local = (to_local && n <= kLocalCapSmall) ? 1 : 0;
      n_local2 = (to_local && n > kLocalCapSmall) ? 1 : 0;
      W->h_ctr->local_elems = to_local ? (uint64_t)n : 0;
    } else {
      mid_continued = true;
    }
  }
  LevelState S{n_big, n_local, n_local2, n_copy, 0, d.ncols, d.tmp2};
  S.pair_tiles = pair_tiles_mode(d, ks, aos_cols);
  if (R.nsegs == 0 && n_big == 1 && !mid_continued) S.known_len = n;
  if (one_seg_len > 0) S.known_len = one_seg_len;
  int level = 0;
  // Stripe first level: large plain SoA sorts partition
  // stripes of kStripeKeysPerBucket << b1 keys on their own with the first
  // digit, so a tile's scattered runs land in its stripe's window (the
  // second level's scatter, which writes into one bucket's window, measured
  // 5.9 ms per C1 launch against 7.0 for the first one over the whole array)
  // (a balanced first level: its 512 digit-table groups are the buckets)
  const int b1 = balanced ? kMaxDigitBits : choose_bits(n, d.key_bits);
  const int64_t stripe_len = (int64_t)kStripeKeysPerBucket << b1;
  // Only when the first digit (or the digit table) spreads the keys: a
  // plain level skips a digit all keys share, a stripe level cannot (all-zero
  // keys: 9.4 ms plain, 17.7 ms with stripes), so the key sample decides.
  const bool stripes = R.nsegs == 0 && !d.canon_zero && (ks == 4 || ks == 8) &&
                       (balanced || spread) && !ranges_final &&
                       n >= kStripeMinN && n < (int64_t(1) << 32) && n >= 2 * stripe_len &&
                       stripes_enabled();
  if (stripes) {
    const int64_t K = (n + stripe_len - 1) / stripe_len;
    std::vector<Seg> hs(K);
    for (int64_t k = 0; k < K; k++)
      hs[k] = Seg{k * stripe_len, std::min(stripe_len, n - k * stripe_len), d.key_bits, home};
    SRS_TRY(ensure(W->big[0], K * sizeof(Seg)));
    HIP_TRY(hipMemcpyAsync(W->big[0].p, hs.data(), K * sizeof(Seg), hipMemcpyHostToDevice, st));
    const int nb = 1 << b1;
    const size_t pieces = (size_t)K * kMaxBins;
    SRS_TRY(ensure(W->prun, pieces * 4));
    SRS_TRY(ensure(W->ptile, pieces * 4));
    SRS_TRY(ensure(W->btot, kMaxBins * 8));
    SRS_TRY(ensure(W->bnt, kMaxBins * 4));
    SRS_TRY(ensure(W->btile, kMaxBins * 4));
    SRS_TRY(ensure(W->nt_over, kMaxBins * 4));
    // tiles of the gathered level: at most one partial tile per piece
    SRS_TRY(ensure(W->gtile, ((n + kTile - 1) / kTile + (size_t)K * nb) * sizeof(GTile)));
    W->gorder_cap = (n + kTile - 1) / kTile + (int64_t)K * nb;  // + K entries of scratch
    SRS_TRY(ensure(W->gorder, (W->gorder_cap + K) * sizeof(int32_t)));
    HIP_TRY(hipStreamSynchronize(st));  // hs goes out of scope
    S.nbig = K;
    S.known_len = -1;
    LevelMode m1;
    m1.mode = 1;
    m1.key_bits = d.key_bits;
    ++level;
    if (balanced)
      SRS_TRY(run_level(W, ksl, d_desc, S, kMaxDigitBits, d.lut_mode >= 2 ? 2 : 1, st,
                        (const int32_t*)W->lut_rbits.p, m1));
    else
      SRS_TRY(run_level(W, ksl, d_desc, S, -b1, false, st, nullptr, m1));
    LevelMode m2;
    m2.mode = 2;
    m2.gt = (const GTile*)W->gtile.p;
    m2.nt_over = (const int32_t*)W->nt_over.p;
    m2.torder = (const int32_t*)W->gorder.p;
    ++level;
    if (S.nbig > 0) SRS_TRY(run_level(W, ksl, d_desc, S, 0, false, st, nullptr, m2));
  }
  if (balanced && !stripes && S.nbig > 0) {
    ++level;
    LevelMode m0;
    m0.home = ranges_final;  // (single-valued buckets: written home directly)
    SRS_TRY(run_level(W, ksl, d_desc, S, kMaxDigitBits, d.lut_mode >= 2 ? 2 : 1, st,
                      (const int32_t*)W->lut_rbits.p, m0));
  }
  while (S.nbig > 0) {
    if (++level > 80) return fail(SRS_ERR_INTERNAL, "level limit exceeded");
    SRS_TRY(run_level(W, ksl, d_desc, S, 0, false, st));
  }
  n_local = S.n_local;
  n_local2 = S.n_local2;
  n_copy = S.n_copy;

  if (n_local + n_local2 > 0) {
    note_elems("local", (double)W->h_ctr->local_elems);
    TimedScope ts("local", (double)0, st);
    // fast kernel -> (large buckets) stable kernel -> (wide keys) LSD kernel;
    // the fallback kernels read their list lengths on device
    SRS_TRY(ensure(W->fallback, (n_local + n_local2) * sizeof(Seg)));
    SRS_TRY(ensure(W->fallback2, (n_local + n_local2) * sizeof(Seg)));
    Seg* fb = (Seg*)W->fallback.p;         // [0, n_local2): large, then small
    Seg* fb1 = fb + n_local2;
    Seg* fb2 = (Seg*)W->fallback2.p;
    unsigned long long* nfb = &d_ctr->n_fallback;
    unsigned long long* nfb1 = &d_ctr->n_fallback1;
    unsigned long long* nfb2 = &d_ctr->n_fallback2;
    // Medium sorts (latency-bound launches) run the large class's chain --
    // its local kernel and its stable fallback -- on a second stream beside
    // the small class's; they join before the LSD fallback, which takes both
    // classes' hand-overs (round 6: a 2^21-key sort splits its buckets half
    // and half between the classes, and the two ~21 us launches ran back to
    // back). Large sorts keep one stream: there the kernels already share the
    // memory system's limit (§4: a side stream was slower).
    hipStream_t s2 = st;
    if (n_local > 0 && n_local2 > 0 && n <= kLocalForkMaxN && local_fork_enabled()) {
      if (!W->side) {
        HIP_TRY(hipStreamCreateWithFlags(&W->side, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&W->ev_fork, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&W->ev_join, hipEventDisableTiming));
      }
      HIP_TRY(hipEventRecord(W->ev_fork, st));
      HIP_TRY(hipStreamWaitEvent(W->side, W->ev_fork, 0));
      s2 = W->side;
    }
    {
      TimedScope ts1("local_fast", 0, st);
      const bool rec16 = aos_cols && R.elem_size == 16;
      // the common shapes take the direct kernel at four workgroups per CU
      // (two in the large class); what it hands over runs through the fast
      // kernel: pm 0 a 4/8-byte key + one 8-byte payload (C1),
      // 1 16-byte records of an 8-byte key as slices (C3), 2 a key + two
      // 4-byte payloads (C2)
      int pm = -1;
      if (!R.aos && R.ncols == 2 && R.widths[1] == 8 && !d.pair) pm = 0;
      else if (rec16 && ks == 8) pm = 1;
      else if (d.pair && ks == 4) pm = 2;
      if (pm >= 0 && !direct_layout_ok(d, pm, ks)) pm = -1;  // (the kernel assumes it)
      const bool direct_any = pm >= 0 && (ks == 4 || ks == 8) && !d.canon_zero &&
                              direct_local_enabled();
      const bool direct = direct_any && n_local >= direct_min_segs();
      const bool direct2 = direct_any && direct_local2_enabled() && n_local2 >= direct_min_segs();
      if (n_local2 > 0 && direct2) {
        SRS_TRY(ensure(W->redo2, n_local2 * sizeof(Seg)));
        launch_local_direct(ks, pm, d_desc, (Seg*)W->local2.p, n_local2, (Seg*)W->redo2.p,
                            &d_ctr->n_redo2, fb, nfb, s2, true);
        launch_local_list(ks, d_desc, (Seg*)W->redo2.p, &d_ctr->n_redo2,
                          (int)std::min<int64_t>(n_local2, 1024), fb, nfb, s2, true);
      } else if (n_local2 > 0) {
        launch_local(ksl, d_desc, (Seg*)W->local2.p, n_local2, 1, fb, nfb, s2, rec16);
      }
      if (n_local > 0 && direct) {
        SRS_TRY(ensure(W->redo, n_local * sizeof(Seg)));
        launch_local_direct(ks, pm, d_desc, (Seg*)W->local.p, n_local, (Seg*)W->redo.p,
                            &d_ctr->n_redo, fb1, nfb1, st);
        launch_local_list(ks, d_desc, (Seg*)W->redo.p, &d_ctr->n_redo,
                          (int)std::min<int64_t>(n_local, 2048), fb1, nfb1, st);
      } else if (n_local > 0) {
        launch_local(ksl, d_desc, (Seg*)W->local.p, n_local, 0, fb1, nfb1, st, rec16);
      }
    }
    {
      TimedScope ts2("local_stable", 0, st);
      // grid-stride over the handed-over segments (the list length is only
      // known on device): at most 2048 workgroups, so an empty list costs a
      // few microseconds instead of one exiting workgroup per local segment
      // (0.11 ms at C1)
      auto grid = [](int64_t m) { return (int)std::min<int64_t>(m, 2048); };
      if (n_local2 > 0) launch_local_stable(ksl, d_desc, fb, nfb, 1, fb2, nfb2, grid(n_local2), s2);
      if (n_local > 0) launch_local_stable(ksl, d_desc, fb1, nfb1, 0, fb2, nfb2, grid(n_local), st);
      if (s2 != st) {  // (the join: the LSD fallback reads both classes' hand-overs)
        HIP_TRY(hipEventRecord(W->ev_join, s2));
        HIP_TRY(hipStreamWaitEvent(st, W->ev_join, 0));
      }
    }
    {
      TimedScope ts3("local_lsd", 0, st);
      const int fgrid = (int)std::min<int64_t>(512, n_local + n_local2);
      launch_local_lsd(ksl, d_desc, fb2, nfb2, fgrid, st);
    }
    if (trace_levels()) {
      // diagnostics: how many segments took each fallback (a host wait; kept
      // out of the timing mode, which only adds event markers)
      ListCounters c;
      HIP_TRY(hipMemcpyAsync(&c, d_ctr, sizeof(c), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      fprintf(stderr, "[srs] local: %lld + %lld segs (%llu keys); stable fallback %llu + %llu, "
              "lsd fallback %llu\n", (long long)n_local, (long long)n_local2,
              c.local_elems, c.n_fallback1, c.n_fallback, c.n_fallback2);
      fprintf(stderr, "[srs] local: %llu + %llu small / large-class segments handed from the "
              "direct kernel\n", c.n_redo, c.n_redo2);
    }
  }
  if (n_copy > 0) {
    // the list stays on the device (the level scratch arrays are free now)
    SRS_TRY(ensure(W->tcount, n_copy * 8));
    SRS_TRY(ensure(W->tbase, n_copy * 8));
    SRS_TRY(ensure(W->scan_tmp, scan_temp_elems(n_copy) * 8));
    TimedScope ts("copy", (double)0, st);
    launch_copy_list(d_desc, (const Seg*)W->copy.p, n_copy, (uint64_t*)W->tcount.p,
                     (uint64_t*)W->tbase.p, (uint64_t*)W->scan_tmp.p,
                     (uint64_t*)W->totals.p + 2, st);
  }
  HIP_TRY(hipGetLastError());
  return SRS_OK;
}

// One LUT-digit level: stable partition of the columns into num_parts groups
// (multi-GPU shard). The scatter's destination buffer (TMP) is
// the caller's output arrays.
int run_partition(Workspace* W, const Request& R, int bits, const int32_t* d_lut,
                  int nparts, int64_t* counts, hipStream_t st) {
  W->last_small = false;  // (srs_debug_last_fallbacks then reports this call's counters)
  const int ks = key_size_of(R.kind);
  const int64_t n = R.num;
  SortDesc d;
  memset(&d, 0, sizeof d);
  key_masks(R.kind, R.up, d);
  for (int c = 0; c < R.ncols; c++) {
    char* in = (char*)R.in_cols[c];
    char* out = (char*)R.out_cols[c];
    const uint32_t w = R.widths[c];
    d.cols[c] = Col{{in, out, out, nullptr}, w, {w, w, w, w}};
  }
  d.key = d.cols[0];
  d.ncols = R.ncols;
  d.digit_lut = d_lut;
  d.lut_shift = d.key_bits - bits;
  d.lut_bits = bits;
  // Groups that are the ranges of the top fb key bits (uniform keys over a
  // power-of-two group count: 4096 bins -> 512 groups of 8) need no table:
  // the plain digit scatter is cheaper than the table lookups (C1 1e9:
  // ~8 ms for the table pass)
  int fb0 = 1;
  while ((1 << fb0) < nparts) fb0++;
  bool aligned = (1 << fb0) == nparts && fb0 <= bits;
  if (aligned) {
    std::vector<int32_t> t((size_t)1 << bits);
    HIP_TRY(hipMemcpyAsync(t.data(), d_lut, t.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (size_t b = 0; b < t.size() && aligned; b++) aligned = t[b] == (int32_t)(b >> (bits - fb0));
  }
  if (aligned) d.digit_lut = nullptr;
  SRS_TRY(ensure(W->desc, sizeof(SortDesc)));
  SortDesc* d_desc = (SortDesc*)W->desc.p;
  SRS_TRY(ensure(W->big[0], 1024 * sizeof(Seg)));
  SRS_TRY(ensure(W->big[1], 1024 * sizeof(Seg)));
  SRS_TRY(ensure(W->local, 1024 * sizeof(Seg)));
  SRS_TRY(ensure(W->local2, 1024 * sizeof(Seg)));
  SRS_TRY(ensure(W->copy, 1024 * sizeof(Seg)));
  SRS_TRY(ensure(W->ctr, sizeof(ListCounters)));
  SRS_TRY(ensure(W->totals, 4 * sizeof(uint64_t)));
  Seg seg0{0, n, d.key_bits, BUF_IN};
  launch_start(d, d_desc, seg0, 0, (Seg*)W->big[0].p, (Seg*)W->local.p, (Seg*)W->local2.p,
               (ListCounters*)W->ctr.p, st);
  int fb = 1;
  while ((1 << fb) < nparts) fb++;
  LevelState S{1, 0, 0, 0, 0, d.ncols, 0};
  // the plain-digit partition takes the tile-pair scatter like a sort's
  // levels (C1 chunks: 6.6 -> ~5.9 ms per 1e9 keys)
  if (aligned && partition_pairs_enabled()) S.pair_tiles = pair_tiles_mode(d, ks, false);
  SRS_TRY(run_level(W, ks, d_desc, S, aligned ? -fb : fb, aligned ? 0 : 1, st));
  // group sizes from the segment's bucket bases (sbase row 0)
  std::vector<uint64_t> sb((size_t)1 << fb);
  HIP_TRY(hipMemcpyAsync(sb.data(), W->sbase.p, sb.size() * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  bool single = false;
  for (int p = 0; p < nparts; p++) {
    const uint64_t lo = sb[p], hi = (p + 1 < (int)sb.size()) ? sb[p + 1] : (uint64_t)n;
    counts[p] = p + 1 < nparts ? (int64_t)(hi - lo) : (int64_t)((uint64_t)n - lo);
    single |= counts[p] == n;
  }
  if (single) {  // the scatter was skipped (one group holds everything): copy
    for (int c = 0; c < R.ncols; c++)
      HIP_TRY(hipMemcpyAsync(R.out_cols[c], R.in_cols[c], (size_t)n * R.widths[c],
                             hipMemcpyDeviceToDevice, st));
  }
  return SRS_OK;
}

int validate_common(int64_t num, int kind) {
  if (key_size_of(kind) == 0) return fail(SRS_ERR_INVALID_ARG, "invalid key_kind");
  (void)num;
  return SRS_OK;
}

int copy_through(const Request& R, hipStream_t st) {
  // num <= 1 with distinct output arrays: the result is the input
  const int64_t n = R.num < 0 ? 0 : R.num;
  for (int c = 0; c < R.ncols; c++) {
    if (R.in_cols[c] == R.out_cols[c] || n == 0) continue;
    const size_t w = R.aos ? R.elem_size : R.widths[c];
    HIP_TRY(hipMemcpyAsync(R.out_cols[c], R.in_cols[c], n * w, hipMemcpyDeviceToDevice, st));
  }
  return SRS_OK;
}

// CmpSorterNoSort with num <= cmpSortThreshold: the whole input is one leaf,
// which the reference leaves as it is (radixSort.hpp:1743, cmp_sorters.hpp:66-78)
bool whole_input_is_unsorted_leaf(const Request& R) {
  return R.leaf_mode == SRS_LEAF_UNSORTED && R.num <= R.thresh;
}

int sort_device(Request& R, hipStream_t st) {
  if (R.num <= 1 || whole_input_is_unsorted_leaf(R)) return copy_through(R, st);
  Workspace* W = nullptr;
  WsLock lk;
  SRS_TRY(acquire_ws(&W, &lk));
  // (a small sort touches no workspace buffer but its stream's debug slot)
  if (R.num <= kLocalCap) return run_small(W, R, st);
  WsUse use;
  SRS_TRY(use.begin(W, st));
  return run_sort(W, R, st);
}

// ---------------------------------------------------------------------------
// host arrays (the reference's calling convention, radixSort.hpp:1780):
// staged PCIe copies, and the split of one host array over several GPUs
// ---------------------------------------------------------------------------
// PCIe on the MI355X box (tools/probe/host_copy.hip, 4 GB): pageable
// hipMemcpy 55-56 GB/s H2D but 48-49 GB/s D2H (and 17 GB/s on a first
// call); hipHostRegister costs ~19 GB/s, more than the copy it would speed
// up; pinned DMA 57 GB/s both ways. Four host threads, each streaming its
// stripe of a column through its own ring of pinned buffers (memcpy of one
// chunk overlapping the DMA of the previous ones), reach 55.5 H2D / 54.7 D2H.
constexpr int kStageThreads = 4;
constexpr int kStageBufs = 3;
constexpr size_t kStageChunk = size_t(32) << 20;
// below: one pageable hipMemcpy per column. Round 6 (tools/host_latency.py,
// host_rate.py; profiles/r06/host/): with ROCm 7.2 the runtime's own pageable
// copy reaches 1.06-1.12x the PCIe bound for columns of 16 MB to 2 GB, where
// the staging rings managed 1.25-2.2x; at 8 GB columns (1e9 records) the
// rings stay ahead (1.07-1.10x against 1.13x). (round 5: 16 MB)
constexpr size_t kStageMinBytesDefault = size_t(4) << 30;
constexpr size_t kPackedMaxBytes = size_t(256) << 10;       // below: all columns in one DMA
constexpr size_t kZeroCopyMaxBytes = size_t(2) << 20;       // below: kernels on host memory
size_t stage_min_bytes() {  // (SRS_STAGE_MIN_MB overrides, for experiments)
  static const size_t v = [] {
    const char* e = getenv("SRS_STAGE_MIN_MB");
    return e && *e ? (size_t)atoll(e) << 20 : kStageMinBytesDefault;
  }();
  return v;
}

struct HostStage {  // per device, kept between calls
  std::mutex mu;
  int dev = 0;
  char* pin[kStageThreads][kStageBufs] = {};
  hipStream_t cst[kStageThreads] = {};  // copy streams (one per host thread)
  hipEvent_t ev[kStageThreads][kStageBufs] = {};
  hipStream_t st = nullptr;             // the sort's stream
  char* zc = nullptr;                   // kZeroCopyMaxBytes of coherent host memory
  // freed when the last holder lets go (as Workspace)
  ~HostStage() {
    for (int t = 0; t < kStageThreads; t++) {
      if (cst[t]) (void)hipStreamSynchronize(cst[t]);
      for (int b = 0; b < kStageBufs; b++) {
        if (pin[t][b]) (void)hipHostFree(pin[t][b]);
        if (ev[t][b]) (void)hipEventDestroy(ev[t][b]);
      }
      if (cst[t]) (void)hipStreamDestroy(cst[t]);
    }
    if (st) {
      (void)hipStreamSynchronize(st);
      (void)hipStreamDestroy(st);
    }
    if (zc) (void)hipHostFree(zc);
    (void)hipGetLastError();  // (nothing above may leave a sticky error behind)
  }
};
using StageRef = std::shared_ptr<HostStage>;
std::mutex g_smu;
std::map<int, StageRef>& g_stage = *new std::map<int, StageRef>;  // (never destroyed: as g_ws)

// (the calling thread's current device is `dev`). The caller holds the
// returned reference for as long as it uses the stage, so
// srs_release_workspace can never free a stage under a running sort.
int get_stage(int dev, StageRef* out) {
  std::lock_guard<std::mutex> g(g_smu);
  auto it = g_stage.find(dev);
  if (it != g_stage.end()) {
    *out = it->second;
    return SRS_OK;
  }
  auto S = std::make_shared<HostStage>();
  S->dev = dev;
  for (int t = 0; t < kStageThreads; t++) {
    HIP_TRY(hipStreamCreateWithFlags(&S->cst[t], hipStreamNonBlocking));
    for (int b = 0; b < kStageBufs; b++) {
      HIP_TRY(hipHostMalloc((void**)&S->pin[t][b], kStageChunk, hipHostMallocDefault));
      HIP_TRY(hipEventCreateWithFlags(&S->ev[t][b], hipEventDisableTiming));
    }
  }
  HIP_TRY(hipStreamCreateWithFlags(&S->st, hipStreamNonBlocking));
  HIP_TRY(hipHostMalloc((void**)&S->zc, kZeroCopyMaxBytes, hipHostMallocCoherent));
  g_stage[dev] = S;
  *out = S;
  return SRS_OK;
}

// Drops the registry's references; each stage is freed by its last holder.
void release_host_stages() {
  std::map<int, StageRef> old;
  {
    std::lock_guard<std::mutex> g(g_smu);
    old.swap(g_stage);
  }
  old.clear();  // (outside g_smu: a destructor waits for the stage's streams)
}

// One thread's stripe [a, a + len) of a host <-> device copy through its ring.
int stage_stripe(HostStage* S, int t, char* dptr, char* hptr, size_t len, bool h2d) {
  HIP_TRY(hipSetDevice(S->dev));
  const size_t m = (len + kStageChunk - 1) / kStageChunk;
  hipStream_t cs = S->cst[t];
  auto piece = [&](size_t i, size_t* off) {
    *off = i * kStageChunk;
    return std::min(kStageChunk, len - *off);
  };
  if (h2d) {
    for (size_t i = 0; i < m; i++) {
      size_t off;
      const size_t n = piece(i, &off);
      const int b = (int)(i % kStageBufs);
      if (i >= (size_t)kStageBufs) HIP_TRY(hipEventSynchronize(S->ev[t][b]));  // its last DMA
      memcpy(S->pin[t][b], hptr + off, n);
      HIP_TRY(hipMemcpyAsync(dptr + off, S->pin[t][b], n, hipMemcpyHostToDevice, cs));
      HIP_TRY(hipEventRecord(S->ev[t][b], cs));
    }
  } else {
    for (size_t i = 0; i < m + kStageBufs; i++) {
      if (i >= (size_t)kStageBufs) {  // drain chunk i - NB (its DMA went first)
        size_t off;
        const size_t j = i - kStageBufs, n = piece(j, &off);
        const int b = (int)(j % kStageBufs);
        HIP_TRY(hipEventSynchronize(S->ev[t][b]));
        memcpy(hptr + off, S->pin[t][b], n);
      }
      if (i < m) {
        size_t off;
        const size_t n = piece(i, &off);
        const int b = (int)(i % kStageBufs);
        HIP_TRY(hipMemcpyAsync(S->pin[t][b], dptr + off, n, hipMemcpyDeviceToHost, cs));
        HIP_TRY(hipEventRecord(S->ev[t][b], cs));
      }
    }
  }
  HIP_TRY(hipStreamSynchronize(cs));
  return SRS_OK;
}

// A host <-> device copy of `bytes` (device S->dev; S->mu held by the caller).
int staged_copy(HostStage* S, char* dptr, char* hptr, size_t bytes, bool h2d) {
  if (bytes == 0) return SRS_OK;
  if (bytes < stage_min_bytes()) {
    HIP_TRY(hipMemcpy(h2d ? (void*)dptr : (void*)hptr, h2d ? (void*)hptr : (void*)dptr, bytes,
                      h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost));
    return SRS_OK;
  }
  const size_t per = align_up((bytes + kStageThreads - 1) / kStageThreads, 4096);
  int rc[kStageThreads];
  std::string err[kStageThreads];
  std::vector<std::thread> th;
  for (int t = 0; t < kStageThreads; t++) {
    rc[t] = SRS_OK;
    const size_t a = std::min(bytes, per * t), e = std::min(bytes, per * (t + 1));
    if (a >= e) continue;
    th.emplace_back([&, t, a, e] {
      rc[t] = stage_stripe(S, t, dptr + a, hptr + a, e - a, h2d);
      if (rc[t] != SRS_OK) err[t] = g_err;  // (thread-local message)
    });
  }
  for (auto& x : th) x.join();
  for (int t = 0; t < kStageThreads; t++)
    if (rc[t] != SRS_OK) return fail(rc[t], err[t]);
  return SRS_OK;
}

// Restores the calling thread's current device on scope exit.
struct DeviceGuard {
  int dev = -1;
  DeviceGuard() { (void)hipGetDevice(&dev); }
  ~DeviceGuard() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
};

size_t col_width(const Request& R, int c) { return R.aos ? R.elem_size : R.widths[c]; }

// One device: every column staged into HBM (W->stage), sorted there in
// place, copied back.
int host_sort_single(Request& R, int dev) {
  DeviceGuard keep;
  HIP_TRY(hipSetDevice(dev));
  StageRef Sref;
  SRS_TRY(get_stage(dev, &Sref));
  HostStage* S = Sref.get();
  std::lock_guard<std::mutex> slk(S->mu);
  Workspace* W = nullptr;
  WsLock lk;
  SRS_TRY(acquire_ws(&W, &lk));
  std::vector<size_t> off;
  size_t total = 0;
  for (int c = 0; c < R.ncols; c++) {
    off.push_back(total);
    total += align_up((size_t)R.num * col_width(R, c), 256);
  }
  hipStream_t st = S->st;
  WsUse use;
  SRS_TRY(use.begin(W, st));
  SRS_TRY(sync_poll(st));  // (the previous call's kernels may still read stage)
  Request D = R;
  if (total <= kZeroCopyMaxBytes && R.nsegs == 0) {
    // the kernels read and write the columns in coherent host memory
    // themselves (no DMA commands: a small or mid-size sort's PCIe round
    // trips cost less than two copy launches and their waits)
    for (int c = 0; c < R.ncols; c++) {
      memcpy(S->zc + off[c], R.in_cols[c], (size_t)R.num * col_width(R, c));
      D.in_cols[c] = D.out_cols[c] = S->zc + off[c];
    }
    SRS_TRY(run_sort(W, D, st));
    SRS_TRY(sync_poll(st));
    for (int c = 0; c < R.ncols; c++)
      memcpy(R.out_cols[c], S->zc + off[c], (size_t)R.num * col_width(R, c));
    return SRS_OK;
  }
  SRS_TRY(ensure(W->stage, total));
  for (int c = 0; c < R.ncols; c++) D.in_cols[c] = D.out_cols[c] = (char*)W->stage.p + off[c];
  if (total <= kPackedMaxBytes) {
    // small: every column packed into one pinned buffer, one DMA each way (a
    // pageable hipMemcpy per column and direction cost ~10-15 us each: 80 us
    // per call of <= 8192 records of a key and a payload). Larger copies keep
    // the pageable / staged paths, which overlap the host copy with the DMA.
    char* pin = S->pin[0][0];
    for (int c = 0; c < R.ncols; c++)
      memcpy(pin + off[c], R.in_cols[c], (size_t)R.num * col_width(R, c));
    HIP_TRY(hipMemcpyAsync(W->stage.p, pin, total, hipMemcpyHostToDevice, st));
    SRS_TRY(run_sort(W, D, st));
    HIP_TRY(hipMemcpyAsync(pin, W->stage.p, total, hipMemcpyDeviceToHost, st));
    SRS_TRY(sync_poll(st));
    for (int c = 0; c < R.ncols; c++)
      memcpy(R.out_cols[c], pin + off[c], (size_t)R.num * col_width(R, c));
    return SRS_OK;
  }
  for (int c = 0; c < R.ncols; c++)
    SRS_TRY(staged_copy(S, (char*)D.in_cols[c], (char*)R.in_cols[c],
                        (size_t)R.num * col_width(R, c), true));
  SRS_TRY(run_sort(W, D, st));
  SRS_TRY(sync_poll(st));
  for (int c = 0; c < R.ncols; c++)
    SRS_TRY(staged_copy(S, (char*)D.out_cols[c], (char*)R.out_cols[c],
                        (size_t)R.num * col_width(R, c), false));
  return SRS_OK;
}

// ---- one host array over several GPUs -------------------------------------
// Shard g (device devs[g]) takes the g-th contiguous chunk of the host array
// over its own PCIe link and histograms its top key bits; the host cuts the
// bins into G key ranges of ~equal size; every shard partitions its chunk
// into the G ranges (srs_partition_device's stable LUT scatter: the first
// radix level); range h is gathered on its device, source shard by source
// shard (xGMI peer copies), sorted there and copied back to its place in the
// host array. Every byte crosses PCIe once each way, spread over G links.
// The result is stable (partition and gather keep input order), so it is
// the same array a one-GPU sort gives.
constexpr int kSplitBits = 12;
constexpr int64_t kSplitMinN = int64_t(1) << 22;

std::mutex g_hdmu;
std::vector<int> g_host_devs;  // srs_set_host_devices; empty = the current device
bool g_host_devs_set = false;

std::vector<int> host_devices() {
  std::lock_guard<std::mutex> g(g_hdmu);
  if (!g_host_devs_set) {
    g_host_devs_set = true;
    const char* e = getenv("SRS_HOST_DEVICES");  // "all" or "0,1,2,3"
    if (e && *e) {
      int ndev = 0;
      if (!strcmp(e, "all")) {
        if (hipGetDeviceCount(&ndev) == hipSuccess)
          for (int d = 0; d < ndev; d++) g_host_devs.push_back(d);
      } else {
        for (const char* p = e; *p;) {
          char* q = nullptr;
          long v = strtol(p, &q, 10);
          if (q == p) break;
          g_host_devs.push_back((int)v);
          p = *q == ',' ? q + 1 : q;
        }
      }
    }
  }
  return g_host_devs;
}

struct ShardBufs {  // device buffers of one shard, kept between calls
  int dev = 0;
  DevBuf in, part, recv, hist, lut;
};
// One split at a time: the shard buffers are shared by every split call,
// and a call uses them across all of its phases (also from its per-shard
// threads). Held for the whole of host_sort_split and by
// srs_release_workspace around freeing them. Lock order: g_split_mu, then
// g_smu / HostStage::mu, then g_wmu / Workspace::mu.
std::mutex g_split_mu;
std::vector<ShardBufs*> g_shards;  // (under g_split_mu)

void free_shard(ShardBufs* B) {
  DevBuf* bufs[] = {&B->in, &B->part, &B->recv, &B->hist, &B->lut};
  for (DevBuf* b : bufs) free_buf(*b);
}

ShardBufs* shard_bufs(int g, int dev) {  // (g_split_mu held)
  while ((int)g_shards.size() <= g) g_shards.push_back(new ShardBufs());
  ShardBufs* B = g_shards[g];
  if (B->dev != dev) {  // (another device list than last time)
    free_shard(B);
    B->dev = dev;
  }
  return B;
}

// Runs f(g) for every shard in its own thread; the first failure wins.
template <typename F>
int for_shards(int G, F f) {
  std::vector<int> rc(G, SRS_OK);
  std::vector<std::string> err(G);
  std::vector<std::thread> th;
  for (int g = 0; g < G; g++)
    th.emplace_back([&, g] {
      rc[g] = f(g);
      if (rc[g] != SRS_OK) err[g] = g_err;
    });
  for (auto& x : th) x.join();
  for (int g = 0; g < G; g++)
    if (rc[g] != SRS_OK) return fail(rc[g], err[g]);
  return SRS_OK;
}

int host_sort_split(Request& R, const std::vector<int>& devs) {
  std::lock_guard<std::mutex> split(g_split_mu);
  const int G = (int)devs.size();
  const int64_t n = R.num;
  const int ks = key_size_of(R.kind);
  const int bits = std::min(kSplitBits, 8 * ks);
  const int nbins = 1 << bits;
  SortDesc dm;
  memset(&dm, 0, sizeof dm);
  key_masks(R.kind, R.up, dm);
  std::vector<int64_t> lo(G + 1);
  for (int g = 0; g <= G; g++) lo[g] = n * g / G;
  int64_t maxchunk = 0;
  for (int g = 0; g < G; g++) maxchunk = std::max(maxchunk, lo[g + 1] - lo[g]);
  std::vector<ShardBufs*> B(G);
  std::vector<StageRef> S(G);
  for (int g = 0; g < G; g++) B[g] = shard_bufs(g, devs[g]);
  std::vector<std::vector<uint64_t>> hist(G, std::vector<uint64_t>(nbins));

  // A. H2D of every shard's chunk + its histogram
  SRS_TRY(for_shards(G, [&](int g) -> int {
    HIP_TRY(hipSetDevice(devs[g]));
    SRS_TRY(get_stage(devs[g], &S[g]));
    std::lock_guard<std::mutex> slk(S[g]->mu);
    std::vector<size_t> off(R.ncols + 1);
    size_t t = 0;
    for (int c = 0; c < R.ncols; c++) {
      off[c] = t;
      t += align_up((size_t)maxchunk * R.widths[c], 256);
    }
    SRS_TRY(ensure(B[g]->in, t));
    SRS_TRY(ensure(B[g]->part, t));
    SRS_TRY(ensure(B[g]->hist, nbins * sizeof(uint64_t)));
    const int64_t m = lo[g + 1] - lo[g];
    for (int c = 0; c < R.ncols; c++)
      SRS_TRY(staged_copy(S[g].get(), (char*)B[g]->in.p + off[c],
                          (char*)R.in_cols[c] + (size_t)lo[g] * R.widths[c],
                          (size_t)m * R.widths[c], true));
    hipStream_t st = S[g]->st;
    HIP_TRY(hipMemsetAsync(B[g]->hist.p, 0, nbins * sizeof(uint64_t), st));
    if (m > 0)
      launch_key_hist(ks, m, B[g]->in.p, dm, bits, (unsigned long long*)B[g]->hist.p, st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(hist[g].data(), B[g]->hist.p, nbins * sizeof(uint64_t),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return SRS_OK;
  }));

  // the bins -> G contiguous key ranges of ~n/G keys (bin b goes to range
  // floor(G * (keys before b + half of b) / n), non-decreasing)
  std::vector<int32_t> lut(nbins);
  {
    double before = 0;
    int prev = 0;
    for (int b = 0; b < nbins; b++) {
      uint64_t hb = 0;
      for (int g = 0; g < G; g++) hb += hist[g][b];
      int r = (int)((before + 0.5 * (double)hb) * G / (double)n);
      r = std::min(std::max(r, prev), G - 1);
      lut[b] = prev = r;
      before += (double)hb;
    }
  }

  // B. every shard partitions its chunk into the G ranges
  std::vector<std::vector<int64_t>> cnt(G, std::vector<int64_t>(G, 0));
  SRS_TRY(for_shards(G, [&](int g) -> int {
    HIP_TRY(hipSetDevice(devs[g]));
    std::lock_guard<std::mutex> slk(S[g]->mu);
    const int64_t m = lo[g + 1] - lo[g];
    if (m == 0) return SRS_OK;
    hipStream_t st = S[g]->st;
    SRS_TRY(ensure(B[g]->lut, nbins * sizeof(int32_t)));
    HIP_TRY(hipMemcpyAsync(B[g]->lut.p, lut.data(), nbins * sizeof(int32_t),
                           hipMemcpyHostToDevice, st));
    std::vector<size_t> off(R.ncols);
    size_t t = 0;
    for (int c = 0; c < R.ncols; c++) {
      off[c] = t;
      t += align_up((size_t)maxchunk * R.widths[c], 256);
    }
    Request P = R;
    P.num = m;
    for (int c = 0; c < R.ncols; c++) {
      P.in_cols[c] = (char*)B[g]->in.p + off[c];
      P.out_cols[c] = (char*)B[g]->part.p + off[c];
    }
    if (m == 1) {  // (run_partition needs two keys) the one key's range on the host
      uint64_t kb = 0;
      HIP_TRY(hipMemcpyAsync(&kb, P.in_cols[0], ks, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      const uint64_t u = kb ^ ((kb & dm.signbit) ? dm.mneg : dm.mpos);
      cnt[g][lut[(u >> (8 * ks - bits)) & (nbins - 1)]] = 1;
      for (int c = 0; c < R.ncols; c++)
        HIP_TRY(hipMemcpyAsync(P.out_cols[c], P.in_cols[c], R.widths[c],
                               hipMemcpyDeviceToDevice, st));
      HIP_TRY(hipStreamSynchronize(st));
      return SRS_OK;
    }
    Workspace* W = nullptr;
    WsLock lk;
    SRS_TRY(acquire_ws(&W, &lk));
    WsUse use;
    SRS_TRY(use.begin(W, st));
    SRS_TRY(run_partition(W, P, bits, (const int32_t*)B[g]->lut.p, G, cnt[g].data(), st));
    HIP_TRY(hipStreamSynchronize(st));
    return SRS_OK;
  }));

  // C. range h gathered on its device (source-major: input order), sorted,
  // copied back to its place in the host array
  std::vector<int64_t> rtot(G, 0), rstart(G + 1, 0);
  for (int h = 0; h < G; h++) {
    for (int g = 0; g < G; g++) rtot[h] += cnt[g][h];
    rstart[h + 1] = rstart[h] + rtot[h];
  }
  if (rstart[G] != n) return fail(SRS_ERR_INTERNAL, "host split: partition sizes do not add up");
  for (int g = 0; g < G; g++)
    for (int h = 0; h < G; h++)
      if (devs[g] != devs[h]) {  // xGMI peer access (already enabled is fine)
        HIP_TRY(hipSetDevice(devs[h]));
        const hipError_t e = hipDeviceEnablePeerAccess(devs[g], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
      }
  return for_shards(G, [&](int h) -> int {
    HIP_TRY(hipSetDevice(devs[h]));
    std::lock_guard<std::mutex> slk(S[h]->mu);
    const int64_t m = rtot[h];
    if (m == 0) return SRS_OK;
    hipStream_t st = S[h]->st;
    std::vector<size_t> roff(R.ncols), poff(R.ncols);
    size_t t = 0, tp = 0;
    for (int c = 0; c < R.ncols; c++) {
      roff[c] = t;
      t += align_up((size_t)m * R.widths[c], 256);
      poff[c] = tp;
      tp += align_up((size_t)maxchunk * R.widths[c], 256);
    }
    SRS_TRY(ensure(B[h]->recv, t));
    Request D = R;
    D.num = m;
    D.thresh = R.leaf_mode == SRS_LEAF_UNSORTED ? R.thresh : 0;  // (no n <= thresh rule)
    for (int c = 0; c < R.ncols; c++) D.in_cols[c] = D.out_cols[c] = (char*)B[h]->recv.p + roff[c];
    int64_t at = 0;
    for (int g = 0; g < G; g++) {
      int64_t src = 0;  // range h's piece in shard g's partitioned chunk
      for (int q = 0; q < h; q++) src += cnt[g][q];
      const int64_t len = cnt[g][h];
      for (int c = 0; c < R.ncols && len > 0; c++) {
        const size_t w = R.widths[c];
        char* dst = (char*)D.in_cols[c] + (size_t)at * w;
        const char* from = (const char*)B[g]->part.p + poff[c] + (size_t)src * w;
        if (devs[g] == devs[h])
          HIP_TRY(hipMemcpyAsync(dst, from, (size_t)len * w, hipMemcpyDeviceToDevice, st));
        else
          HIP_TRY(hipMemcpyPeerAsync(dst, devs[h], from, devs[g], (size_t)len * w, st));
      }
      at += len;
    }
    {
      Workspace* W = nullptr;
      WsLock lk;
      SRS_TRY(acquire_ws(&W, &lk));
      if (m > 1 && !whole_input_is_unsorted_leaf(D)) {
        if (m <= kLocalCap) {
          SRS_TRY(run_small(W, D, st));
        } else {
          WsUse use;
          SRS_TRY(use.begin(W, st));
          SRS_TRY(run_sort(W, D, st));
        }
      }
      HIP_TRY(hipStreamSynchronize(st));
    }
    for (int c = 0; c < R.ncols; c++)
      SRS_TRY(staged_copy(S[h].get(), (char*)D.out_cols[c],
                          (char*)R.out_cols[c] + (size_t)rstart[h] * R.widths[c],
                          (size_t)m * R.widths[c], false));
    return SRS_OK;
  });
}

int sort_host(Request& R) {
  if (R.num <= 1 || whole_input_is_unsorted_leaf(R)) return SRS_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(SRS_ERR_NO_DEVICE, "no HIP device available");
  const std::vector<int> devs = host_devices();
  for (int d : devs)
    if (d < 0 || d >= ndev) return fail(SRS_ERR_INVALID_ARG, "host device list: no such device");
  // the split needs SoA columns, a size worth G PCIe links, and n > thresh
  // (its shards are sub-ranges of one sort: no whole-input leaf rule)
  if (devs.size() > 1 && !R.aos && R.num >= kSplitMinN && R.num > R.thresh) {
    DeviceGuard keep;
    return host_sort_split(R, devs);
  }
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  return host_sort_single(R, devs.empty() ? dev : devs[0]);
}

int build_soa(Request& R, int64_t num, int kind, int up, int64_t thresh, void* keys,
              int32_t np, void* const* pays, const uint32_t* sizes, void* keys_out,
              void* const* pays_out) {
  SRS_TRY(validate_common(num, kind));
  if (np < 0 || np > SRS_MAX_PAYLOADS) return fail(SRS_ERR_INVALID_ARG, "num_payloads out of range");
  if (num > 1 && !keys) return fail(SRS_ERR_INVALID_ARG, "keys is NULL");
  if (np > 0 && (!pays || !sizes)) return fail(SRS_ERR_INVALID_ARG, "payload arrays missing");
  if ((keys_out && np > 0 && !pays_out) || (!keys_out && pays_out))
    return fail(SRS_ERR_INVALID_ARG, "keys_out and payloads_out must both be set or both NULL");
  R.num = num;
  R.kind = kind;
  R.up = up ? 1 : 0;
  R.thresh = thresh;
  R.aos = false;
  R.elem_size = 0;
  R.ncols = 1 + np;
  R.in_cols[0] = keys;
  R.out_cols[0] = keys_out ? keys_out : keys;
  R.widths[0] = (uint32_t)key_size_of(kind);
  for (int i = 0; i < np; i++) {
    const uint32_t w = sizes[i];
    if (w != 1 && w != 2 && w != 4 && w != 8)
      return fail(SRS_ERR_UNSUPPORTED, "payload sizes must be 1, 2, 4 or 8 bytes");
    if (num > 1 && !pays[i]) return fail(SRS_ERR_INVALID_ARG, "payload pointer is NULL");
    R.in_cols[1 + i] = pays[i];
    R.out_cols[1 + i] = keys_out ? pays_out[i] : pays[i];
    R.widths[1 + i] = w;
  }
  return SRS_OK;
}

// Device columns are read and written as whole 1/2/4/8-byte words, so every
// device pointer must be aligned to its word (hipMalloc and torch
// allocations always are). Host arrays may be unaligned, as in the reference
// (loadu, src/simd.hpp): they are staged through HBM.
int check_device_alignment(const Request& R) {
  if (R.num <= 1) return SRS_OK;
  for (int c = 0; c < R.ncols; c++) {
    const uint32_t a = R.aos ? (R.elem_size < 8 ? R.elem_size : 8) : R.widths[c];
    if (((uintptr_t)R.in_cols[c] | (uintptr_t)R.out_cols[c]) % a != 0)
      return fail(SRS_ERR_INVALID_ARG, "device arrays must be aligned to their element size "
                                       "(records: to min(elem_size, 8))");
  }
  return SRS_OK;
}

int build_aos(Request& R, int64_t num, int kind, int up, int64_t thresh, void* elems,
              uint32_t esz, void* elems_out) {
  SRS_TRY(validate_common(num, kind));
  const int ks = key_size_of(kind);
  // static_assert(is_power_of_two<sizeof(DataElement<K, Ps...>)>),
  // radixSort.hpp:1774
  if (esz < (uint32_t)ks || esz > 64 || (esz & (esz - 1)) != 0)
    return fail(SRS_ERR_UNSUPPORTED,
                "elem_size must be a power of two in [sizeof(key), 64]");
  if (num > 1 && !elems) return fail(SRS_ERR_INVALID_ARG, "elements is NULL");
  R.num = num;
  R.kind = kind;
  R.up = up ? 1 : 0;
  R.thresh = thresh;
  R.aos = true;
  R.elem_size = esz;
  R.ncols = 1;
  R.in_cols[0] = elems;
  R.out_cols[0] = elems_out ? elems_out : elems;
  R.widths[0] = esz;
  return SRS_OK;
}

int set_leaf_mode(Request& R, int leaf_mode) {
  if (leaf_mode != SRS_LEAF_SORTED && leaf_mode != SRS_LEAF_UNSORTED)
    return fail(SRS_ERR_INVALID_ARG, "leaf_mode must be SRS_LEAF_SORTED or SRS_LEAF_UNSORTED");
  R.leaf_mode = leaf_mode;
  return SRS_OK;
}

}  // namespace

// (other translation units of the library report errors through this)
int set_error(int code, const std::string& msg) { return fail(code, msg); }

void defer_workspace_frees(bool on) { t_defer = on; }

// Frees what defer_workspace_frees held back (the caller's exchange is over);
// returns how many buffers that was.
int64_t release_deferred_frees() {
  std::vector<std::pair<void*, int>> v;
  v.swap(t_deferred);
  for (auto& f : v) (void)big_free(f.first, f.second);
  (void)hipGetLastError();
  return (int64_t)v.size();
}

// Grows the current device's workspace so that a later
// srs_sort_segments_device of up to `num` records of these column widths
// allocates no large buffer: the multi-GPU shard reserves it before its first
// message is posted, so that no rank can fail an allocation (or wait in one)
// once its peers depend on it (srs_shard.hip).
int reserve_segments_workspace(int64_t num, int ncols, const uint32_t* widths) {
  size_t tmp_bytes = 0;
  for (int c = 0; c < ncols; c++) tmp_bytes += align_up((size_t)std::max<int64_t>(num, 1) * widths[c], 256);
  Workspace* W = nullptr;
  WsLock lk;
  SRS_TRY(acquire_ws(&W, &lk));
  if (W->tmp.p && W->tmp.bytes >= tmp_bytes) return SRS_OK;
  if (W->idle && W->idle_pending) HIP_TRY(hipEventSynchronize(W->idle));  // (the old TMP's last use)
  return ensure(W->tmp, tmp_bytes, ws_alloc_mode(), true);
}
}  // namespace srs

using namespace srs;

extern "C" {

int srs_sort_soa(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold, void* keys,
                 int32_t num_payloads, void* const* payloads, const uint32_t* payload_sizes) {
  Request R;
  SRS_TRY(build_soa(R, num, key_kind, up, cmp_sort_threshold, keys, num_payloads, payloads,
                    payload_sizes, nullptr, nullptr));
  return sort_host(R);
}

int srs_sort_aos(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                 void* elements, uint32_t elem_size) {
  Request R;
  SRS_TRY(build_aos(R, num, key_kind, up, cmp_sort_threshold, elements, elem_size, nullptr));
  return sort_host(R);
}

int srs_sort_soa_leaf(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                      int leaf_mode, void* keys, int32_t num_payloads, void* const* payloads,
                      const uint32_t* payload_sizes) {
  Request R;
  SRS_TRY(build_soa(R, num, key_kind, up, cmp_sort_threshold, keys, num_payloads, payloads,
                    payload_sizes, nullptr, nullptr));
  SRS_TRY(set_leaf_mode(R, leaf_mode));
  return sort_host(R);
}

int srs_sort_aos_leaf(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                      int leaf_mode, void* elements, uint32_t elem_size) {
  Request R;
  SRS_TRY(build_aos(R, num, key_kind, up, cmp_sort_threshold, elements, elem_size, nullptr));
  SRS_TRY(set_leaf_mode(R, leaf_mode));
  return sort_host(R);
}

int srs_sort_soa_device_leaf(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                             int leaf_mode, void* keys, int32_t num_payloads,
                             void* const* payloads, const uint32_t* payload_sizes,
                             void* keys_out, void* const* payloads_out, void* stream) {
  Request R;
  SRS_TRY(build_soa(R, num, key_kind, up, cmp_sort_threshold, keys, num_payloads, payloads,
                    payload_sizes, keys_out, payloads_out));
  SRS_TRY(set_leaf_mode(R, leaf_mode));
  SRS_TRY(check_device_alignment(R));
  return sort_device(R, (hipStream_t)stream);
}

int srs_sort_aos_device_leaf(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                             int leaf_mode, void* elements, uint32_t elem_size,
                             void* elements_out, void* stream) {
  Request R;
  SRS_TRY(build_aos(R, num, key_kind, up, cmp_sort_threshold, elements, elem_size,
                    elements_out));
  SRS_TRY(set_leaf_mode(R, leaf_mode));
  SRS_TRY(check_device_alignment(R));
  return sort_device(R, (hipStream_t)stream);
}

int srs_sort_soa_device(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                        void* keys, int32_t num_payloads, void* const* payloads,
                        const uint32_t* payload_sizes, void* keys_out,
                        void* const* payloads_out, void* stream) {
  Request R;
  SRS_TRY(build_soa(R, num, key_kind, up, cmp_sort_threshold, keys, num_payloads, payloads,
                    payload_sizes, keys_out, payloads_out));
  SRS_TRY(check_device_alignment(R));
  return sort_device(R, (hipStream_t)stream);
}

int srs_sort_segments_device(int64_t num, int key_kind, int up, void* keys,
                             int32_t num_payloads, void* const* payloads,
                             const uint32_t* payload_sizes, int64_t num_segments,
                             const int64_t* segment_bounds, int32_t known_top_bits,
                             void* stream) {
  if (num_segments < 0) return fail(SRS_ERR_INVALID_ARG, "num_segments < 0");
  if (known_top_bits < 0 || known_top_bits >= 8 * key_size_of(key_kind))
    return fail(SRS_ERR_INVALID_ARG, "known_top_bits out of range");
  if (num_segments > 0 && !segment_bounds) return fail(SRS_ERR_INVALID_ARG, "segment_bounds is NULL");
  for (int64_t i = 0; i < num_segments; i++)
    if (segment_bounds[i] < 0 || segment_bounds[i] > segment_bounds[i + 1] ||
        segment_bounds[i + 1] > num)
      return fail(SRS_ERR_INVALID_ARG, "segment_bounds must be non-decreasing within [0, num]");
  Request R;
  SRS_TRY(build_soa(R, num, key_kind, up, 0, keys, num_payloads, payloads, payload_sizes,
                    nullptr, nullptr));
  SRS_TRY(check_device_alignment(R));
  if (num_segments == 0 || num <= 1) return SRS_OK;
  R.seg_bounds = segment_bounds;
  R.nsegs = num_segments;
  R.known_top_bits = known_top_bits;
  Workspace* W = nullptr;
  WsLock lk;
  SRS_TRY(acquire_ws(&W, &lk));
  WsUse use;
  SRS_TRY(use.begin(W, (hipStream_t)stream));
  return run_sort(W, R, (hipStream_t)stream);
}

int srs_sort_aos_device(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                        void* elements, uint32_t elem_size, void* elements_out,
                        void* stream) {
  Request R;
  SRS_TRY(build_aos(R, num, key_kind, up, cmp_sort_threshold, elements, elem_size,
                    elements_out));
  SRS_TRY(check_device_alignment(R));
  return sort_device(R, (hipStream_t)stream);
}

int srs_fill_synthetic_device(int64_t num, int key_kind, uint64_t seed, uint64_t first_index,
                              void* keys, int32_t num_payloads, void* const* payloads,
                              const uint32_t* payload_sizes, void* stream) {
  if (key_size_of(key_kind) == 0) return fail(SRS_ERR_INVALID_ARG, "invalid key_kind");
  if (num_payloads < 0 || num_payloads > SRS_MAX_PAYLOADS)
    return fail(SRS_ERR_INVALID_ARG, "num_payloads out of range");
  if (num <= 0) return SRS_OK;
  hipStream_t st = (hipStream_t)stream;
  Col cols[SRS_MAX_PAYLOADS];
  for (int i = 0; i < num_payloads; i++) {
    const uint32_t w = payload_sizes[i];
    if (w != 1 && w != 2 && w != 4 && w != 8)
      return fail(SRS_ERR_UNSUPPORTED, "payload sizes must be 1, 2, 4 or 8 bytes");
    cols[i] = Col{{(char*)payloads[i], nullptr, nullptr, nullptr}, w, {w, w, w, w}};
  }
  void* d_cols = nullptr;
  if (num_payloads > 0) {
    HIP_TRY(hipMalloc(&d_cols, sizeof(Col) * num_payloads));
    HIP_TRY(hipMemcpy(d_cols, cols, sizeof(Col) * num_payloads, hipMemcpyHostToDevice));
  }
  launch_fill(num, key_kind, seed, first_index, keys, num_payloads, (const Col*)d_cols, st);
  HIP_TRY(hipGetLastError());
  if (d_cols) {
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipFree(d_cols));
  }
  return SRS_OK;
}

int srs_key_histogram_device(int64_t num, int key_kind, int up, const void* keys, int bits,
                             uint64_t* hist, void* stream) {
  const int ks = key_size_of(key_kind);
  if (ks == 0) return fail(SRS_ERR_INVALID_ARG, "invalid key_kind");
  if (bits < 1 || bits > kHistMaxBits || bits > 8 * ks)
    return fail(SRS_ERR_INVALID_ARG, "bits must be in [1, min(12, key bits)]");
  if (num <= 0) return SRS_OK;
  if (!keys || !hist) return fail(SRS_ERR_INVALID_ARG, "NULL pointer");
  if ((uintptr_t)keys % ks != 0 || (uintptr_t)hist % 8 != 0)
    return fail(SRS_ERR_INVALID_ARG, "device arrays must be aligned to their element size");
  SortDesc d;
  memset(&d, 0, sizeof d);
  key_masks(key_kind, up, d);
  launch_key_hist(ks, num, keys, d, bits, (unsigned long long*)hist, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return SRS_OK;
}

int srs_partition_device(int64_t num, int key_kind, int up, const void* keys,
                         int32_t num_payloads, const void* const* payloads,
                         const uint32_t* payload_sizes, int bits, const int32_t* part_of_bucket,
                         int32_t num_parts, void* keys_out, void* const* payloads_out,
                         int64_t* part_counts, void* stream) {
  const int ks = key_size_of(key_kind);
  if (ks == 0) return fail(SRS_ERR_INVALID_ARG, "invalid key_kind");
  if (bits < 1 || bits > 16 || bits > 8 * ks)
    return fail(SRS_ERR_INVALID_ARG, "bits must be in [1, min(16, key bits)]");
  if (num_parts < 1 || num_parts > kMaxBins)
    return fail(SRS_ERR_INVALID_ARG, "num_parts must be in [1, 512]");
  if (!part_counts || !part_of_bucket) return fail(SRS_ERR_INVALID_ARG, "NULL pointer");
  for (int p = 0; p < num_parts; p++) part_counts[p] = 0;
  if (num <= 0) return SRS_OK;
  Request R;
  SRS_TRY(build_soa(R, num, key_kind, up, 0, (void*)keys, num_payloads, (void* const*)payloads,
                    payload_sizes, keys_out, payloads_out));
  if (!keys_out) return fail(SRS_ERR_INVALID_ARG, "keys_out is NULL");
  SRS_TRY(check_device_alignment(R));
  if (num == 1) {
    // a single key: its group from the table, then a plain copy
    int32_t one = 0;
    SortDesc d;
    memset(&d, 0, sizeof d);
    key_masks(key_kind, up, d);
    uint64_t bitsv = 0;
    HIP_TRY(hipMemcpy(&bitsv, keys, ks, hipMemcpyDeviceToHost));
    uint64_t u = bitsv ^ ((bitsv & d.signbit) ? d.mneg : d.mpos);
    HIP_TRY(hipMemcpy(&one, part_of_bucket + (u >> (8 * ks - bits)), 4, hipMemcpyDeviceToHost));
    if (one < 0 || one >= num_parts) return fail(SRS_ERR_INVALID_ARG, "part id out of range");
    part_counts[one] = 1;
    return copy_through(R, (hipStream_t)stream);
  }
  Workspace* W = nullptr;
  WsLock lk;
  SRS_TRY(acquire_ws(&W, &lk));
  WsUse use;
  SRS_TRY(use.begin(W, (hipStream_t)stream));
  return run_partition(W, R, bits, part_of_bucket, num_parts, part_counts, (hipStream_t)stream);
}

const char* srs_last_error(void) { return g_err.c_str(); }

#ifndef SRS_SRC_HASH
#define SRS_SRC_HASH "unknown"
#endif
const char* srs_version(void) { return "srs_amd 0.1.0 gfx950 src:" SRS_SRC_HASH; }

int srs_set_host_devices(int32_t num_devices, const int32_t* devices) {
  if (num_devices < 0 || num_devices > 512 || (num_devices > 0 && !devices))
    return fail(SRS_ERR_INVALID_ARG, "num_devices must be in [0, 512] with a device array");
  int ndev = 0;
  if (num_devices > 0 && (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0))
    return fail(SRS_ERR_NO_DEVICE, "no HIP device available");
  for (int i = 0; i < num_devices; i++)
    if (devices[i] < 0 || devices[i] >= ndev)
      return fail(SRS_ERR_INVALID_ARG, "no such device in the host device list");
  std::lock_guard<std::mutex> g(g_hdmu);
  g_host_devs.assign(devices, devices + num_devices);
  g_host_devs_set = true;
  return SRS_OK;
}

int srs_set_kernel_timing(int enable) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_timing = enable == 2 ? 2 : enable != 0;
  return SRS_OK;
}

int srs_reset_kernel_stats(void) {
  std::lock_guard<std::mutex> lk(g_tmu);
  drain_timing_locked();
  g_stats.clear();
  return SRS_OK;
}

int srs_kernel_stats(const char* name, int64_t* launches, double* total_ms, double* elements) {
  std::lock_guard<std::mutex> lk(g_tmu);
  drain_timing_locked();
  if (!name) return fail(SRS_ERR_INVALID_ARG, "name is NULL");
  auto it = g_stats.find(name);
  const KStat k = it == g_stats.end() ? KStat{} : it->second;
  if (launches) *launches = k.launches;
  if (total_ms) *total_ms = k.ms;
  if (elements) *elements = k.elems;
  return SRS_OK;
}

int srs_debug_set_stamp_buffer(void* device_acc) {
  g_stamp_acc = (unsigned long long*)device_acc;
  return SRS_OK;
}

// (diagnostic builds, SRS_DIAG_LOOKBACK: status words of at least ntiles * 512
// u32, zeroed by the caller before every level, and 4 u64 error counters)
int srs_debug_set_lookback(void* status, void* err) {
  g_lb_status = (uint32_t*)status;
  g_lb_err = (unsigned long long*)err;
  return SRS_OK;
}

int srs_debug_last_local_counts(int64_t* counts) {
  if (!counts) return fail(SRS_ERR_INVALID_ARG, "counts is NULL");
  Workspace* W = nullptr;
  WsLock lk;
  SRS_TRY(acquire_ws(&W, &lk));
  counts[0] = counts[1] = 0;
  if (W->last_small || !W->ctr.p) return SRS_OK;
  HIP_TRY(hipDeviceSynchronize());
  ListCounters c;
  HIP_TRY(hipMemcpy(&c, W->ctr.p, sizeof c, hipMemcpyDeviceToHost));
  counts[0] = (int64_t)(c.n_local + c.n_local2);
  counts[1] = (int64_t)(c.n_redo + c.n_redo2);
  return SRS_OK;
}

int srs_debug_last_local_classes(int64_t* counts) {
  if (!counts) return fail(SRS_ERR_INVALID_ARG, "counts is NULL");
  Workspace* W = nullptr;
  WsLock lk;
  SRS_TRY(acquire_ws(&W, &lk));
  counts[0] = counts[1] = counts[2] = counts[3] = 0;
  if (W->last_small || !W->ctr.p) return SRS_OK;
  HIP_TRY(hipDeviceSynchronize());
  ListCounters c;
  HIP_TRY(hipMemcpy(&c, W->ctr.p, sizeof c, hipMemcpyDeviceToHost));
  counts[0] = (int64_t)c.n_local;
  counts[1] = (int64_t)c.n_local2;
  counts[2] = (int64_t)c.n_redo;
  counts[3] = (int64_t)c.n_redo2;
  return SRS_OK;
}

int srs_debug_set_super_scan(int64_t min_groups) {
  set_super_scan_min_groups(min_groups);
  return SRS_OK;
}

int srs_debug_last_fallbacks(int64_t* counts) {
  if (!counts) return fail(SRS_ERR_INVALID_ARG, "counts is NULL");
  Workspace* W = nullptr;
  WsLock lk;
  SRS_TRY(acquire_ws(&W, &lk));
  counts[0] = counts[1] = 0;
  if (W->last_small) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(counts, W->small_taken[W->last_small_stream].p, 2 * sizeof(int64_t),
                      hipMemcpyDeviceToHost));
    return SRS_OK;
  }
  if (!W->ctr.p) return SRS_OK;
  HIP_TRY(hipDeviceSynchronize());
  ListCounters c;
  HIP_TRY(hipMemcpy(&c, W->ctr.p, sizeof c, hipMemcpyDeviceToHost));
  counts[0] = (int64_t)(c.n_fallback + c.n_fallback1);
  counts[1] = (int64_t)c.n_fallback2;
  return SRS_OK;
}

int srs_debug_plan_table(const uint32_t* hist, int64_t num, int key_bits, int32_t* mode,
                         int32_t* groups, double* overflow, double* overflow_other,
                         int32_t* table, int32_t* rbits) {
  if (!hist || !mode || !table || !rbits || (key_bits != 32 && key_bits != 64) || num < 1)
    return fail(SRS_ERR_INVALID_ARG, "srs_debug_plan_table: arguments");
  std::vector<uint32_t> h(hist, hist + 65536);
  TablePlan P;
  plan_table(h, num, key_bits, &P);
  *mode = P.mode;
  if (groups) *groups = P.groups;
  if (overflow) *overflow = P.over;
  if (overflow_other) *overflow_other = P.over_other;
  if (P.mode == 1) memcpy(table, P.lut16.data(), 65536 * 4);
  if (P.mode == 3) memcpy(table, P.tab3.data(), 512 * 4);
  if (P.mode) memcpy(rbits, P.rbits.data(), kGroups * 4);
  return SRS_OK;
}

int srs_alloc_device(uint64_t bytes, void** ptr) {
  if (!ptr) return fail(SRS_ERR_INVALID_ARG, "srs_alloc_device: ptr is NULL");
  *ptr = nullptr;
  if (bytes == 0) return SRS_OK;
  HIP_TRY(placed_alloc(ptr, (size_t)bytes, ALLOC_MALLOC));
  std::lock_guard<std::mutex> g(g_pub_amu);
  g_pub_allocs[*ptr] = (size_t)bytes;
  return SRS_OK;
}

int srs_free_device(void* ptr) {
  if (!ptr) return SRS_OK;
  {
    std::lock_guard<std::mutex> g(g_pub_amu);
    auto it = g_pub_allocs.find(ptr);
    if (it == g_pub_allocs.end())
      return fail(SRS_ERR_INVALID_ARG, "srs_free_device: not from srs_alloc_device");
    g_pub_allocs.erase(it);
  }
  HIP_TRY(hipFree(ptr));
  return SRS_OK;
}

std::mutex g_dbg_amu;
std::map<void*, int> g_dbg_allocs;  // srs_debug_alloc: pointer -> mode

int srs_debug_alloc(uint64_t bytes, int mode, void** ptr) {
  if (!ptr || mode < ALLOC_MALLOC || mode >= ALLOC_MODES || bytes == 0)
    return fail(SRS_ERR_INVALID_ARG, "srs_debug_alloc: ptr, mode 0..4 and bytes > 0");
  HIP_TRY(big_alloc(ptr, (size_t)bytes, mode));
  std::lock_guard<std::mutex> g(g_dbg_amu);
  g_dbg_allocs[*ptr] = mode;
  return SRS_OK;
}

int srs_debug_free(void* ptr) {
  int mode = 0;
  {
    std::lock_guard<std::mutex> g(g_dbg_amu);
    auto it = g_dbg_allocs.find(ptr);
    if (it == g_dbg_allocs.end()) return fail(SRS_ERR_INVALID_ARG, "srs_debug_free: unknown pointer");
    mode = it->second;
    g_dbg_allocs.erase(it);
  }
  HIP_TRY(big_free(ptr, mode));
  return SRS_OK;
}

int srs_debug_probe_write(void* ptr, uint64_t bytes, float* ms) {
  if (!ptr || !ms) return fail(SRS_ERR_INVALID_ARG, "srs_debug_probe_write: ptr and ms");
  hipStream_t ps = nullptr;
  HIP_TRY(hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
  *ms = probe_write_ms(ptr, (size_t)bytes, ps);
  (void)hipStreamDestroy(ps);
  HIP_TRY(hipGetLastError());
  return SRS_OK;
}

int srs_debug_workspace(void** tmp, uint64_t* tmp_bytes, void** tmp2, uint64_t* tmp2_bytes) {
  Workspace* W = nullptr;
  WsLock lk;
  SRS_TRY(acquire_ws(&W, &lk));
  if (tmp) *tmp = W->tmp.p;
  if (tmp_bytes) *tmp_bytes = W->tmp.bytes;
  if (tmp2) *tmp2 = W->tmp2.p;
  if (tmp2_bytes) *tmp2_bytes = W->tmp2.bytes;
  return SRS_OK;
}

int srs_release_workspace(void) {
  release_host_stages();
  {
    std::lock_guard<std::mutex> g(g_split_mu);  // (waits for a running split)
    for (ShardBufs* B : g_shards) {
      free_shard(B);
      delete B;
    }
    g_shards.clear();
  }
  std::map<int, std::shared_ptr<Workspace>> old;
  {
    std::lock_guard<std::mutex> lk(g_wmu);
    old.swap(g_ws);
  }
  old.clear();  // each workspace is freed by its last holder (~Workspace)
  (void)hipGetLastError();
  return SRS_OK;
}

}  // extern "C"

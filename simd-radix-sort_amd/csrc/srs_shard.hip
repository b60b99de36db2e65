// srs_shard.hip — the multi-GPU shard sort behind the C ABI (srs_shard_*):
// one array spread over N GPUs is sorted across them, rank r ending with the
// r-th key range. This is the one implementation of the protocol: C/C++
// callers, bench.py --gpus N (through ctypes) and the tests all run it.
//
// Protocol:
//   1. per input chunk, a histogram of the transformed top 12 key bits
//      (srs_key_histogram_device); their sum is all-reduced together with a
//      header every rank must agree on (key kind, direction, payload sizes,
//      chunks, rounds) and each rank's status;
//   2. the 4096 bins -> 512 key-range groups of ~equal size, contiguous runs
//      of groups -> ranks (ShardPlan::split: identical on every rank, since
//      every rank sees the same histogram);
//   3. every rank's group sizes per chunk are all-gathered (exact: a group is
//      a union of bins), so every receive is sized before any data moves.
//      Every buffer, and the round sorts' workspace, is allocated before the
//      first message, and a status all-reduce makes one rank's failed
//      allocation every rank's failure;
//   4. the input is partitioned chunk by chunk into the groups
//      (srs_partition_device: the sort's first radix level), each chunk's
//      first-round messages posted as soon as it is partitioned;
//   5. every later round is posted right after the partition (grouped
//      send/recv, one message per (round, peer, chunk, column), <= 256 MB
//      each: RCCL returns messages above 1 GiB corrupted) on a
//      communication stream, so the links stay busy; round r's key range is
//      sorted on a side stream (srs_sort_segments_device) once it is in;
//   6. a last status all-reduce. A rank whose partition or round sort failed
//      after the first message kept to the message plan (its peers wait for
//      nothing that never comes) and now fails every rank. A transport
//      failure aborts the communicator instead; every host wait on peers is
//      bounded (SRS_SHARD_TIMEOUT_S, 600 s by default).
// Equal keys share a group; inside a round they arrive in (source rank,
// chunk, input index) order, so the whole sort is stable.
//
// The collectives and the peer messages go through a Transport: RCCL over
// xGMI (the product), or a host-staged one that lets several ranks share one
// GPU as threads of one process (tests; RCCL puts no two ranks on one
// device). Nothing else in the protocol knows which one runs.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/srs_c_api.h"
#include "srs_kernels.h"

namespace srs {
int set_error(int code, const std::string& msg);                                  // (srs_api.hip)
int reserve_segments_workspace(int64_t num, int ncols, const uint32_t* widths);  // (srs_api.hip)
// workspace frees of this thread held back while peers' messages are queued
// on the device (a hipFree would wait for them, unbounded); srs_api.hip
void defer_workspace_frees(bool on);
int64_t release_deferred_frees();

namespace {

// ---- RCCL, resolved at first use (the library itself does not need it) ----
struct Rccl {
  bool ok = false;
  std::string why;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*CommAbort)(ncclComm_t);
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*);
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t);
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
  const char* (*GetErrorString)(ncclResult_t);
};

const Rccl& rccl() {
  static Rccl R;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      R.why = std::string("RCCL not found: ") + dlerror();
      return;
    }
    bool ok = true;
    auto sym = [&](auto& f, const char* name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
      if (!f) {
        ok = false;
        R.why = std::string("RCCL lacks ") + name;
      }
    };
    sym(R.GetUniqueId, "ncclGetUniqueId");
    sym(R.CommInitRank, "ncclCommInitRank");
    sym(R.CommInitAll, "ncclCommInitAll");
    sym(R.CommDestroy, "ncclCommDestroy");
    sym(R.CommAbort, "ncclCommAbort");
    sym(R.CommGetAsyncError, "ncclCommGetAsyncError");
    sym(R.AllReduce, "ncclAllReduce");
    sym(R.AllGather, "ncclAllGather");
    sym(R.Send, "ncclSend");
    sym(R.Recv, "ncclRecv");
    sym(R.GroupStart, "ncclGroupStart");
    sym(R.GroupEnd, "ncclGroupEnd");
    sym(R.GetErrorString, "ncclGetErrorString");
    R.ok = ok;
  });
  return R;
}

int hip_rc(hipError_t e, const char* what) {
  if (e == hipSuccess) return SRS_OK;
  return set_error(e == hipErrorOutOfMemory ? SRS_ERR_OUT_OF_MEMORY : SRS_ERR_HIP,
                   std::string(what) + " -> " + hipGetErrorString(e));
}

int nccl_rc(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return SRS_OK;
  return set_error(SRS_ERR_HIP, std::string(what) + " -> " + rccl().GetErrorString(r));
}

#define SH_HIP(expr)                                   \
  do {                                                 \
    const int r_ = hip_rc((expr), #expr);              \
    if (r_ != SRS_OK) return r_;                       \
  } while (0)

constexpr int kBits = 12;                        // histogram bits
constexpr int kHistBins = 1 << kBits;
constexpr int kGroups = 512;                     // key-range groups
constexpr int kMaxChunks = 16;                   // partition chunks
constexpr int kMaxRounds = 64;                   // exchange rounds
// (world > 1. Round 6: the world-1 line with the 8-rank plan measured one
// rank's HBM work at 41.1 ms with 8 rounds / 4 chunks against 44.7 ms with
// 16 / 8 -- each round sort and each partition chunk costs fixed stalls --
// while the rounds' tail grows 0.65 -> 1.0 ms)
constexpr int kDefaultChunks = 4;                // (world 1: one chunk)
constexpr int kDefaultRounds = 8;                // (world 1: 8)
constexpr int kDefaultRounds1 = 8;
constexpr int kHdr = 18;                         // header slots after the histogram
constexpr size_t kMsgBytes = size_t(256) << 20;  // largest message (default)
constexpr int64_t kMsgBytesMax = int64_t(1) << 30;  // RCCL corrupts larger ones

double timeout_s() {
  const char* e = getenv("SRS_SHARD_TIMEOUT_S");
  const double t = e && *e ? atof(e) : 600.0;
  return t > 0 ? t : 600.0;
}

int key_bytes(int kind) {
  switch (kind) {
    case SRS_KEY_U8: case SRS_KEY_I8: return 1;
    case SRS_KEY_U16: case SRS_KEY_I16: return 2;
    case SRS_KEY_U32: case SRS_KEY_I32: case SRS_KEY_F32: return 4;
    case SRS_KEY_U64: case SRS_KEY_I64: case SRS_KEY_F64: return 8;
    default: return 0;
  }
}

std::string rank_list(uint64_t mask) {
  std::string s;
  for (int r = 0; r < 64; r++)
    if (mask >> r & 1) s += (s.empty() ? "" : ",") + std::to_string(r);
  return s.empty() ? "?" : s;
}

// ---------------------------------------------------------------------------
// the transport seam
// ---------------------------------------------------------------------------
struct Transport {
  virtual ~Transport() {}
  virtual const char* name() const = 0;
  // in place over `count` uint64 of device memory, enqueued on st
  virtual int all_reduce_sum(uint64_t* buf, size_t count, hipStream_t st) = 0;
  // every rank's `count` int64 (device), rank order, into recv (device)
  virtual int all_gather(const int64_t* send, int64_t* recv, size_t count, hipStream_t st) = 0;
  // one group of peer messages (device buffers) on st; matched per peer pair
  // in posting order
  virtual int group_start() = 0;
  virtual int send(const void* buf, size_t bytes, int peer, hipStream_t st) = 0;
  virtual int recv(void* buf, size_t bytes, int peer, hipStream_t st) = 0;
  virtual int group_end() = 0;
  // host waits for a stream / an event; bounded, and a peer's failure ends
  // them with an error
  virtual int wait(hipStream_t st) = 0;
  virtual int wait_event(hipEvent_t e) = 0;
  virtual void abort(const std::string& why) = 0;
  virtual bool dead() const = 0;
};

// RCCL over xGMI. Comms made together by srs_shard_comm_init_all share
// `group_fail`: one aborting rank makes the others' waits abort too.
struct RcclTransport : Transport {
  ncclComm_t comm = nullptr;
  std::shared_ptr<std::atomic<int>> group_fail;
  std::atomic<bool> aborted{false};
  std::string why;

  ~RcclTransport() override {
    if (comm && !aborted) (void)rccl().CommDestroy(comm);
  }
  const char* name() const override { return "rccl"; }
  int all_reduce_sum(uint64_t* b, size_t n, hipStream_t st) override {
    return nccl_rc(rccl().AllReduce(b, b, n, ncclUint64, ncclSum, comm, st), "ncclAllReduce");
  }
  int all_gather(const int64_t* s, int64_t* r, size_t n, hipStream_t st) override {
    return nccl_rc(rccl().AllGather(s, r, n, ncclInt64, comm, st), "ncclAllGather");
  }
  int group_start() override { return nccl_rc(rccl().GroupStart(), "ncclGroupStart"); }
  int send(const void* b, size_t bytes, int peer, hipStream_t st) override {
    return nccl_rc(rccl().Send(b, bytes, ncclUint8, peer, comm, st), "ncclSend");
  }
  int recv(void* b, size_t bytes, int peer, hipStream_t st) override {
    return nccl_rc(rccl().Recv(b, bytes, ncclUint8, peer, comm, st), "ncclRecv");
  }
  int group_end() override { return nccl_rc(rccl().GroupEnd(), "ncclGroupEnd"); }

  template <typename Q>
  int poll(Q query, const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    const double lim = timeout_s();
    for (int i = 0;; i++) {
      const hipError_t q = query();
      if (q == hipSuccess) return SRS_OK;
      if (q != hipErrorNotReady) return hip_rc(q, what);
      if (group_fail && group_fail->load()) {
        abort("another rank of this process aborted");
        return set_error(SRS_ERR_HIP, "shard: another rank of this process aborted the exchange");
      }
      if ((i & 63) == 0) {
        ncclResult_t ae = ncclSuccess;
        if (rccl().CommGetAsyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess &&
            ae != ncclInProgress) {
          abort("RCCL asynchronous error");
          return set_error(SRS_ERR_HIP, std::string("shard: RCCL asynchronous error: ") +
                                            rccl().GetErrorString(ae));
        }
        const double dt =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt > lim) {
          abort("timed out");
          return set_error(SRS_ERR_HIP, std::string("shard: ") + what + " timed out after " +
                                            std::to_string((int)lim) +
                                            " s (a peer failed or stopped; SRS_SHARD_TIMEOUT_S)");
        }
      }
      if (i < 20000) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  int wait(hipStream_t st) override {
    return poll([&] { return hipStreamQuery(st); }, "waiting for the exchange");
  }
  int wait_event(hipEvent_t e) override {
    return poll([&] { return hipEventQuery(e); }, "waiting for a round");
  }
  void abort(const std::string& w) override {
    if (aborted.exchange(true)) return;
    why = w;
    if (group_fail) group_fail->store(1);
    (void)rccl().CommAbort(comm);  // (ends this rank's queued RCCL work)
  }
  bool dead() const override { return aborted; }
};

// Host-staged transport: world ranks in one process (threads), any devices,
// every collective and message through host memory. Messages between a pair
// of ranks are matched in posting order (FIFO per pair), as RCCL's are.
struct StagedHub {
  explicit StagedHub(int w) : world(w), in(w), box((size_t)w * w) {}
  int world;
  std::mutex mu;
  std::condition_variable cv;
  bool aborted = false;
  std::string why;
  uint64_t gen = 0;  // completed collectives
  int arrived = 0;
  std::vector<std::vector<uint64_t>> in;
  std::vector<uint64_t> out;
  std::vector<std::deque<std::vector<char>>> box;  // [src * world + dst]
};

struct StagedTransport : Transport {
  std::shared_ptr<StagedHub> hub;
  int me = 0;
  struct Op {
    bool send;
    void* buf;
    size_t bytes;
    int peer;
    hipStream_t st;
  };
  std::vector<Op> ops;

  const char* name() const override { return "staged"; }

  int aborted_error() {
    return set_error(SRS_ERR_HIP, "shard: the exchange was aborted (" + hub->why + ")");
  }
  void abort_locked(const std::string& w) {
    if (!hub->aborted) hub->why = w;
    hub->aborted = true;
    hub->cv.notify_all();
  }
  std::chrono::duration<double> limit() const { return std::chrono::duration<double>(timeout_s()); }

  // op 0: element-wise sum; 1: concatenation in rank order
  int exchange(std::vector<uint64_t>& v, int op) {
    StagedHub& H = *hub;
    std::unique_lock<std::mutex> lk(H.mu);
    if (H.aborted) return aborted_error();
    H.in[me] = v;
    const uint64_t g = H.gen;
    if (++H.arrived == H.world) {
      if (op == 0) {
        H.out = H.in[0];
        for (int r = 1; r < H.world; r++) {
          if (H.in[r].size() != H.out.size()) {
            abort_locked("collective sizes differ");
            return aborted_error();
          }
          for (size_t i = 0; i < H.out.size(); i++) H.out[i] += H.in[r][i];
        }
      } else {
        H.out.clear();
        for (int r = 0; r < H.world; r++) H.out.insert(H.out.end(), H.in[r].begin(), H.in[r].end());
      }
      H.arrived = 0;
      H.gen++;
      H.cv.notify_all();
    } else if (!H.cv.wait_for(lk, limit(), [&] { return H.gen != g || H.aborted; })) {
      abort_locked("a collective timed out");
      return aborted_error();
    }
    if (H.gen == g) return aborted_error();
    v = H.out;
    return SRS_OK;
  }
  int all_reduce_sum(uint64_t* b, size_t n, hipStream_t st) override {
    std::vector<uint64_t> v(n);
    SH_HIP(hipMemcpyAsync(v.data(), b, n * 8, hipMemcpyDeviceToHost, st));
    SH_HIP(hipStreamSynchronize(st));
    const int rc = exchange(v, 0);
    if (rc != SRS_OK) return rc;
    SH_HIP(hipMemcpyAsync(b, v.data(), n * 8, hipMemcpyHostToDevice, st));
    SH_HIP(hipStreamSynchronize(st));
    return SRS_OK;
  }
  int all_gather(const int64_t* s, int64_t* r, size_t n, hipStream_t st) override {
    std::vector<uint64_t> v(n);
    SH_HIP(hipMemcpyAsync(v.data(), s, n * 8, hipMemcpyDeviceToHost, st));
    SH_HIP(hipStreamSynchronize(st));
    const int rc = exchange(v, 1);
    if (rc != SRS_OK) return rc;
    SH_HIP(hipMemcpyAsync(r, v.data(), v.size() * 8, hipMemcpyHostToDevice, st));
    SH_HIP(hipStreamSynchronize(st));
    return SRS_OK;
  }
  int group_start() override {
    ops.clear();
    return SRS_OK;
  }
  int send(const void* b, size_t bytes, int peer, hipStream_t st) override {
    ops.push_back(Op{true, const_cast<void*>(b), bytes, peer, st});
    return SRS_OK;
  }
  int recv(void* b, size_t bytes, int peer, hipStream_t st) override {
    ops.push_back(Op{false, b, bytes, peer, st});
    return SRS_OK;
  }
  // every send of the group is deposited before any receive waits, so the
  // ranks' groups cannot wait on each other in a cycle
  int group_end() override {
    StagedHub& H = *hub;
    const int w = H.world;
    for (const Op& o : ops) {
      if (!o.send) continue;
      std::vector<char> m(o.bytes);
      SH_HIP(hipMemcpyAsync(m.data(), o.buf, o.bytes, hipMemcpyDeviceToHost, o.st));
      SH_HIP(hipStreamSynchronize(o.st));
      std::lock_guard<std::mutex> lk(H.mu);
      if (H.aborted) return aborted_error();
      H.box[(size_t)me * w + o.peer].push_back(std::move(m));
      H.cv.notify_all();
    }
    for (const Op& o : ops) {
      if (o.send) continue;
      std::vector<char> m;
      {
        std::unique_lock<std::mutex> lk(H.mu);
        auto& q = H.box[(size_t)o.peer * w + me];
        if (!H.cv.wait_for(lk, limit(), [&] { return !q.empty() || H.aborted; })) {
          abort_locked("a receive timed out");
          return aborted_error();
        }
        if (q.empty()) return aborted_error();
        m = std::move(q.front());
        q.pop_front();
        if (m.size() != o.bytes) {
          abort_locked("message sizes differ");
          return set_error(SRS_ERR_INTERNAL, "shard: a message's size differs between its sender "
                                             "and its receiver");
        }
      }
      SH_HIP(hipMemcpyAsync(o.buf, m.data(), o.bytes, hipMemcpyHostToDevice, o.st));
      SH_HIP(hipStreamSynchronize(o.st));
    }
    ops.clear();
    return SRS_OK;
  }
  int wait(hipStream_t st) override {
    SH_HIP(hipStreamSynchronize(st));
    return SRS_OK;
  }
  int wait_event(hipEvent_t e) override {
    SH_HIP(hipEventSynchronize(e));
    return SRS_OK;
  }
  void abort(const std::string& w) override {
    std::lock_guard<std::mutex> lk(hub->mu);
    abort_locked(w);
  }
  bool dead() const override {
    std::lock_guard<std::mutex> lk(hub->mu);
    return hub->aborted;
  }
};

// ---------------------------------------------------------------------------
// the plan (host only; the same on every rank up to `me`)
// ---------------------------------------------------------------------------
// bins -> parts: part of bin b = floor(parts * (keys before b + half of b) /
// total), non-decreasing
std::vector<int32_t> balanced_split(const uint64_t* h, int nbins, int parts) {
  std::vector<int32_t> out(nbins, 0);
  double total = 0;
  for (int b = 0; b < nbins; b++) total += (double)h[b];
  if (total <= 0) return out;
  double before = 0;
  int prev = 0;
  for (int b = 0; b < nbins; b++) {
    int p = (int)std::floor((before + 0.5 * (double)h[b]) * parts / total);
    p = std::min(std::max(p, prev), parts - 1);
    out[b] = prev = p;
    before += (double)h[b];
  }
  return out;
}

// Input chunk c of n records (of CH) starts at chunk_bound(n, c, CH): the
// first chunk weighs 1, every other 4, so the first partition (which every
// message waits for) is short. Rounds follow the same idea at the other end:
// the last round weighs 1, the others 4, so the last round's sort (which
// nothing overlaps) is short (head and tail).
int64_t weighted_bound(int64_t m, int i, int parts, bool first_small) {
  if (i <= 0) return 0;
  if (i >= parts) return m;
  const int64_t tot = 4 * (int64_t)parts - 3;
  const int64_t w = first_small ? 4 * (int64_t)i - 3 : 4 * (int64_t)i;
  return (int64_t)((__int128)m * w / tot);
}
int64_t chunk_bound(int64_t n, int c, int CH) { return weighted_bound(n, c, CH, true); }

// The posting schedule: message group k carries the pieces (round r, chunk
// c) with r + c == k ("wavefront"). Group k < CH goes out right after chunk
// k is partitioned and already carries later rounds of the earlier chunks,
// so the links have work during the whole partition (posting only round 0
// per chunk left them ~80 % idle then at 8 ranks); round r is complete after
// group CH - 1 + r. Every rank posts the same groups in the same order.
std::vector<std::vector<std::pair<int, int>>> post_schedule(int CH, int R) {
  std::vector<std::vector<std::pair<int, int>>> g(CH + R - 1);
  for (int k = 0; k < CH + R - 1; k++)
    for (int c = 0; c < CH; c++) {
      const int r = k - c;
      if (r >= 0 && r < R) g[k].push_back({r, c});
    }
  return g;
}

struct Msg {
  int op;        // 0 send, 1 receive, 2 own piece (a device copy)
  int peer;
  int64_t src;   // record offset in the partitioned buffer (send, copy)
  int64_t dst;   // record offset in the receive buffer (receive, copy)
  int64_t cnt;
};

struct ShardPlan {
  int w = 1, me = 0, CH = 1, G = 1, R = 1, bits = kBits, kbits = 64, nb = kHistBins;
  std::vector<int32_t> gob, rog;          // bin -> group, group -> rank
  std::vector<int> gfirst, glast;         // each group's first / last bin (-1: none)
  std::vector<std::vector<int>> owned;    // rank -> its groups
  std::vector<int64_t> mat;               // [src][chunk][group] records
  std::vector<int64_t> cb;                // this rank's chunk bounds
  std::vector<int64_t> roff;              // [round][src][chunk] receive offsets
  std::vector<int64_t> rb0, rb1;          // each round's receive range
  std::vector<int64_t> soff;              // [chunk][group + 1] partitioned offsets
  int64_t total = 0;
  bool alias = false;                     // one rank, one chunk: receive = partition buffer
  bool self = false;                      // own pieces as messages to this rank (not copies)

  void init(int world, int rank, int chunks, int rounds, int key_bits, bool self_msgs = false) {
    w = world;
    me = rank;
    CH = chunks;
    R = rounds;
    kbits = key_bits;
    bits = std::min(kBits, kbits);
    nb = 1 << bits;
    G = std::min(kGroups, nb);
    self = self_msgs;
    alias = w == 1 && CH == 1 && !self;
  }
  void split(const uint64_t* tot) {
    gob = balanced_split(tot, nb, G);
    std::vector<uint64_t> gtot(G, 0);
    for (int b = 0; b < nb; b++) gtot[gob[b]] += tot[b];
    rog = balanced_split(gtot.data(), G, w);
    gfirst.assign(G, -1);
    glast.assign(G, -1);
    for (int b = 0; b < nb; b++) {
      if (gfirst[gob[b]] < 0) gfirst[gob[b]] = b;
      glast[gob[b]] = b;
    }
    owned.assign(w, {});
    for (int g = 0; g < G; g++) owned[rog[g]].push_back(g);
  }
  // this rank's group sizes per chunk from its chunk histograms [CH][nb]
  std::vector<int64_t> chunk_groups(const uint64_t* hc) const {
    std::vector<int64_t> cc((size_t)CH * G, 0);
    for (int c = 0; c < CH; c++)
      for (int b = 0; b < nb; b++) cc[(size_t)c * G + gob[b]] += (int64_t)hc[(size_t)c * nb + b];
    return cc;
  }
  int64_t M(int src, int c, int g) const { return mat[((size_t)src * CH + c) * G + g]; }
  // round r of rank d: groups owned[d][lo, hi)
  void rgrp(int d, int r, int* lo, int* hi) const {
    const int64_t m = (int64_t)owned[d].size();
    *lo = (int)weighted_bound(m, r, R, false);
    *hi = (int)weighted_bound(m, r + 1, R, false);
  }
  // (first group, records) of the round-r piece source `src` holds for rank
  // d in chunk c: a contiguous run of groups, so one range of its buffer
  int64_t piece(int src, int c, int d, int r, int* g0) const {
    int lo, hi;
    rgrp(d, r, &lo, &hi);
    *g0 = lo < hi ? owned[d][lo] : 0;
    int64_t cnt = 0;
    for (int i = lo; i < hi; i++) cnt += M(src, c, owned[d][i]);
    return cnt;
  }
  void layout(const int64_t* all, int64_t n) {
    mat.assign(all, all + (size_t)w * CH * G);
    cb.resize(CH + 1);
    for (int c = 0; c <= CH; c++) cb[c] = chunk_bound(n, c, CH);
    // receive layout: round-major, then source, then chunk
    roff.assign((size_t)R * w * CH, 0);
    rb0.assign(R, 0);
    rb1.assign(R, 0);
    int64_t pos = 0;
    for (int r = 0; r < R; r++) {
      rb0[r] = pos;
      for (int src = 0; src < w; src++)
        for (int c = 0; c < CH; c++) {
          int g0;
          roff[((size_t)r * w + src) * CH + c] = pos;
          pos += piece(src, c, me, r, &g0);
        }
      rb1[r] = pos;
    }
    total = pos;
    soff.assign((size_t)CH * (G + 1), 0);
    for (int c = 0; c < CH; c++) {
      soff[(size_t)c * (G + 1)] = cb[c];
      for (int g = 0; g < G; g++)
        soff[(size_t)c * (G + 1) + g + 1] = soff[(size_t)c * (G + 1) + g] + M(me, c, g);
    }
  }
  // the messages of (round r, chunk c), in posting order: per peer, the
  // send then the receive; this rank's own piece last (a device copy), or,
  // with self messages, a send and a receive to itself in rank order
  std::vector<Msg> messages(int r, int c) const {
    std::vector<Msg> out;
    for (int d = 0; d < w; d++) {
      int gs;
      if (d == me && !self) continue;
      const int64_t scnt = piece(me, c, d, r, &gs);
      if (scnt) out.push_back(Msg{0, d, soff[(size_t)c * (G + 1) + gs], 0, scnt});
      const int64_t rcnt = piece(d, c, me, r, &gs);
      if (rcnt) out.push_back(Msg{1, d, 0, roff[((size_t)r * w + d) * CH + c], rcnt});
    }
    if (!alias && !self) {
      int gs;
      const int64_t cnt = piece(me, c, me, r, &gs);
      if (cnt)
        out.push_back(Msg{2, me, soff[(size_t)c * (G + 1) + gs], roff[((size_t)r * w + me) * CH + c],
                          cnt});
    }
    return out;
  }
  // top key bits every key of groups owned[me][ga, gb) shares
  int shared_bits(int ga, int gb) const {
    int b0 = -1, b1 = -1;
    for (int g = ga; g < gb; g++) {
      const int q = owned[me][g];
      if (gfirst[q] < 0) continue;
      if (b0 < 0) b0 = gfirst[q];
      b1 = glast[q];
    }
    if (b0 < 0) return 0;
    int diff = b0 ^ b1, l = 0;
    while (diff) {
      l++;
      diff >>= 1;
    }
    return std::min(bits - l, kbits - 1);
  }
  // the segments (relative to rb0[r]) round r is sorted as, and their known bits
  void round_segments(int r, std::vector<int64_t>* bounds, int* known) const {
    int lo, hi;
    rgrp(me, r, &lo, &hi);
    bounds->clear();
    if (alias) {  // one source: every group lies contiguous, its own segment
      bounds->push_back(0);
      *known = kbits;
      for (int i = lo; i < hi; i++) {
        bounds->push_back(bounds->back() + M(me, 0, owned[me][i]));
        *known = std::min(*known, shared_bits(i, i + 1));
      }
      if (*known >= kbits) *known = 0;
    } else {  // several sources or chunks interleave the groups: one segment
      bounds->push_back(0);
      bounds->push_back(rb1[r] - rb0[r]);
      *known = shared_bits(lo, hi);
    }
  }
  // records this rank sends each peer in round r (itself too with self
  // messages)
  std::vector<int64_t> sent(int r) const {
    std::vector<int64_t> s(w, 0);
    for (int d = 0; d < w; d++) {
      if (d == me && !self) continue;
      for (int c = 0; c < CH; c++) {
        int gs;
        s[d] += piece(me, c, d, r, &gs);
      }
    }
    return s;
  }
};

// A device buffer from srs_alloc_device, grown on demand.
struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t want) {
    if (bytes >= want && p) return SRS_OK;
    if (p) srs_free_device(p);
    p = nullptr;
    bytes = 0;
    const int rc = srs_alloc_device(std::max<size_t>(want, 256), &p);
    if (rc != SRS_OK) return rc;
    bytes = std::max<size_t>(want, 256);
    return SRS_OK;
  }
  void release() {
    if (p) srs_free_device(p);
    p = nullptr;
    bytes = 0;
  }
};

// Timing events of one sort's phases (read after the sort has completed).
struct PhaseClock {
  std::vector<hipEvent_t> ev;
  std::vector<std::string> names;
  size_t used = 0;
  void reset() {
    used = 0;
    names.clear();
  }
  // records a stamp on st; the event (for stream waits) or nullptr
  hipEvent_t stamp(const std::string& name, hipStream_t st) {
    if (used == ev.size()) {
      hipEvent_t e = nullptr;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      ev.push_back(e);
    }
    hipEvent_t e = ev[used];
    if (hipEventRecord(e, st) != hipSuccess) return nullptr;
    used++;
    names.push_back(name);
    return e;
  }
  void destroy() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    ev.clear();
    reset();
  }
};

}  // namespace
}  // namespace srs

using namespace srs;

struct srs_shard_comm_s {
  std::unique_ptr<Transport> tr;
  int world = 1, rank = 0, device = 0;
  int rounds = 0, chunks = 0;  // 0: the defaults
  int self_msgs = 0;           // srs_shard_set_message_options: own pieces as self messages
  int64_t msg_cap = 0;         // largest message in bytes (0: kMsgBytes)
  int inject = 0;              // srs_shard_debug_inject (one sort)
  hipStream_t cs = nullptr;    // communication stream
  hipStream_t ss = nullptr;    // round sorts
  hipStream_t own = nullptr;   // the stream srs_shard_sort_multi drives the rank on
  hipEvent_t ev_a = nullptr, ev_b = nullptr;  // stream joins
  PhaseClock clk;
  Buf hdr, hist, stage, flag, lut, part[1 + SRS_MAX_PAYLOADS], recv[1 + SRS_MAX_PAYLOADS];
  // the last sort, for srs_shard_last_report
  int last_chunks = 0, last_rounds = 0, last_groups = 0, last_rec_bytes = 0, last_ok = 0;
  int64_t last_in = 0, last_out = 0;
  int last_self = 0;
  int64_t last_cap = 0, last_sends = 0, last_recvs = 0;  // message cap, transport calls posted
  int64_t last_deferred = 0;  // workspace frees held back during the exchange
  std::vector<std::vector<int64_t>> last_sent;  // [round][peer] records
  std::mutex mu;
};

namespace {

int make_comm_state(srs_shard_comm c) {
  SH_HIP(hipSetDevice(c->device));
  SH_HIP(hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking));
  SH_HIP(hipStreamCreateWithFlags(&c->ss, hipStreamNonBlocking));
  SH_HIP(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
  SH_HIP(hipEventCreateWithFlags(&c->ev_a, hipEventDisableTiming));
  SH_HIP(hipEventCreateWithFlags(&c->ev_b, hipEventDisableTiming));
  // everything the steps before the first message need, so that no rank can
  // fail there alone (the header collective is the first thing every rank does)
  int rc = c->hdr.ensure((size_t)(kHistBins + kHdr) * 8);
  if (rc == SRS_OK) rc = c->hist.ensure((size_t)kMaxChunks * kHistBins * 8);
  if (rc == SRS_OK) rc = c->stage.ensure((size_t)(c->world + 1) * kMaxChunks * kGroups * 8);
  if (rc == SRS_OK) rc = c->flag.ensure(64);
  return rc;
}

#define SH_ABORT(expr)                                     \
  do {                                                     \
    const int r_ = (expr);                                 \
    if (r_ != SRS_OK) {                                    \
      const std::string m_ = srs_last_error();             \
      T.abort(m_);                                         \
      return set_error(r_, m_);                            \
    }                                                      \
  } while (0)

// One rank's part of the shard sort (the protocol above), on stream st.
// arg_err: this rank's arguments are invalid (it still takes part in the
// header collective, which fails every rank).
int shard_sort(srs_shard_comm C, int64_t n, int kind, int up, const void* keys, int32_t np,
               const void* const* pays, const uint32_t* psz, void** keys_out, void** pays_out,
               int64_t* num_out, hipStream_t st, int arg_err, const std::string& arg_msg) {
  Transport& T = *C->tr;
  const int w = C->world, me = C->rank;
  const int inject = C->inject;
  C->inject = 0;
  C->last_ok = 0;
  if (T.dead())
    return set_error(SRS_ERR_HIP, "shard: this communicator was aborted by an earlier failure; "
                                  "create a new one");
  int err = arg_err;
  std::string emsg = arg_msg;
  if (inject == 1 && !err) {
    err = SRS_ERR_INVALID_ARG;
    emsg = "shard: injected argument error (srs_shard_debug_inject 1)";
  }
  auto note = [&](int rc) {
    if (rc != SRS_OK && !err) {
      err = rc;
      emsg = srs_last_error();
    }
  };
  if (err) np = 0;
  const int ks = err ? 8 : key_bytes(kind);
  const int kbits = 8 * ks;
  const int CH = C->chunks > 0 ? C->chunks : (w > 1 ? kDefaultChunks : 1);
  const int R = C->rounds > 0 ? C->rounds : (w > 1 ? kDefaultRounds : kDefaultRounds1);
  const bool selfm = C->self_msgs != 0;
  const size_t cap = C->msg_cap > 0 ? (size_t)C->msg_cap : kMsgBytes;
  const int ncols = 1 + np;
  std::vector<uint32_t> width(ncols);
  width[0] = (uint32_t)ks;
  for (int c = 0; c < np; c++) width[1 + c] = psz[c];
  ShardPlan P;
  P.init(w, me, CH, R, kbits, selfm);
  const int nb = P.nb, G = P.G;
  if (err) n = 0;
  std::vector<int64_t> cb(CH + 1);
  for (int c = 0; c <= CH; c++) cb[c] = chunk_bound(n, c, CH);
  C->clk.reset();
  C->clk.stamp("start", st);

  // 1. chunk histograms; their sum and the header in one all-reduce
  uint64_t* dh = (uint64_t*)C->hist.p;
  std::vector<uint64_t> hc((size_t)CH * nb, 0);
  if (!err) note(hip_rc(hipMemsetAsync(dh, 0, (size_t)CH * nb * 8, st), "hipMemsetAsync"));
  for (int c = 0; c < CH && !err; c++)
    if (cb[c + 1] > cb[c])
      note(srs_key_histogram_device(cb[c + 1] - cb[c], kind, up,
                                    (const char*)keys + (size_t)cb[c] * ks, P.bits,
                                    dh + (size_t)c * nb, st));
  if (!err) note(hip_rc(hipMemcpyAsync(hc.data(), dh, hc.size() * 8, hipMemcpyDeviceToHost, st),
                        "hipMemcpyAsync"));
  if (!err) note(hip_rc(hipStreamSynchronize(st), "hipStreamSynchronize"));  // (local work only)
  std::vector<uint64_t> H((size_t)kHistBins + kHdr, 0);
  if (!err)
    for (int c = 0; c < CH; c++)
      for (int b = 0; b < nb; b++) H[b] += hc[(size_t)c * nb + b];
  uint64_t sig = 0;
  for (int k = 0; k < np; k++) sig = (sig * 131 + psz[k]) % 1000003;
  uint64_t* hs = H.data() + kHistBins;
  auto put = [&](int i, uint64_t v) {
    hs[i] = v;
    hs[i + 1] = v * v;
  };
  hs[0] = err ? 1 : 0;
  put(1, err ? 0 : (uint64_t)kind);
  put(3, up ? 1 : 0);
  put(5, (uint64_t)np);
  put(7, sig);
  put(9, (uint64_t)CH);
  put(11, (uint64_t)R);
  hs[13] = 1;
  hs[14] = err ? 1ull << std::min(me, 63) : 0;  // (names the ranks; hs[0] counts them)
  put(15, (uint64_t)(cap / 64));
  C->clk.stamp("hist", st);
  uint64_t* dH = (uint64_t*)C->hdr.p;
  // (every read-back of a collective's result waits for the collective with
  // the transport's bounded wait first: a device-to-host copy into pageable
  // memory would block the host inside the copy, unbounded, on a peer that
  // never joins)
  auto read_back = [&](void* host, const void* dev, size_t bytes) -> int {
    int rc = T.wait(st);
    if (rc == SRS_OK) rc = hip_rc(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, st), "read-back");
    if (rc == SRS_OK) rc = hip_rc(hipStreamSynchronize(st), "read-back");  // (local work only)
    return rc;
  };
  SH_ABORT(hip_rc(hipMemcpyAsync(dH, H.data(), H.size() * 8, hipMemcpyHostToDevice, st), "header"));
  SH_ABORT(T.all_reduce_sum(dH, H.size(), st));
  SH_ABORT(read_back(H.data(), dH, H.size() * 8));
  if (hs[0]) {
    if (err) return set_error(err, emsg);
    return set_error(SRS_ERR_INVALID_ARG, "shard: rank(s) " + rank_list(hs[14]) +
                                              " failed before the exchange (see their errors)");
  }
  if (hs[13] != (uint64_t)w) return set_error(SRS_ERR_INTERNAL, "shard: world size mismatch");
  static const char* what[] = {"key kind", "direction", "payload count", "payload sizes",
                               "chunks (srs_shard_set_options)", "rounds (srs_shard_set_options)",
                               "message cap (srs_shard_set_message_options)"};
  static const int slot[] = {1, 3, 5, 7, 9, 11, 15};  // (13: the world count, 14: failing ranks)
  for (int i = 0; i < 7; i++) {
    const uint64_t s = hs[slot[i]], q = hs[slot[i] + 1];
    if ((uint64_t)w * q != s * s)
      return set_error(SRS_ERR_INVALID_ARG, std::string("shard: the ranks disagree on the ") +
                                                what[i] + "; every rank must pass the same");
  }

  // 2. the plan; every rank's group sizes per chunk
  P.split(H.data());
  const std::vector<int64_t> cc = P.chunk_groups(hc.data());
  int64_t* dcc = (int64_t*)C->stage.p;
  std::vector<int64_t> mat((size_t)w * CH * G);
  SH_ABORT(hip_rc(hipMemcpyAsync(dcc, cc.data(), cc.size() * 8, hipMemcpyHostToDevice, st), "sizes"));
  SH_ABORT(T.all_gather(dcc, dcc + cc.size(), cc.size(), st));
  SH_ABORT(read_back(mat.data(), dcc + cc.size(), mat.size() * 8));
  P.layout(mat.data(), n);

  // 3. every buffer before the first message; one status for all ranks
  for (int c = 0; c < ncols && !err; c++) {
    note(C->part[c].ensure((size_t)std::max<int64_t>(n, 1) * width[c]));
    if (!P.alias && !err) note(C->recv[c].ensure((size_t)std::max<int64_t>(P.total, 1) * width[c]));
  }
  if (!err) note(C->lut.ensure((size_t)nb * 4));
  int64_t biggest = 0;
  for (int r = 0; r < R; r++) biggest = std::max(biggest, P.rb1[r] - P.rb0[r]);
  if (!err && biggest > 1) note(reserve_segments_workspace(biggest, ncols, width.data()));
  if (inject == 2 && !err) {
    err = SRS_ERR_OUT_OF_MEMORY;
    emsg = "shard: injected allocation failure (srs_shard_debug_inject 2)";
  }
  if (!err) note(hip_rc(hipMemcpyAsync(C->lut.p, P.gob.data(), (size_t)nb * 4,
                                       hipMemcpyHostToDevice, st), "hipMemcpyAsync"));
  // status: {failing ranks, their bits} (the count decides: a sum of bits
  // could wrap beyond 64 ranks; the bits only name the ranks)
  uint64_t* dflag = (uint64_t*)C->flag.p;
  uint64_t stat[2] = {err ? 1ull : 0ull, err ? 1ull << std::min(me, 63) : 0ull};
  SH_ABORT(hip_rc(hipMemcpyAsync(dflag, stat, 16, hipMemcpyHostToDevice, st), "status"));
  SH_ABORT(T.all_reduce_sum(dflag, 2, st));
  SH_ABORT(read_back(stat, dflag, 16));
  if (stat[0]) {
    if (err) return set_error(err, emsg);
    return set_error(SRS_ERR_OUT_OF_MEMORY, "shard: rank(s) " + rank_list(stat[1]) +
                                                " could not allocate before the exchange");
  }
  C->clk.stamp("plan", st);
  auto rcol = [&](int c) { return (char*)(P.alias ? C->part[c].p : C->recv[c].p); };

  // one message group of the schedule, (round, chunk) pieces in order, on
  // the communication stream
  const auto sched = post_schedule(CH, R);
  int64_t nsend = 0, nrecv = 0;
  auto issue = [&](const std::vector<std::pair<int, int>>& pieces) -> int {
    int rc = T.group_start();
    for (size_t q = 0; q < pieces.size() && rc == SRS_OK; q++)
      for (const Msg& m : P.messages(pieces[q].first, pieces[q].second)) {
        if (m.op == 2) continue;
        for (int k = 0; k < ncols && rc == SRS_OK; k++) {
          const size_t wd = width[k];
          const int64_t per = (int64_t)std::max<size_t>(1, cap / wd);
          for (int64_t a = 0; a < m.cnt && rc == SRS_OK; a += per) {
            const size_t bytes = (size_t)std::min(per, m.cnt - a) * wd;
            if (m.op == 0) {
              rc = T.send((const char*)C->part[k].p + (size_t)(m.src + a) * wd, bytes, m.peer, C->cs);
              nsend++;
            } else {
              rc = T.recv(rcol(k) + (size_t)(m.dst + a) * wd, bytes, m.peer, C->cs);
              nrecv++;
            }
          }
        }
      }
    const int re = T.group_end();
    if (rc == SRS_OK) rc = re;
    for (size_t q = 0; q < pieces.size() && rc == SRS_OK; q++)
      for (const Msg& m : P.messages(pieces[q].first, pieces[q].second))
        for (int k = 0; k < ncols && m.op == 2 && rc == SRS_OK; k++) {
          const size_t wd = width[k];
          rc = hip_rc(hipMemcpyAsync(rcol(k) + (size_t)m.dst * wd,
                                     (const char*)C->part[k].p + (size_t)m.src * wd,
                                     (size_t)m.cnt * wd, hipMemcpyDeviceToDevice, C->cs),
                      "own piece");
        }
    return rc;
  };

  // 4. partition chunk by chunk; after chunk c, message group c leaves.
  // A failure from here on is "late": the rank keeps to the message plan.
  // Until the last status, a workspace buffer that must grow frees its old
  // memory later (a hipFree now would wait for every receive
  // already queued, unbounded, and serialise the rounds behind the exchange)
  struct DeferScope {
    int64_t* freed;
    explicit DeferScope(int64_t* f) : freed(f) { defer_workspace_frees(true); }
    ~DeferScope() {
      defer_workspace_frees(false);
      *freed = release_deferred_frees();
    }
  } defer_scope(&C->last_deferred);
  int late = 0;
  std::string lmsg;
  auto late_fail = [&](int rc) {
    if (rc != SRS_OK && !late) {
      late = rc;
      lmsg = srs_last_error();
    }
  };
  std::vector<const void*> pin(np);
  std::vector<void*> pout(np);
  std::vector<hipEvent_t> arrived(R, nullptr);
  for (int c = 0; c < CH; c++) {
    const int64_t a = cb[c], m = cb[c + 1] - cb[c];
    if (m > 0 && !late) {
      for (int k = 0; k < np; k++) {
        pin[k] = (const char*)pays[k] + (size_t)a * width[1 + k];
        pout[k] = (char*)C->part[1 + k].p + (size_t)a * width[1 + k];
      }
      std::vector<int64_t> got(G, 0);
      const int rc =
          inject == 3 && c == std::min(1, CH - 1)
              ? set_error(SRS_ERR_HIP, "shard: injected partition failure (srs_shard_debug_inject 3)")
              : srs_partition_device(m, kind, up, (const char*)keys + (size_t)a * ks, np, pin.data(),
                                     psz, P.bits, (const int32_t*)C->lut.p, G,
                                     (char*)C->part[0].p + (size_t)a * ks, pout.data(), got.data(),
                                     st);
      late_fail(rc);
      if (rc == SRS_OK)
        for (int g = 0; g < G; g++)
          if (got[g] != P.M(me, c, g)) {
            late_fail(set_error(SRS_ERR_INTERNAL,
                                "shard: partition sizes differ from the histogram plan"));
            break;
          }
    }
    hipEvent_t e = C->clk.stamp("partition" + std::to_string(c), st);
    if (!e) SH_ABORT(set_error(SRS_ERR_HIP, "shard: event record failed"));
    SH_ABORT(hip_rc(hipStreamWaitEvent(C->cs, e, 0), "hipStreamWaitEvent"));
    SH_ABORT(issue(sched[c]));
    if (c == CH - 1) {
      arrived[0] = C->clk.stamp("round0_recv", C->cs);
      if (!arrived[0]) SH_ABORT(set_error(SRS_ERR_HIP, "shard: event record failed"));
    }
  }
  if (inject == 5) {
    T.abort("injected transport failure");
    return set_error(SRS_ERR_HIP, "shard: injected transport failure (srs_shard_debug_inject 5)");
  }
  // 5. the rest of the schedule posted now (group CH - 1 + r completes round
  // r): the links stay busy while the rounds sort
  for (int r = 1; r < R; r++) {
    SH_ABORT(issue(sched[CH - 1 + r]));
    arrived[r] = C->clk.stamp("round" + std::to_string(r) + "_recv", C->cs);
    if (!arrived[r]) SH_ABORT(set_error(SRS_ERR_HIP, "shard: event record failed"));
  }
  std::vector<int64_t> bounds;
  for (int r = 0; r < R; r++) {
    SH_ABORT(hip_rc(hipStreamWaitEvent(C->ss, arrived[r], 0), "hipStreamWaitEvent"));
    C->clk.stamp("round" + std::to_string(r) + "_sort_start", C->ss);
    const int64_t len = P.rb1[r] - P.rb0[r];
    if (!late && len >= 2) {
      // (bounded: the sort's own read-backs would otherwise wait on the
      // round's receives without a limit)
      SH_ABORT(T.wait_event(arrived[r]));
      int known = 0;
      P.round_segments(r, &bounds, &known);
      std::vector<void*> cols(ncols);
      for (int k = 0; k < ncols; k++) cols[k] = rcol(k) + (size_t)P.rb0[r] * width[k];
      late_fail(inject == 4 && r == R - 1
                    ? set_error(SRS_ERR_HIP,
                                "shard: injected round-sort failure (srs_shard_debug_inject 4)")
                    : srs_sort_segments_device(len, kind, up, cols[0], np,
                                               np ? cols.data() + 1 : nullptr, psz,
                                               (int64_t)bounds.size() - 1, bounds.data(), known,
                                               C->ss));
    }
    C->clk.stamp("round" + std::to_string(r) + "_sort_end", C->ss);
  }
  SH_ABORT(hip_rc(hipEventRecord(C->ev_a, C->ss), "hipEventRecord"));
  SH_ABORT(hip_rc(hipStreamWaitEvent(st, C->ev_a, 0), "hipStreamWaitEvent"));
  SH_ABORT(hip_rc(hipEventRecord(C->ev_b, C->cs), "hipEventRecord"));
  SH_ABORT(hip_rc(hipStreamWaitEvent(st, C->ev_b, 0), "hipStreamWaitEvent"));
  C->clk.stamp("end", st);

  // 6. every rank learns whether any rank failed after the first message
  stat[0] = late ? 1ull : 0ull;
  stat[1] = late ? 1ull << std::min(me, 63) : 0ull;
  SH_ABORT(hip_rc(hipMemcpyAsync(dflag, stat, 16, hipMemcpyHostToDevice, st), "status"));
  SH_ABORT(T.all_reduce_sum(dflag, 2, st));
  SH_ABORT(read_back(stat, dflag, 16));
  if (stat[0]) {
    if (late) return set_error(late, lmsg);
    return set_error(SRS_ERR_INTERNAL, "shard: rank(s) " + rank_list(stat[1]) +
                                           " failed during the exchange (see their errors)");
  }
  *keys_out = rcol(0);
  for (int k = 0; k < np; k++) pays_out[k] = rcol(1 + k);
  *num_out = P.total;
  C->last_chunks = CH;
  C->last_rounds = R;
  C->last_groups = G;
  C->last_in = n;
  C->last_out = P.total;
  C->last_rec_bytes = 0;
  for (int k = 0; k < ncols; k++) C->last_rec_bytes += (int)width[k];
  C->last_self = selfm ? 1 : 0;
  C->last_cap = (int64_t)cap;
  C->last_sends = nsend;
  C->last_recvs = nrecv;
  C->last_sent.clear();
  for (int r = 0; r < R; r++) C->last_sent.push_back(P.sent(r));
  C->last_ok = 1;
  return SRS_OK;
}

int argument_error(int64_t num, int key_kind, int32_t np, const void* keys,
                   const void* const* payloads, const uint32_t* psz, void** keys_out,
                   void** payloads_out, int64_t* num_out, std::string* msg) {
  if (!keys_out || !num_out || num < 0 || (num > 0 && !keys) || key_bytes(key_kind) == 0 ||
      np < 0 || np > SRS_MAX_PAYLOADS || (np > 0 && (!payloads || !psz || !payloads_out))) {
    *msg = "srs_shard_sort_device: arguments";
    return SRS_ERR_INVALID_ARG;
  }
  for (int k = 0; k < np; k++) {
    const uint32_t s = psz[k];
    if (s != 1 && s != 2 && s != 4 && s != 8) {
      *msg = "srs_shard_sort_device: payload sizes must be 1, 2, 4 or 8 bytes";
      return SRS_ERR_UNSUPPORTED;
    }
  }
  return SRS_OK;
}

srs_shard_comm new_comm(int world, int rank, int device, std::unique_ptr<Transport> t) {
  auto* c = new srs_shard_comm_s();
  c->world = world;
  c->rank = rank;
  c->device = device;
  c->tr = std::move(t);
  return c;
}

}  // namespace

extern "C" {

int srs_shard_unique_id(void* id) {
  if (!id) return set_error(SRS_ERR_INVALID_ARG, "srs_shard_unique_id: id is NULL");
  const Rccl& R = rccl();
  if (!R.ok) return set_error(SRS_ERR_NO_DEVICE, R.why);
  ncclUniqueId u;
  const int rc = nccl_rc(R.GetUniqueId(&u), "ncclGetUniqueId");
  if (rc != SRS_OK) return rc;
  memcpy(id, &u, sizeof u);
  return SRS_OK;
}

int srs_shard_comm_init(int32_t world, int32_t rank, const void* id, srs_shard_comm* comm) {
  if (!comm || !id || world < 1 || rank < 0 || rank >= world)
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_comm_init: world, rank, id, comm");
  *comm = nullptr;
  const Rccl& R = rccl();
  if (!R.ok) return set_error(SRS_ERR_NO_DEVICE, R.why);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess)
    return set_error(SRS_ERR_NO_DEVICE, "srs_shard_comm_init: no current device");
  auto t = std::make_unique<RcclTransport>();
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  const int r = nccl_rc(R.CommInitRank(&t->comm, world, u, rank), "ncclCommInitRank");
  if (r != SRS_OK) return r;
  srs_shard_comm c = new_comm(world, rank, dev, std::move(t));
  const int rc = make_comm_state(c);
  if (rc != SRS_OK) {
    srs_shard_comm_destroy(c);
    return rc;
  }
  *comm = c;
  return SRS_OK;
}

int srs_shard_comm_init_all(int32_t num_devices, const int32_t* devices, srs_shard_comm* comms) {
  if (num_devices < 1 || !devices || !comms)
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_comm_init_all: devices and comms");
  const Rccl& R = rccl();
  if (!R.ok) return set_error(SRS_ERR_NO_DEVICE, R.why);
  std::vector<ncclComm_t> cm(num_devices);
  std::vector<int> dv(devices, devices + num_devices);
  const int r = nccl_rc(R.CommInitAll(cm.data(), num_devices, dv.data()), "ncclCommInitAll");
  if (r != SRS_OK) return r;
  int dev0 = 0;
  (void)hipGetDevice(&dev0);
  auto fail = std::make_shared<std::atomic<int>>(0);
  int rc = SRS_OK;
  for (int i = 0; i < num_devices; i++) {
    auto t = std::make_unique<RcclTransport>();
    t->comm = cm[i];
    t->group_fail = fail;
    comms[i] = new_comm(num_devices, i, dv[i], std::move(t));
    if (rc == SRS_OK) rc = make_comm_state(comms[i]);
  }
  (void)hipSetDevice(dev0);
  if (rc != SRS_OK)
    for (int i = 0; i < num_devices; i++) {
      srs_shard_comm_destroy(comms[i]);
      comms[i] = nullptr;
    }
  return rc;
}

int srs_shard_comm_init_staged(int32_t world, srs_shard_comm* comms) {
  if (world < 1 || world > 64 || !comms)
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_comm_init_staged: world in [1, 64], comms");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess)
    return set_error(SRS_ERR_NO_DEVICE, "srs_shard_comm_init_staged: no current device");
  auto hub = std::make_shared<StagedHub>(world);
  int rc = SRS_OK;
  for (int i = 0; i < world; i++) {
    auto t = std::make_unique<StagedTransport>();
    t->hub = hub;
    t->me = i;
    comms[i] = new_comm(world, i, dev, std::move(t));
    if (rc == SRS_OK) rc = make_comm_state(comms[i]);
  }
  (void)hipSetDevice(dev);
  if (rc != SRS_OK)
    for (int i = 0; i < world; i++) {
      srs_shard_comm_destroy(comms[i]);
      comms[i] = nullptr;
    }
  return rc;
}

int srs_shard_set_options(srs_shard_comm comm, int32_t rounds, int32_t chunks) {
  if (!comm || rounds < 0 || rounds > kMaxRounds || chunks < 0 || chunks > kMaxChunks)
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_set_options: rounds in [0, 64], chunks in "
                                          "[0, 16] (0 = default)");
  std::lock_guard<std::mutex> g(comm->mu);
  comm->rounds = rounds;
  comm->chunks = chunks;
  return SRS_OK;
}

int srs_shard_set_message_options(srs_shard_comm comm, int32_t self_messages,
                                  int64_t max_message_bytes) {
  if (!comm || self_messages < 0 || self_messages > 1 || max_message_bytes < 0 ||
      max_message_bytes > kMsgBytesMax || max_message_bytes % 64)
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_set_message_options: self_messages 0 or 1, "
                                          "max_message_bytes a multiple of 64 in [0, 2^30] "
                                          "(0 = 256 MiB)");
  std::lock_guard<std::mutex> g(comm->mu);
  comm->self_msgs = self_messages;
  comm->msg_cap = max_message_bytes;
  return SRS_OK;
}

int srs_shard_debug_inject(srs_shard_comm comm, int32_t point) {
  if (!comm || point < 0 || point > 5)
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_debug_inject: point in [0, 5]");
  std::lock_guard<std::mutex> g(comm->mu);
  comm->inject = point;
  return SRS_OK;
}

int srs_shard_comm_destroy(srs_shard_comm c) {
  if (!c) return SRS_OK;
  {
    std::lock_guard<std::mutex> g(c->mu);
    int dev0 = 0;
    (void)hipGetDevice(&dev0);
    (void)hipSetDevice(c->device);
    hipStream_t ss[] = {c->cs, c->ss, c->own};
    for (hipStream_t s : ss)
      if (s) (void)hipStreamSynchronize(s);
    Buf* bufs[] = {&c->hdr, &c->hist, &c->stage, &c->flag, &c->lut};
    for (Buf* b : bufs) b->release();
    for (auto& b : c->part) b.release();
    for (auto& b : c->recv) b.release();
    c->clk.destroy();
    if (c->ev_a) (void)hipEventDestroy(c->ev_a);
    if (c->ev_b) (void)hipEventDestroy(c->ev_b);
    for (hipStream_t s : ss)
      if (s) (void)hipStreamDestroy(s);
    c->tr.reset();
    (void)hipSetDevice(dev0);
    (void)hipGetLastError();
  }
  delete c;
  return SRS_OK;
}

int srs_shard_sort_device(srs_shard_comm comm, int64_t num, int key_kind, int up,
                          const void* keys, int32_t num_payloads, const void* const* payloads,
                          const uint32_t* payload_sizes, void** keys_out, void** payloads_out,
                          int64_t* num_out, void* stream) {
  if (!comm) return set_error(SRS_ERR_INVALID_ARG, "srs_shard_sort_device: comm is NULL");
  std::string msg;
  const int aerr = argument_error(num, key_kind, num_payloads, keys, payloads, payload_sizes,
                                  keys_out, payloads_out, num_out, &msg);
  std::lock_guard<std::mutex> g(comm->mu);
  int dev0 = 0;
  (void)hipGetDevice(&dev0);
  const int drc = hip_rc(hipSetDevice(comm->device), "hipSetDevice");
  if (drc != SRS_OK) return drc;
  const int rc = shard_sort(comm, num, key_kind, up, keys, num_payloads, payloads, payload_sizes,
                            keys_out, payloads_out, num_out, (hipStream_t)stream, aerr, msg);
  (void)hipSetDevice(dev0);
  return rc;
}

int srs_shard_sort_multi(int32_t num_devices, const srs_shard_comm* comms, const int64_t* nums,
                         int key_kind, int up, const void* const* keys, int32_t num_payloads,
                         const void* const* payloads, const uint32_t* payload_sizes,
                         void** keys_out, void** payloads_out, int64_t* nums_out) {
  if (num_devices < 1 || !comms || !nums || !keys || !keys_out || !nums_out ||
      (num_payloads > 0 && (!payloads || !payloads_out)))
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_sort_multi: arguments");
  for (int i = 0; i < num_devices; i++)
    if (!comms[i] || comms[i]->world != num_devices || comms[i]->rank != i)
      return set_error(SRS_ERR_INVALID_ARG, "srs_shard_sort_multi: comms must be ranks 0..N-1 of "
                                            "one communicator set");
  std::vector<int> rc(num_devices, SRS_OK);
  std::vector<std::string> err(num_devices);
  std::vector<std::thread> th;
  for (int i = 0; i < num_devices; i++)
    th.emplace_back([&, i] {
      srs_shard_comm c = comms[i];
      if (hipSetDevice(c->device) != hipSuccess) {
        rc[i] = SRS_ERR_HIP;
        err[i] = "hipSetDevice failed";
        c->tr->abort("hipSetDevice failed");  // (its peers must not wait for it)
        return;
      }
      rc[i] = srs_shard_sort_device(
          c, nums[i], key_kind, up, keys[i], num_payloads,
          num_payloads ? payloads + (size_t)i * num_payloads : nullptr, payload_sizes,
          keys_out + i, num_payloads ? payloads_out + (size_t)i * num_payloads : nullptr,
          nums_out + i, c->own);
      if (rc[i] == SRS_OK) rc[i] = hip_rc(hipStreamSynchronize(c->own), "hipStreamSynchronize");
      if (rc[i] != SRS_OK) err[i] = srs_last_error();
    });
  for (auto& t : th) t.join();
  // every failing rank's own message (a rank that only learnt of a peer's
  // failure from a status collective says so; the peer's message says why)
  int first = SRS_OK;
  std::string msg;
  for (int i = 0; i < num_devices; i++)
    if (rc[i] != SRS_OK) {
      if (first == SRS_OK) first = rc[i];
      msg += (msg.empty() ? "" : "; ") + ("rank " + std::to_string(i) + ": " + err[i]);
    }
  if (first != SRS_OK) return set_error(first, msg);
  return SRS_OK;
}

int srs_shard_last_report(srs_shard_comm comm, char* buf, int64_t cap) {
  if (!comm || !buf || cap < 2)
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_last_report: comm, buf, cap");
  std::lock_guard<std::mutex> g(comm->mu);
  if (!comm->last_ok) return set_error(SRS_ERR_INVALID_ARG, "srs_shard_last_report: no sort yet");
  std::string s = "{\"transport\":\"" + std::string(comm->tr->name()) + "\",\"world\":" +
                  std::to_string(comm->world) + ",\"rank\":" + std::to_string(comm->rank) +
                  ",\"chunks\":" + std::to_string(comm->last_chunks) +
                  ",\"rounds\":" + std::to_string(comm->last_rounds) +
                  ",\"groups\":" + std::to_string(comm->last_groups) +
                  ",\"records_in\":" + std::to_string(comm->last_in) +
                  ",\"records_out\":" + std::to_string(comm->last_out) +
                  ",\"record_bytes\":" + std::to_string(comm->last_rec_bytes) +
                  ",\"self_messages\":" + std::to_string(comm->last_self) +
                  ",\"max_message_bytes\":" + std::to_string(comm->last_cap) +
                  ",\"sends\":" + std::to_string(comm->last_sends) +
                  ",\"recvs\":" + std::to_string(comm->last_recvs) +
                  ",\"deferred_frees\":" + std::to_string(comm->last_deferred) + ",\"stamps_ms\":{";
  const PhaseClock& k = comm->clk;
  for (size_t i = 0; i < k.used; i++) {
    float ms = 0;
    const hipError_t e = hipEventElapsedTime(&ms, k.ev[0], k.ev[i]);
    if (e != hipSuccess) return hip_rc(e, "srs_shard_last_report (sort not complete?)");
    char num[64];
    snprintf(num, sizeof num, "%.4f", (double)ms);
    s += (i ? ",\"" : "\"") + k.names[i] + "\":" + num;
  }
  s += "},\"bytes_to_peer_per_round\":[";
  for (size_t r = 0; r < comm->last_sent.size(); r++) {
    s += r ? ",[" : "[";
    for (size_t d = 0; d < comm->last_sent[r].size(); d++)
      s += (d ? "," : "") + std::to_string(comm->last_sent[r][d] * comm->last_rec_bytes);
    s += "]";
  }
  s += "]}";
  if ((int64_t)s.size() + 1 > cap)
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_last_report: buffer too small (need " +
                                              std::to_string(s.size() + 1) + " bytes)");
  memcpy(buf, s.c_str(), s.size() + 1);
  return SRS_OK;
}

int srs_debug_shard_plan(int32_t world, int32_t rank, int32_t chunks, int32_t rounds,
                         int32_t key_bits, int32_t self_messages, const uint64_t* chunk_hists,
                         int64_t num, char* json, int64_t cap) {
  if (world < 1 || rank < 0 || rank >= world || chunks < 1 || chunks > kMaxChunks ||
      rounds < 1 || rounds > kMaxRounds || !chunk_hists || num < 0 || !json ||
      (self_messages != 0 && self_messages != 1) ||
      (key_bits != 8 && key_bits != 16 && key_bits != 32 && key_bits != 64))
    return set_error(SRS_ERR_INVALID_ARG, "srs_debug_shard_plan: arguments");
  ShardPlan P;
  P.init(world, rank, chunks, rounds, key_bits, self_messages != 0);
  const size_t per = (size_t)chunks * P.nb;
  std::vector<uint64_t> tot(P.nb, 0);
  for (int s = 0; s < world; s++)
    for (int c = 0; c < chunks; c++)
      for (int b = 0; b < P.nb; b++) tot[b] += chunk_hists[s * per + (size_t)c * P.nb + b];
  P.split(tot.data());
  std::vector<int64_t> mat;
  for (int s = 0; s < world; s++) {
    const std::vector<int64_t> cc = P.chunk_groups(chunk_hists + s * per);
    mat.insert(mat.end(), cc.begin(), cc.end());
  }
  P.layout(mat.data(), num);
  auto arr = [](const auto& v) {
    std::string s = "[";
    for (size_t i = 0; i < v.size(); i++) s += (i ? "," : "") + std::to_string(v[i]);
    return s + "]";
  };
  std::string s = "{\"bits\":" + std::to_string(P.bits) + ",\"groups\":" + std::to_string(P.G) +
                  ",\"group_of_bin\":" + arr(P.gob) + ",\"rank_of_group\":" + arr(P.rog) +
                  ",\"chunk_bounds\":" + arr(P.cb) + ",\"total\":" + std::to_string(P.total) +
                  ",\"alias\":" + (P.alias ? "true" : "false") + ",\"posts\":[";
  // the posting order of shard_sort (post_schedule)
  bool first = true;
  auto post = [&](const std::vector<std::pair<int, int>>& pieces) {
    s += first ? "{" : ",{";
    first = false;
    s += "\"pieces\":[";
    for (size_t q = 0; q < pieces.size(); q++)
      s += (q ? ",[" : "[") + std::to_string(pieces[q].first) + "," +
           std::to_string(pieces[q].second) + "]";
    s += "],\"msgs\":[";
    bool f2 = true;
    for (const auto& pc : pieces)
      for (const Msg& m : P.messages(pc.first, pc.second)) {
        s += f2 ? "[" : ",[";
        f2 = false;
        s += std::to_string(m.op) + "," + std::to_string(m.peer) + "," + std::to_string(m.src) +
             "," + std::to_string(m.dst) + "," + std::to_string(m.cnt) + "]";
      }
    s += "]}";
  };
  for (const auto& g : post_schedule(chunks, rounds)) post(g);
  s += "],\"rounds\":[";
  std::vector<int64_t> bounds;
  for (int r = 0; r < rounds; r++) {
    int known = 0;
    P.round_segments(r, &bounds, &known);
    s += (r ? ",{" : "{") + std::string("\"start\":") + std::to_string(P.rb0[r]) +
         ",\"end\":" + std::to_string(P.rb1[r]) + ",\"bounds\":" + arr(bounds) +
         ",\"known_bits\":" + std::to_string(known) + "}";
  }
  s += "]}";
  if ((int64_t)s.size() + 1 > cap)
    return set_error(SRS_ERR_INVALID_ARG, "srs_debug_shard_plan: buffer too small (need " +
                                              std::to_string(s.size() + 1) + " bytes)");
  memcpy(json, s.c_str(), s.size() + 1);
  return SRS_OK;
}

}  // extern "C"

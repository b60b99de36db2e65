// srs_shard.hip — the multi-GPU shard sort behind the C ABI (srs_shard_*),
// over RCCL (loaded at first use), for C/C++ callers: one array spread over
// N GPUs is sorted across them, rank r ending with the r-th key range.
//
// Protocol (the same one srs_amd/dist.py drives from Python):
//   1. per input chunk, a histogram of the transformed top 12 key bits
//      (srs_key_histogram_device); the sum is all-reduced (RCCL, 32 KB);
//   2. the 4096 bins -> 512 key-range groups of ~equal size, contiguous runs
//      of groups -> ranks (balanced_split, on the host, identical on every
//      rank since every rank sees the same histogram);
//   3. every rank's group sizes per chunk are all-gathered (exact: a group is
//      a union of bins), so every receive is sized before any data moves;
//   4. the input is partitioned chunk by chunk into the groups
//      (srs_partition_device: the sort's first radix level), each chunk's
//      first-round messages going out as soon as it is partitioned;
//   5. rounds of grouped send/recv (one message per (round, peer, chunk,
//      column), <= 256 MB each: RCCL returns messages above 1 GiB corrupted,
//      DESIGN.md §7) on a communication stream; round r's key range is
//      sorted on a side stream (srs_sort_segments_device) once it has
//      arrived, while the next rounds are in flight.
// Equal keys share a group; inside a round they arrive in (source rank,
// chunk, input index) order, so the whole sort is stable.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/srs_c_api.h"
#include "srs_kernels.h"

namespace srs {
int set_error(int code, const std::string& msg);  // (srs_api.hip)

namespace {

// ---- RCCL, resolved at first use (the library itself does not need it) ----
struct Rccl {
  bool ok = false;
  std::string why;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*CommCount)(const ncclComm_t, int*);
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*);
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
    sym(R.CommCount, "ncclCommCount");
    sym(R.CommUserRank, "ncclCommUserRank");
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

#define SH_HIP(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_error(e_ == hipErrorOutOfMemory ? SRS_ERR_OUT_OF_MEMORY : SRS_ERR_HIP, \
                       std::string(#expr " -> ") + hipGetErrorString(e_));             \
  } while (0)
#define SH_NCCL(expr)                                                                    \
  do {                                                                                   \
    ncclResult_t r_ = (expr);                                                            \
    if (r_ != ncclSuccess)                                                               \
      return set_error(SRS_ERR_HIP, std::string(#expr " -> ") + rccl().GetErrorString(r_)); \
  } while (0)
#define SH_TRY(expr)           \
  do {                         \
    int r_ = (expr);           \
    if (r_ != SRS_OK) return r_; \
  } while (0)

constexpr int kBits = 12;               // histogram bits
constexpr int kGroups = 512;            // key-range groups
constexpr int kRounds = 4;              // exchange rounds
constexpr size_t kMsgBytes = size_t(256) << 20;  // largest message

int key_bytes(int kind) {
  switch (kind) {
    case SRS_KEY_U8: case SRS_KEY_I8: return 1;
    case SRS_KEY_U16: case SRS_KEY_I16: return 2;
    case SRS_KEY_U32: case SRS_KEY_I32: case SRS_KEY_F32: return 4;
    case SRS_KEY_U64: case SRS_KEY_I64: case SRS_KEY_F64: return 8;
    default: return 0;
  }
}

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

// bins -> parts: part of bin b = floor(parts * (keys before b + half of b) /
// total), non-decreasing (srs_amd.dist.balanced_split)
std::vector<int32_t> balanced_split(const std::vector<uint64_t>& h, int parts) {
  std::vector<int32_t> out(h.size(), 0);
  double total = 0;
  for (uint64_t v : h) total += (double)v;
  if (total <= 0) return out;
  double before = 0;
  int prev = 0;
  for (size_t b = 0; b < h.size(); b++) {
    int p = (int)std::floor((before + 0.5 * (double)h[b]) * parts / total);
    p = std::min(std::max(p, prev), parts - 1);
    out[b] = prev = p;
    before += (double)h[b];
  }
  return out;
}

}  // namespace
}  // namespace srs

using namespace srs;

struct srs_shard_comm_s {
  ncclComm_t comm = nullptr;
  int world = 1, rank = 0, device = 0;
  hipStream_t cs = nullptr;   // communication stream
  hipStream_t ss = nullptr;   // round sorts
  hipStream_t own = nullptr;  // the stream srs_shard_sort_multi drives the rank on
  hipEvent_t ev_sort = nullptr;
  std::vector<hipEvent_t> ev;  // partition-chunk and round events
  Buf hist, lut, stage, part[1 + SRS_MAX_PAYLOADS], recv[1 + SRS_MAX_PAYLOADS];
  std::mutex mu;
};

namespace {

int make_comm_state(srs_shard_comm c) {
  SH_HIP(hipSetDevice(c->device));
  SH_HIP(hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking));
  SH_HIP(hipStreamCreateWithFlags(&c->ss, hipStreamNonBlocking));
  SH_HIP(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
  SH_HIP(hipEventCreateWithFlags(&c->ev_sort, hipEventDisableTiming));
  c->ev.resize(16);
  for (auto& e : c->ev) SH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return SRS_OK;
}

// One rank's part of the shard sort (the protocol above), on stream st.
int shard_sort(srs_shard_comm C, int64_t n, int kind, int up, const void* keys, int32_t np,
               const void* const* pays, const uint32_t* psz, void** keys_out,
               void** pays_out, int64_t* num_out, hipStream_t st) {
  const Rccl& R = rccl();
  const int w = C->world, me = C->rank;
  const int ks = key_bytes(kind);
  const int kbits = 8 * ks;
  const int bits = std::min(kBits, kbits);
  const int nb = 1 << bits;
  const int G = std::min(kGroups, nb);
  const int ncols = 1 + np;
  std::vector<uint32_t> width(ncols);
  width[0] = (uint32_t)ks;
  for (int c = 0; c < np; c++) width[1 + c] = psz[c];
  const int chunks = w > 1 ? 4 : 1;
  const int CH = (int)std::max<int64_t>(1, std::min<int64_t>(chunks, n));
  std::vector<int64_t> cb(CH + 1);
  for (int c = 0; c <= CH; c++) cb[c] = n * c / CH;
  if ((int)C->ev.size() < CH + kRounds + 1) return set_error(SRS_ERR_INTERNAL, "shard: events");

  // 1. chunk histograms, summed and all-reduced
  SH_TRY(C->hist.ensure((size_t)(CH + 1) * nb * 8));
  uint64_t* dh = (uint64_t*)C->hist.p;
  SH_HIP(hipMemsetAsync(dh, 0, (size_t)(CH + 1) * nb * 8, st));
  for (int c = 0; c < CH; c++)
    if (cb[c + 1] > cb[c])
      SH_TRY(srs_key_histogram_device(cb[c + 1] - cb[c], kind, up,
                                      (const char*)keys + (size_t)cb[c] * ks, bits,
                                      dh + (size_t)c * nb, st));
  std::vector<uint64_t> hc((size_t)CH * nb), tot(nb, 0);
  SH_HIP(hipMemcpyAsync(hc.data(), dh, hc.size() * 8, hipMemcpyDeviceToHost, st));
  SH_HIP(hipStreamSynchronize(st));
  for (int c = 0; c < CH; c++)
    for (int b = 0; b < nb; b++) tot[b] += hc[(size_t)c * nb + b];
  uint64_t* dt = dh + (size_t)CH * nb;
  SH_HIP(hipMemcpyAsync(dt, tot.data(), nb * 8, hipMemcpyHostToDevice, st));
  SH_NCCL(R.AllReduce(dt, dt, nb, ncclUint64, ncclSum, C->comm, st));
  SH_HIP(hipMemcpyAsync(tot.data(), dt, nb * 8, hipMemcpyDeviceToHost, st));
  SH_HIP(hipStreamSynchronize(st));

  // 2. bins -> groups -> ranks; each group's first / last bin
  const std::vector<int32_t> gob = balanced_split(tot, G);
  std::vector<uint64_t> gtot(G, 0);
  for (int b = 0; b < nb; b++) gtot[gob[b]] += tot[b];
  const std::vector<int32_t> rog = balanced_split(gtot, w);
  std::vector<int> gfirst(G, -1), glast(G, -1);
  for (int b = 0; b < nb; b++) {
    if (gfirst[gob[b]] < 0) gfirst[gob[b]] = b;
    glast[gob[b]] = b;
  }

  // 3. every rank's group sizes per chunk: mat[src][c][g]
  std::vector<int64_t> cc((size_t)CH * G, 0);
  for (int c = 0; c < CH; c++)
    for (int b = 0; b < nb; b++) cc[(size_t)c * G + gob[b]] += (int64_t)hc[(size_t)c * nb + b];
  SH_TRY(C->stage.ensure((size_t)(w + 1) * CH * G * 8));
  int64_t* dcc = (int64_t*)C->stage.p;
  SH_HIP(hipMemcpyAsync(dcc, cc.data(), cc.size() * 8, hipMemcpyHostToDevice, st));
  SH_NCCL(R.AllGather(dcc, dcc + cc.size(), cc.size(), ncclInt64, C->comm, st));
  std::vector<int64_t> mat((size_t)w * CH * G);
  SH_HIP(hipMemcpyAsync(mat.data(), dcc + cc.size(), mat.size() * 8, hipMemcpyDeviceToHost, st));
  SH_HIP(hipStreamSynchronize(st));
  auto M = [&](int src, int c, int g) { return mat[((size_t)src * CH + c) * G + g]; };

  // receive layout: round-major, then source, then chunk
  std::vector<std::vector<int>> owned(w);
  for (int g = 0; g < G; g++) owned[rog[g]].push_back(g);
  // round r of rank d: groups owned[d][lo_r, hi_r)
  auto rgrp = [&](int d, int r, int* lo, int* hi) {
    const int m = (int)owned[d].size();
    *lo = r * m / kRounds;
    *hi = (r + 1) * m / kRounds;
  };
  // (first group, records) of the round-r piece a source holds for rank d in chunk c
  auto piece = [&](int src, int c, int d, int r, int* g0) {
    int lo, hi;
    rgrp(d, r, &lo, &hi);
    *g0 = lo < hi ? owned[d][lo] : 0;
    int64_t cnt = 0;
    for (int i = lo; i < hi; i++) cnt += M(src, c, owned[d][i]);
    return cnt;
  };
  std::vector<int64_t> roff((size_t)kRounds * w * CH);
  std::vector<int64_t> rb0(kRounds), rb1(kRounds);
  int64_t pos = 0;
  for (int r = 0; r < kRounds; r++) {
    rb0[r] = pos;
    for (int src = 0; src < w; src++)
      for (int c = 0; c < CH; c++) {
        int g0;
        roff[((size_t)r * w + src) * CH + c] = pos;
        pos += piece(src, c, me, r, &g0);
      }
    rb1[r] = pos;
  }
  const int64_t total = pos;
  // where group g of chunk c starts in this rank's partitioned buffer
  std::vector<int64_t> soff((size_t)CH * (G + 1));
  for (int c = 0; c < CH; c++) {
    soff[(size_t)c * (G + 1)] = cb[c];
    for (int g = 0; g < G; g++)
      soff[(size_t)c * (G + 1) + g + 1] = soff[(size_t)c * (G + 1) + g] + M(me, c, g);
  }

  // buffers: partitioned input, receive (one rank, one chunk: the partition
  // buffer already has the receive layout, so the rounds sort it in place)
  const bool alias = w == 1 && CH == 1;
  for (int c = 0; c < ncols; c++) {
    SH_TRY(C->part[c].ensure((size_t)std::max<int64_t>(n, 1) * width[c]));
    if (!alias) SH_TRY(C->recv[c].ensure((size_t)std::max<int64_t>(total, 1) * width[c]));
  }
  auto rcol = [&](int c) { return (char*)(alias ? C->part[c].p : C->recv[c].p); };
  SH_TRY(C->lut.ensure((size_t)nb * 4));
  SH_HIP(hipMemcpyAsync(C->lut.p, gob.data(), (size_t)nb * 4, hipMemcpyHostToDevice, st));

  // messages of (round r, chunks [c0, c1)) on the communication stream
  auto issue = [&](int r, int c0, int c1) -> int {
    SH_NCCL(R.GroupStart());
    for (int d = 0; d < w; d++) {
      if (d == me) continue;
      for (int c = c0; c < c1; c++) {
        int g0;
        const int64_t scnt = piece(me, c, d, r, &g0);
        const int64_t rcnt = piece(d, c, me, r, &g0);
        for (int k = 0; k < ncols; k++) {
          const size_t wd = width[k];
          const int64_t per = (int64_t)std::max<size_t>(1, kMsgBytes / wd);
          int gs;
          piece(me, c, d, r, &gs);
          const char* sb = (const char*)C->part[k].p + (size_t)soff[(size_t)c * (G + 1) + gs] * wd;
          for (int64_t a = 0; a < scnt; a += per)
            SH_NCCL(R.Send(sb + (size_t)a * wd, (size_t)std::min(per, scnt - a) * wd, ncclUint8, d,
                           C->comm, C->cs));
          char* rbp = rcol(k) + (size_t)roff[((size_t)r * w + d) * CH + c] * wd;
          for (int64_t a = 0; a < rcnt; a += per)
            SH_NCCL(R.Recv(rbp + (size_t)a * wd, (size_t)std::min(per, rcnt - a) * wd, ncclUint8, d,
                           C->comm, C->cs));
        }
      }
    }
    SH_NCCL(R.GroupEnd());
    if (!alias)  // this rank's own piece
      for (int c = c0; c < c1; c++) {
        int gs;
        const int64_t cnt = piece(me, c, me, r, &gs);
        if (!cnt) continue;
        for (int k = 0; k < ncols; k++) {
          const size_t wd = width[k];
          SH_HIP(hipMemcpyAsync(rcol(k) + (size_t)roff[((size_t)r * w + me) * CH + c] * wd,
                                (const char*)C->part[k].p +
                                    (size_t)soff[(size_t)c * (G + 1) + gs] * wd,
                                (size_t)cnt * wd, hipMemcpyDeviceToDevice, C->cs));
        }
      }
    return SRS_OK;
  };

  // 4. partition chunk by chunk; round 0 of a chunk leaves right after it
  bool bad = false;
  std::vector<const void*> pin(np);
  std::vector<void*> pout(np);
  for (int c = 0; c < CH; c++) {
    const int64_t a = cb[c], m = cb[c + 1] - cb[c];
    if (m > 0) {
      for (int k = 0; k < np; k++) {
        pin[k] = (const char*)pays[k] + (size_t)a * width[1 + k];
        pout[k] = (char*)C->part[1 + k].p + (size_t)a * width[1 + k];
      }
      std::vector<int64_t> got(G, 0);
      SH_TRY(srs_partition_device(m, kind, up, (const char*)keys + (size_t)a * ks, np, pin.data(),
                                  psz, bits, (const int32_t*)C->lut.p, G,
                                  (char*)C->part[0].p + (size_t)a * ks, pout.data(), got.data(),
                                  st));
      for (int g = 0; g < G; g++) bad |= got[g] != M(me, c, g);
    }
    SH_HIP(hipEventRecord(C->ev[c], st));
    SH_HIP(hipStreamWaitEvent(C->cs, C->ev[c], 0));
    SH_TRY(issue(0, c, c + 1));
  }
  // 5. rounds: round r + 1 is queued behind round r on the communication
  // stream; round r's range is sorted on the side stream once it is in
  SH_HIP(hipStreamWaitEvent(C->ss, C->ev[0], 0));  // (after the histogram work on st)
  for (int r = 0; r < kRounds; r++) {
    if (r > 0) SH_TRY(issue(r, 0, CH));
    hipEvent_t er = C->ev[CH + r];
    SH_HIP(hipEventRecord(er, C->cs));
    SH_HIP(hipStreamWaitEvent(C->ss, er, 0));
    if (rb1[r] - rb0[r] < 2) continue;
    int lo, hi;
    rgrp(me, r, &lo, &hi);
    // top key bits every key of the range shares (its groups' bin range)
    auto shared = [&](int ga, int gb) {
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
    };
    std::vector<void*> cols(ncols);
    for (int k = 0; k < ncols; k++) cols[k] = rcol(k) + (size_t)rb0[r] * width[k];
    std::vector<int64_t> bounds;
    int known;
    if (alias) {  // one source: every group is its own segment
      bounds.push_back(0);
      known = kbits;
      for (int i = lo; i < hi; i++) {
        bounds.push_back(bounds.back() + M(me, 0, owned[me][i]));
        known = std::min(known, shared(i, i + 1));
      }
    } else {  // several sources interleave the groups: one segment
      bounds = {0, rb1[r] - rb0[r]};
      known = shared(lo, hi);
    }
    SH_TRY(srs_sort_segments_device(rb1[r] - rb0[r], kind, up, cols[0], np,
                                    np ? cols.data() + 1 : nullptr, psz,
                                    (int64_t)bounds.size() - 1, bounds.data(), known, C->ss));
  }
  SH_HIP(hipEventRecord(C->ev_sort, C->ss));
  SH_HIP(hipStreamWaitEvent(st, C->ev_sort, 0));
  SH_HIP(hipEventRecord(C->ev[CH + kRounds], C->cs));
  SH_HIP(hipStreamWaitEvent(st, C->ev[CH + kRounds], 0));
  // every rank learns whether a partition disagreed with the plan
  int64_t* dflag = dcc;
  const int64_t flag = bad ? 1 : 0;
  SH_HIP(hipMemcpyAsync(dflag, &flag, 8, hipMemcpyHostToDevice, st));
  SH_NCCL(R.AllReduce(dflag, dflag, 1, ncclInt64, ncclMax, C->comm, st));
  int64_t any = 0;
  SH_HIP(hipMemcpyAsync(&any, dflag, 8, hipMemcpyDeviceToHost, st));
  SH_HIP(hipStreamSynchronize(st));
  if (any)
    return set_error(SRS_ERR_INTERNAL, "shard: partition sizes differ from the histogram plan");
  *keys_out = rcol(0);
  for (int k = 0; k < np; k++) pays_out[k] = rcol(1 + k);
  *num_out = total;
  return SRS_OK;
}

}  // namespace

extern "C" {

int srs_shard_unique_id(void* id) {
  if (!id) return set_error(SRS_ERR_INVALID_ARG, "srs_shard_unique_id: id is NULL");
  const Rccl& R = rccl();
  if (!R.ok) return set_error(SRS_ERR_NO_DEVICE, R.why);
  ncclUniqueId u;
  SH_NCCL(R.GetUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return SRS_OK;
}

int srs_shard_comm_init(int32_t world, int32_t rank, const void* id, srs_shard_comm* comm) {
  if (!comm || !id || world < 1 || rank < 0 || rank >= world)
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_comm_init: world, rank, id, comm");
  *comm = nullptr;
  const Rccl& R = rccl();
  if (!R.ok) return set_error(SRS_ERR_NO_DEVICE, R.why);
  auto* c = new srs_shard_comm_s();
  c->world = world;
  c->rank = rank;
  if (hipGetDevice(&c->device) != hipSuccess) {
    delete c;
    return set_error(SRS_ERR_NO_DEVICE, "srs_shard_comm_init: no current device");
  }
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  const ncclResult_t r = R.CommInitRank(&c->comm, world, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return set_error(SRS_ERR_HIP, std::string("ncclCommInitRank -> ") + R.GetErrorString(r));
  }
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
  SH_NCCL(R.CommInitAll(cm.data(), num_devices, dv.data()));
  int dev0 = 0;
  (void)hipGetDevice(&dev0);
  int rc = SRS_OK;
  for (int i = 0; i < num_devices; i++) {
    auto* c = new srs_shard_comm_s();
    c->comm = cm[i];
    c->world = num_devices;
    c->rank = i;
    c->device = dv[i];
    comms[i] = c;
    if (rc == SRS_OK) rc = make_comm_state(c);
  }
  (void)hipSetDevice(dev0);
  if (rc != SRS_OK)
    for (int i = 0; i < num_devices; i++) {
      srs_shard_comm_destroy(comms[i]);
      comms[i] = nullptr;
    }
  return rc;
}

int srs_shard_comm_destroy(srs_shard_comm c) {
  if (!c) return SRS_OK;
  {
    std::lock_guard<std::mutex> g(c->mu);
    int dev0 = 0;
    (void)hipGetDevice(&dev0);
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    Buf* bufs[] = {&c->hist, &c->lut, &c->stage};
    for (Buf* b : bufs) b->release();
    for (auto& b : c->part) b.release();
    for (auto& b : c->recv) b.release();
    for (auto& e : c->ev)
      if (e) (void)hipEventDestroy(e);
    if (c->ev_sort) (void)hipEventDestroy(c->ev_sort);
    hipStream_t ss[] = {c->cs, c->ss, c->own};
    for (hipStream_t s : ss)
      if (s) (void)hipStreamDestroy(s);
    if (c->comm) (void)rccl().CommDestroy(c->comm);
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
  if (!comm || !keys_out || !num_out || num < 0 || (num > 0 && !keys) ||
      key_bytes(key_kind) == 0 || num_payloads < 0 || num_payloads > SRS_MAX_PAYLOADS ||
      (num_payloads > 0 && (!payloads || !payload_sizes || !payloads_out)))
    return set_error(SRS_ERR_INVALID_ARG, "srs_shard_sort_device: arguments");
  for (int k = 0; k < num_payloads; k++) {
    const uint32_t s = payload_sizes[k];
    if (s != 1 && s != 2 && s != 4 && s != 8)
      return set_error(SRS_ERR_UNSUPPORTED, "payload sizes must be 1, 2, 4 or 8 bytes");
  }
  std::lock_guard<std::mutex> g(comm->mu);
  int dev0 = 0;
  (void)hipGetDevice(&dev0);
  SH_HIP(hipSetDevice(comm->device));
  const int rc = shard_sort(comm, num, key_kind, up, keys, num_payloads, payloads, payload_sizes,
                            keys_out, payloads_out, num_out, (hipStream_t)stream);
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
  std::vector<int> rc(num_devices, SRS_OK);
  std::vector<std::string> err(num_devices);
  std::vector<std::thread> th;
  for (int i = 0; i < num_devices; i++)
    th.emplace_back([&, i] {
      srs_shard_comm c = comms[i];
      if (hipSetDevice(c->device) != hipSuccess) {
        rc[i] = SRS_ERR_HIP;
        err[i] = "hipSetDevice failed";
        return;
      }
      rc[i] = srs_shard_sort_device(
          c, nums[i], key_kind, up, keys[i], num_payloads,
          num_payloads ? payloads + (size_t)i * num_payloads : nullptr, payload_sizes,
          keys_out + i, num_payloads ? payloads_out + (size_t)i * num_payloads : nullptr,
          nums_out + i, c->own);
      if (rc[i] == SRS_OK && hipStreamSynchronize(c->own) != hipSuccess) rc[i] = SRS_ERR_HIP;
      if (rc[i] != SRS_OK) err[i] = srs_last_error();
    });
  for (auto& t : th) t.join();
  for (int i = 0; i < num_devices; i++)
    if (rc[i] != SRS_OK) return set_error(rc[i], "rank " + std::to_string(i) + ": " + err[i]);
  return SRS_OK;
}

}  // extern "C"

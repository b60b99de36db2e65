// srs_kernels.hip — CDNA4 (gfx950) kernels of the MSB radix sort.
//
// Replaces, in the reference (jonicho/simd-radix-sort):
//   * BitSorterSIMD::sortBit (radixSort.hpp:1587-1686): the per-bit AVX-512
//     compress-store partition. Here one pass splits a segment by a whole
//     multi-bit digit: ballot-based wave-level match ranks every key within
//     its tile (stable), keys and payload columns are staged in LDS in
//     digit order and written back with coalesced runs per bucket.
//   * radixRecursion (radixSort.hpp:1734-1759): depth-first recursion over
//     single bits. Here a breadth-first work-list of segments; each global
//     level handles all large segments in one launch per kernel.
//   * CmpSorterInsertionSort (radixSort.hpp:159-178): the <=16-element leaf.
//     Here segments that fit in LDS (<= kLocalCap) are finished by one
//     workgroup with LSD digit passes over the bits that still vary.
//
// All kernels are integer byte movement (no MFMA); the roofline is HBM.
// wave64 everywhere; __ballot returns 64-bit masks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "srs_common.h"
#include "srs_kernels.h"

namespace srs {

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
// Every column pointer is read from the SortDesc in memory, so the compiler
// cannot infer its address space and would emit FLAT loads/stores. FLAT ops
// count on lgkmcnt as well as vmcnt: every LDS wait (and the LDS-only
// barrier) would then also wait for the wave's outstanding global stores and
// loads. All data accesses therefore go through address_space(1) pointers
// (global_load / global_store, SGPR base + VGPR offset).
#define SRS_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ T gld(const void* p) {
  return *(const SRS_GLOBAL T*)(p);
}
template <typename T>
__device__ __forceinline__ void gst(void* p, T v) {
#if SRS_DIAG_NT_STORES  // (diagnostic: nontemporal element stores)
  __builtin_nontemporal_store(v, (SRS_GLOBAL T*)(p));
#else
  *(SRS_GLOBAL T*)(p) = v;
#endif
}

__device__ __forceinline__ uint64_t load_w(const char* p, uint32_t w) {
  switch (w) {
    case 1: return gld<uint8_t>(p);
    case 2: return gld<uint16_t>(p);
    case 4: return gld<uint32_t>(p);
    default: return gld<uint64_t>(p);
  }
}

// Width-templated accessors. Hot loops dispatch on the (uniform) column width
// ONCE, outside the unrolled loop (with_width), so that a tile's loads issue
// back to back; a switch per element serialises them (measured: the scatter
// and local kernels ran 25-30 % slower).
template <int W>
__device__ __forceinline__ uint64_t ldw(const char* p) {
  if constexpr (W == 1) return gld<uint8_t>(p);
  else if constexpr (W == 2) return gld<uint16_t>(p);
  else if constexpr (W == 4) return gld<uint32_t>(p);
  else return gld<uint64_t>(p);
}

template <int W>
__device__ __forceinline__ void stw(char* p, uint64_t v) {
  if constexpr (W == 1) gst<uint8_t>(p, (uint8_t)v);
  else if constexpr (W == 2) gst<uint16_t>(p, (uint16_t)v);
  else if constexpr (W == 4) gst<uint32_t>(p, (uint32_t)v);
  else gst<uint64_t>(p, v);
}

template <int W>
struct WidthTag {
  static constexpr int value = W;
};

template <typename F>
__device__ __forceinline__ void with_width(uint32_t w, F&& f) {
  switch (w) {
    case 1: f(WidthTag<1>{}); break;
    case 2: f(WidthTag<2>{}); break;
    case 4: f(WidthTag<4>{}); break;
    default: f(WidthTag<8>{}); break;
  }
}

__device__ __forceinline__ void store_w(char* p, uint32_t w, uint64_t v) {
  switch (w) {
    case 1: gst<uint8_t>(p, (uint8_t)v); break;
    case 2: gst<uint16_t>(p, (uint16_t)v); break;
    case 4: gst<uint32_t>(p, (uint32_t)v); break;
    default: gst<uint64_t>(p, v); break;
  }
}

// Strip access: element ebase + 64 k (k < IT, element < cnt) of a column
// whose element `first` is at `src`. Dense columns (stride == width) get
// compile-time per-k offsets (one 64-bit address per strip, immediate
// offsets after it); strided ones (AoS slices) a multiply per element.
// DENSE: the caller knows stride == width (no strided code path); FW != 0:
// the caller knows the width (no width switch: the compiler's vmcnt
// bookkeeping merges the switch's paths conservatively and then waits for
// stores issued after the loads it needs)
template <int IT, bool DENSE = false, int FW = 0, typename F>
__device__ __forceinline__ void with_strip(uint32_t w, uint32_t st, F&& f) {
  if constexpr (FW != 0) {
    static_assert(DENSE, "fixed width implies a dense strip here");
    f(WidthTag<FW>{}, std::integral_constant<bool, true>{});
  } else if (DENSE || st == w) {
    with_width(w, [&](auto W_) { f(W_, std::integral_constant<bool, true>{}); });
  } else {
    with_width(w, [&](auto W_) { f(W_, std::integral_constant<bool, false>{}); });
  }
}

// Buffer resource over `bytes` bytes at `base` (wave-uniform inputs, made
// provably uniform so the descriptor lives in SGPRs). Loads past `bytes`
// return 0 (hardware range check).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t strip_rsrc(const char* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)n,
                                           0x00020000);
}

// voff: per-lane byte offset; soff: wave-uniform byte offset (an SGPR);
// AUX: the cache-policy bits of the load (0: default)
template <int W, int AUX = 0>
__device__ __forceinline__ uint64_t bld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff = 0) {
  if constexpr (W == 1) return __builtin_amdgcn_raw_buffer_load_b8(r, voff, soff, AUX);
  else if constexpr (W == 2) return __builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, AUX);
  else if constexpr (W == 4) return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX);
  else {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, AUX);
    return (uint64_t)v[0] | ((uint64_t)v[1] << 32);
  }
}

// Loads slot k of a strip (element ebase + 64 k of the cnt elements that
// start at element `first`). Range-checked buffer loads: no branch per
// element and no select, so every load lands in its destination register
// and a tile's loads stay in flight together (guarded flat loads of 1/2/4-byte
// columns were each followed by a full vmcnt(0) wait inside loops; C2
// 29.9 -> 26.0 ms on the same box). Slots past cnt read 0.
template <int IT, bool DENSE = false, int FW = 0, int AUX = 0>
__device__ __forceinline__ void load_strip(uint64_t (&dst)[IT], const char* src, uint32_t w,
                                           uint32_t st, int64_t first, int ebase, int cnt) {
  const __amdgpu_buffer_rsrc_t r =
      strip_rsrc(src + first * (int64_t)st, cnt > 0 ? (uint32_t)cnt * st : 0u);
  with_strip<IT, DENSE, FW>(w, st, [&](auto W_, auto D_) {
    constexpr int W = decltype(W_)::value;
    constexpr bool D = decltype(D_)::value;
    const uint32_t o0 = (uint32_t)ebase * (D ? (uint32_t)W : st);
    // dense: per-slot offsets are immediates; strided: a uniform soffset
    // (a per-slot VGPR offset would be hoisted and held live)
#pragma unroll
    for (int k = 0; k < IT; k++) {
      if constexpr (D) dst[k] = bld<W, AUX>(r, o0 + (uint32_t)k * 64u * W);
      else dst[k] = bld<W, AUX>(r, o0, __builtin_amdgcn_readfirstlane((uint32_t)k * 64u * st));
    }
  });
}

template <int W>
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, uint64_t v, uint32_t voff,
                                    uint32_t soff = 0) {
  if constexpr (W == 1) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, voff, soff, 0);
  else if constexpr (W == 2) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, r, voff, soff, 0);
  else if constexpr (W == 4) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, r, voff, soff, 0);
  else {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    u32x2 x;
    x[0] = (uint32_t)v;
    x[1] = (uint32_t)(v >> 32);
    __builtin_amdgcn_raw_buffer_store_b64(x, r, voff, soff, 0);
  }
}

// Stores slot k of a strip (the layout of load_strip). Range-checked buffer
// stores: slots past cnt are dropped by the hardware, so value(k) must be
// safe to evaluate for every k (the caller clamps its LDS indices).
template <int IT, bool DENSE = false, int FW = 0, typename V>
__device__ __forceinline__ void store_strip(char* out, uint32_t w, uint32_t st, int64_t first,
                                            int ebase, int cnt, V&& value) {
  const __amdgpu_buffer_rsrc_t r =
      strip_rsrc(out + first * (int64_t)st, cnt > 0 ? (uint32_t)cnt * st : 0u);
  with_strip<IT, DENSE, FW>(w, st, [&](auto W_, auto D_) {
    constexpr int W = decltype(W_)::value;
    constexpr bool D = decltype(D_)::value;
    const uint32_t o0 = (uint32_t)ebase * (D ? (uint32_t)W : st);
#pragma unroll
    for (int k = 0; k < IT; k++) {
      if constexpr (D) bst<W>(r, value(k), o0 + (uint32_t)k * 64u * W);
      else bst<W>(r, value(k), o0, __builtin_amdgcn_readfirstlane((uint32_t)k * 64u * st));
    }
  });
}

// Key transform (the reference's bitDirUp table, radixSort.hpp:1568-1581,
// folded into one xor): unsigned order of u == the reference's key order.
//   u = bits ^ (sign ? mneg : mpos) = bits ^ mpos ^ (s & (mpos ^ mneg)),
// s = the key's sign bit smeared over the word (one v_ashr / v_bfe_i32), so a
// key costs ~5 VALU (u64) instead of a 64-bit select. CZ: the n <= thresh
// float case (SortDesc::canon_zero) maps -0.0 to +0.0 first; kernels are
// instantiated with CZ only for that case (SRS_KS_CANON in the dispatch).
template <typename U, bool CZ = false>
struct Xform {
  U mpos, cdiff, negzero;
  int sbit;
  bool canon;
  __device__ __forceinline__ void init(const SortDesc& d) {
    mpos = (U)d.mpos;
    cdiff = (U)(d.mpos ^ d.mneg);
    negzero = (U)d.negzero;
    sbit = d.key_bits - 1;
    canon = d.canon_zero != 0;
  }
  __device__ __forceinline__ U operator()(U bits) const {
    if constexpr (CZ) {
      if (canon && bits == negzero) bits = 0;
    }
    U sm;
    if constexpr (sizeof(U) == 8) sm = (U)((int64_t)bits >> 63);  // U64 only holds 8-byte keys
    else sm = (U)__builtin_amdgcn_sbfe((int)bits, sbit, 1);
    return bits ^ mpos ^ (sm & cdiff);
  }
  // inverse (no canon-zero case): x = u ^ mpos has the original sign bit
  // exactly when the key used mpos; otherwise the key is u ^ mneg
  __device__ __forceinline__ U inv(U u) const {
    const U x = u ^ mpos;
    U sm;
    if constexpr (sizeof(U) == 8) sm = (U)((int64_t)x >> 63);
    else sm = (U)__builtin_amdgcn_sbfe((int)x, sbit, 1);
    return x ^ (sm & cdiff);
  }
};

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }

// Digit table of a LUT pass (partition / balanced first level). Tables are
// read from LDS (u16 entries) when they fit, from global memory otherwise.
//   mode 0: flat, entry [u >> shift] (2^lut_bits entries)
//   mode 1: two-level: entry t = [u >> (shift + 4)] of a 4096-entry table;
//           if t has bit 15 set, the group is [4096 + (t & 0x7fff) * 16 +
//           ((u >> shift) & 15)] (a 12-bit bin split between groups).
//   mode 2: key ranges (SortDesc::rng_*): no table, a few compares.
//   mode 3: split table, u32 entry [u >> shift] (top 9 bits) = first group |
//           lg << 16: group = first + the next lg key bits.
struct DigitLut {
  const uint16_t* s;  // LDS copy, or null
  const int32_t* g;   // global flat table (mode 0 only, when s is null)
  int shift;
  int mode;
  const SortDesc* r;   // mode 2: the key ranges (SortDesc::rng_*)
};

// Digit of a transformed key for a global pass: the key's bits
// [shift, shift + bits), or (LUT) a group id looked up by its top bits.
template <int LUT, typename U>
__device__ __forceinline__ uint32_t pass_digit(U u, int shift, uint32_t mask, const DigitLut& L) {
  if constexpr (LUT) {
    if (L.mode == 2) {  // range c = #{k : u > hi_k} (unused ranges: hi = ~0)
      const uint64_t v = (uint64_t)u;
      const SortDesc* d = L.r;
      const uint32_t a = v > d->rng_hi[2] ? d->rng_adj[3]
                       : v > d->rng_hi[1] ? d->rng_adj[2]
                       : v > d->rng_hi[0] ? d->rng_adj[1] : d->rng_adj[0];
      return (uint32_t)(v >> L.shift) + a;
    }
    const uint64_t x = (uint64_t)u >> L.shift;
    if (L.mode == 3) {  // split table: first group | lg << 16 per top-9-bit bin
      const uint32_t e = ((const uint32_t*)L.s)[(uint32_t)x];
      const uint32_t lg = e >> 16;
      return (e & 0xFFFFu) + ((uint32_t)((uint64_t)u >> (L.shift - (int)lg)) & ((1u << lg) - 1u));
    }
    if (L.mode == 1) {
      const uint32_t t = L.s[x >> 4];
      return (t & 0x8000u) ? L.s[4096 + ((t & 0x7fffu) << 4) + (uint32_t)(x & 15)] : t;
    }
    return L.s ? (uint32_t)L.s[x] : (uint32_t)gld<int32_t>(L.g + x);
  }
  return (uint32_t)(u >> shift) & mask;
}

__device__ __forceinline__ uint32_t popc_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T x = __shfl_up(v, o, 64);
    if (lane >= (uint32_t)o) v += x;
  }
  return v;
}

// Exclusive scan across a workgroup of NT threads (NT / 64 waves). `sh` is
// an LDS array of at least NT / 64 + 1 elements. Returns the exclusive
// prefix; *total receives the workgroup total.
template <int NT, typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* sh, T* total) {
  constexpr int NW = NT / 64;
  const uint32_t wave = threadIdx.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane_id() == 63) sh[wave] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
      T t = sh[w];
      sh[w] = run;
      run += t;
    }
    sh[NW] = run;
  }
  __syncthreads();
  T r = inc - v + sh[wave];
  *total = sh[NW];
  __syncthreads();
  return r;
}

// ---- diagnostic phase stamps (build with -DSRS_STAMPS=1; never in the product
// build). Wave 0 drains its memory counters and reads s_memtime at each phase
// boundary; per-phase cycles are summed over workgroups into
// desc->stamp_acc[kernel * 16 + phase] (slot 0 counts workgroups).
#ifndef SRS_STAMPS
#define SRS_STAMPS 0
#endif
#if SRS_STAMPS
#define STAMP_DECL unsigned long long ts_[16] = {0}; int tsn_ = 0;
#define STAMP()                                                              \
  do {                                                                       \
    if (threadIdx.x == 0) {                                                  \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");            \
      if (tsn_ < 16) ts_[tsn_++] = __builtin_amdgcn_s_memtime();              \
    }                                                                        \
  } while (0)
#define STAMP_FLUSH(kid)                                                     \
  do {                                                                       \
    if (threadIdx.x == 0 && desc->stamp_acc) {                               \
      atomicAdd(&desc->stamp_acc[(kid) * 16], 1ull);                         \
      for (int i_ = 1; i_ < tsn_; i_++)                                      \
        atomicAdd(&desc->stamp_acc[(kid) * 16 + i_], ts_[i_] - ts_[i_ - 1]); \
    }                                                                        \
  } while (0)
#else
#define STAMP_DECL
#define STAMP() do {} while (0)
#define STAMP_FLUSH(kid) do {} while (0)
#endif

// Workgroup barrier that orders LDS accesses only. __syncthreads() also waits
// for every outstanding global load AND store of the wave (s_waitcnt
// vmcnt(0)); kernels that keep stores or prefetch loads in flight across a
// barrier use this one instead.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int NT, typename T>
__device__ __forceinline__ T block_excl_scan_lds(T v, T* sh, T* total) {
  constexpr int NW = NT / 64;
  const uint32_t wave = threadIdx.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane_id() == 63) sh[wave] = inc;
  lds_barrier();
  if (threadIdx.x == 0) {
    T run = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
      T t = sh[w];
      sh[w] = run;
      run += t;
    }
    sh[NW] = run;
  }
  lds_barrier();
  T r = inc - v + sh[wave];
  *total = sh[NW];
  lds_barrier();
  return r;
}

// Exclusive block scan with a single barrier: every thread sums the wave
// totals below its wave itself (broadcast LDS reads). The caller must pass
// another barrier before `sh` is written again.
template <int NT, typename T>
__device__ __forceinline__ T block_excl_scan_1b(T v, T* sh, T* total = nullptr) {
  constexpr int NW = NT / 64;
  const uint32_t wave = threadIdx.x >> 6;
  const T inc = wave_incl_scan(v);
  if (lane_id() == 63) sh[wave] = inc;
  lds_barrier();
  T run = 0, all = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) {
    const T t = sh[w];
    run += (uint32_t)w < wave ? t : (T)0;
    all += t;
  }
  if (total) *total = all;
  return inc - v + run;
}

// Peer mask of a lane's digit: the lanes of the wave whose digit equals it
// (and that are valid), one ballot per digit bit. Per bit: x = 0 / ~0 from
// the lane's bit (v_bfe_i32), m = ballot, peers &= ~(m ^ x) (v_bitop3 on
// gfx950). FIXED: all MAXB bits unconditionally (digits must be < 2^MAXB;
// zero high bits leave the mask unchanged), no per-bit predication;
// otherwise a uniform runtime loop over nbits.
template <int MAXB, bool FIXED>
__device__ __forceinline__ uint64_t wlms_peers(uint32_t d, bool ok, int nbits) {
  const uint64_t v = __ballot(ok);
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  auto step = [&](int b) {
    const uint32_t x = (uint32_t)__builtin_amdgcn_sbfe((int)d, b, 1);
    const uint64_t m = __ballot(x != 0);
    lo &= ~((uint32_t)m ^ x);
    hi &= ~((uint32_t)(m >> 32) ^ x);
  };
  if constexpr (FIXED) {
#pragma unroll
    for (int b = 0; b < MAXB; b++) step(b);
  } else {
    for (int b = 0; b < nbits; b++) step(b);
  }
  return ((uint64_t)hi << 32) | lo;
}

// Wave-level multisplit rank (stable): for each item slot k, lanes whose
// digit matches form a peer group (wlms_peers); the rank of a key is the
// wave's running count of its digit (per-wave LDS counter row `wc`) plus
// the number of lower-lane peers. Items are in striped order (slot k of lane
// l = wave-local element k * 64 + l), so ranks follow input order within a
// digit.
template <int ITEMS, int MAXB = kMaxDigitBits, bool FIXED = false, typename DigitFn,
          typename ValidFn>
__device__ __forceinline__ void wlms_rank_fn(DigitFn digit, ValidFn valid, int nbits,
                                             uint16_t* wc, uint32_t (&rank)[ITEMS]) {
#pragma unroll
  for (int k = 0; k < ITEMS; k++) {
    const bool ok = valid(k);
    const uint32_t d = digit(k);
    const uint64_t peers = wlms_peers<MAXB, FIXED>(d, ok, nbits);
    if (ok) {
      const uint32_t below = popc_below(peers);
      const uint32_t base = wc[d];
      rank[k] = base + below;
      if (below == 0) wc[d] = (uint16_t)(base + (uint32_t)__popcll(peers));
    }
  }
}

template <int ITEMS>
__device__ __forceinline__ void wlms_rank(const uint32_t (&dig)[ITEMS],
                                          const bool (&valid)[ITEMS], int nbits,
                                          uint16_t* wc, uint32_t (&rank)[ITEMS]) {
  wlms_rank_fn<ITEMS, kMaxDigitBits, false>([&](int k) { return dig[k]; },
                                            [&](int k) { return valid[k]; }, nbits, wc, rank);
}

// ---------------------------------------------------------------------------
// plan / bookkeeping kernels
// ---------------------------------------------------------------------------

// (choose_bits: srs_common.h, shared with the host)

// nt_over (gathered level): the segment's tile count from its tile table
// tmp2: bit 0 SortDesc::tmp2, bit 1 the level's buckets are all final (a
// range level of single-valued buckets: scatter them home)
__device__ __forceinline__ SegPlan make_plan(const Seg& g, int force_bits, int tmp2,
                                             const int32_t* nt_over = nullptr, int64_t s = 0) {
  const bool home = (tmp2 & 2) != 0;
  tmp2 &= 1;
  SegPlan p;
  p.start = g.start;
  p.len = g.len;
  // force_bits > 0: a digit-table level (consumes no fixed bits); < 0: a
  // plain digit of -force_bits bits (a partition whose groups are aligned
  // top-bit ranges)
  p.bits = force_bits ? (force_bits > 0 ? force_bits : -force_bits) : choose_bits(g.len, g.rbits);
  p.shift = force_bits > 0 ? g.rbits : g.rbits - p.bits;
  p.ntiles = nt_over ? nt_over[s] : (int32_t)((g.len + kTile - 1) / kTile);
  p.ngroups = (p.ntiles + kScanGroup - 1) / kScanGroup;
  p.buf = g.buf;
  // the last scatter lands in OUT (the local pass then sorts in place); with
  // SoA slice columns (tmp2) scatters alternate TMP / TMP2 and the local pass
  // writes the records home
  if (tmp2) p.dst = (g.buf == BUF_TMP) ? BUF_TMP2 : BUF_TMP;
  else p.dst = (g.buf == BUF_TMP) ? BUF_OUT : BUF_TMP;
  // a digit that takes every remaining bit leaves single-valued buckets,
  // which are final: write them home directly (no copy list; e.g. two-valued
  // keys, or the last level of a narrow key range)
  if (!tmp2 && (home || (force_bits <= 0 && p.shift == 0)) && g.buf == BUF_IN) p.dst = BUF_OUT;
  p.skip = 0;
  p.tile_base = 0;
  p.group_base = 0;
  return p;
}

__global__ void plan_kernel(const Seg* __restrict__ big, int64_t nbig,
                            SegPlan* __restrict__ plan, int64_t* __restrict__ tcount,
                            int64_t* __restrict__ gcount,
                            unsigned long long* __restrict__ var_or,
                            uint64_t* __restrict__ elems, int force_bits, int tmp2,
                            const int32_t* __restrict__ nt_over) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nbig) return;
  const Seg g = big[s];
  atomicAdd((unsigned long long*)elems, (unsigned long long)g.len);
  const SegPlan p = make_plan(g, force_bits, tmp2, nt_over, s);
  plan[s] = p;
  tcount[s] = p.ntiles;
  gcount[s] = p.ngroups;
  var_or[s] = 0;            // OR of the segment's (transformed) keys
  var_or[nbig + s] = ~0ull;  // and their AND (count_flush)
}

// Few segments (nbig <= kPlanSmallMax): the whole plan step in one
// workgroup, i.e. plan_kernel + both exclusive scans + plan_bases_kernel in
// one launch (the step is launch-bound for small sorts). Writes
// totals[0] = tiles, totals[1] = scan groups, totals[3] = keys, and zeroes
// the big-list counter the level's seg_scan appends to (the host has read it).
constexpr int kPlanSmallThreads = 1024;
__global__ __launch_bounds__(kPlanSmallThreads) void plan_small_kernel(
    const Seg* __restrict__ big, int64_t nbig, SegPlan* __restrict__ plan,
    int64_t* __restrict__ tbase, int64_t* __restrict__ gbase,
    unsigned long long* __restrict__ var_or, uint64_t* __restrict__ totals,
    unsigned long long* __restrict__ n_big_next, int force_bits, int tmp2,
    const int32_t* __restrict__ nt_over) {
  constexpr int NT = kPlanSmallThreads;
  __shared__ uint64_t sh[3][NT / 64 + 1];
  uint64_t tc = 0, gc = 0, ec = 0;
  for (int64_t s0 = 0; s0 < nbig; s0 += NT) {
    const int64_t s = s0 + threadIdx.x;
    SegPlan p{};
    uint64_t nt = 0, ng = 0, len = 0;
    if (s < nbig) {
      const Seg g = big[s];
      p = make_plan(g, force_bits, tmp2, nt_over, s);
      nt = (uint64_t)p.ntiles;
      ng = (uint64_t)p.ngroups;
      len = (uint64_t)g.len;
    }
    uint64_t tt, gt, et;
    const uint64_t tex = block_excl_scan<NT>(nt, sh[0], &tt);
    const uint64_t gex = block_excl_scan<NT>(ng, sh[1], &gt);
    block_excl_scan<NT>(len, sh[2], &et);
    if (s < nbig) {
      p.tile_base = (int64_t)(tc + tex);
      p.group_base = (int64_t)(gc + gex);
      plan[s] = p;
      tbase[s] = p.tile_base;
      gbase[s] = p.group_base;
      var_or[s] = 0;
      var_or[nbig + s] = ~0ull;
    }
    tc += tt;
    gc += gt;
    ec += et;
  }
  if (threadIdx.x == 0) {
    totals[0] = tc;
    totals[1] = gc;
    totals[3] = ec;
    *n_big_next = 0;
  }
}

__global__ void plan_bases_kernel(SegPlan* __restrict__ plan, int64_t nbig,
                                  const int64_t* __restrict__ tbase,
                                  const int64_t* __restrict__ gbase) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nbig) return;
  plan[s].tile_base = tbase[s];
  plan[s].group_base = gbase[s];
}

// index -> segment (binary search over the segments' exclusive bases);
// both maps of a level in one launch: threads [0, ntiles) map tiles,
// [ntiles, ntiles + ngroups) map scan groups
__global__ void seg_map2_kernel(const int64_t* __restrict__ tbase, int64_t ntiles,
                                int32_t* __restrict__ tile_seg, const int64_t* __restrict__ gbase,
                                int64_t ngroups, int32_t* __restrict__ group_seg, int64_t nbig) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t* bases = tbase;
  int32_t* out = tile_seg;
  if (t >= ntiles) {
    t -= ntiles;
    if (t >= ngroups) return;
    bases = gbase;
    out = group_seg;
  }
  int64_t lo = 0, hi = nbig - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (bases[mid] <= t) lo = mid; else hi = mid - 1;
  }
  out[t] = (int32_t)lo;
}

// XCD-aware block -> tile map: consecutive tiles run on one XCD (blocks are
// dealt round-robin over the 8 XCDs), so the partial cache lines that two
// neighbouring tiles write into the same bucket meet in one L2. Bijective for
// any grid size. Placement only affects speed, never results.
// The OR of every thread's `v` into the workgroup's slots, one per wave:
// reduced across the wave first, then one plain store per wave (64 lanes'
// LDS atomics on one address serialise: with them, this step took ~3 us of
// a small sort's 12). The caller barriers, then reads wave_or_read.
// (DPP row operations, no LDS crossbar and no address registers: the
// quad_perms, half-row and row mirrors leave each row's OR in all its lanes,
// row_bcast:15 / :31 carry rows 0-2 into row 3; lane 63 holds the result)
__device__ __forceinline__ uint32_t wave_or32(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ unsigned long long wave_or(unsigned long long v) {
  return ((unsigned long long)wave_or32((uint32_t)(v >> 32)) << 32) | wave_or32((uint32_t)v);
}
// max over the wave of v in [0, 2^15) from 15 ballots (scalar masks: no
// vector registers beyond the compares)
__device__ __forceinline__ int wave_max(int v) {
  uint64_t cand = __ballot(true);
  int r = 0;
#pragma unroll
  for (int b = 14; b >= 0; b--) {
    const uint64_t m = __ballot((v >> b) & 1) & cand;
    if (m) {
      cand = m;
      r |= 1 << b;
    }
  }
  return r;
}
// atomicMax of every thread's m into one LDS word: one atomic per wave
__device__ __forceinline__ void block_max_into(int* dst, int m) {  // (m < 2^15: bucket sizes)
  m = wave_max(m);
  if (lane_id() == 0 && m > 0) atomicMax(dst, m);
}
template <int NW>
__device__ __forceinline__ void wave_or_add(unsigned long long (&wor)[NW], uint32_t wave,
                                            uint32_t lane, unsigned long long v) {
  v = wave_or(v);
  if (lane == 0) wor[wave] = v;
}
template <int NW>
__device__ __forceinline__ unsigned long long wave_or_read(const unsigned long long (&wor)[NW]) {
  unsigned long long v = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) v |= wor[w];
  return v;
}

__device__ int g_xcd_rot;  // phase of each XCD's walk over its range (set_xcd_rotation)

__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nwg) {
  constexpr int64_t X = 8;
  const int64_t q = nwg / X, r = nwg % X;
  const int64_t xcd = bid % X, local = bid / X;
  const int64_t start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int64_t len = xcd < r ? q + 1 : q;
  const int m = g_xcd_rot;
  int64_t l = local;
  if (m == 1) l = (local + xcd * len / 8) % len;
  else if (m == 2) l = (local + (xcd * 5 % 8) * len / 8 + (xcd * len) / 61) % len;
  else if (m == 3 && (xcd & 1)) l = len - 1 - local;
  else if (m == 4) l = (local + xcd * len / 16) % len;
  return start + l;
}

// Partition passes: the digit table (2^lut_bits int32) is read once per
// element in two places of the scatter and once in the count; a per-element
// global lookup made the LUT scatter 1.7x slower than a plain digit pass.
// Tables up to 2^kLdsLutBits entries are staged in LDS instead (the caller
// barriers before the first use). Returns the table to read.
// LDS the digit table of a pass takes (u16 entries): LUT 1 any table kind
// (up to the 24 KB two-level table), LUT 2 the small kinds only (key ranges,
// the 2 KB split table), 0 none. The small instantiations keep the count at
// eight waves per SIMD and the scatter's staged digits.
template <int LUT>
constexpr int kLutLdsEntries = LUT == 1 ? kLdsLutEntries : LUT == 2 ? 1024 : 8;

template <int LUT, int NT>
__device__ __forceinline__ DigitLut stage_lut(const SortDesc* desc, uint16_t* slut) {
  DigitLut L{};
  if (!LUT) return L;
  L.shift = desc->lut_shift;
  L.mode = desc->lut_mode;
  L.r = desc;
  if constexpr (LUT == 2) {  // (small kinds only: the host never sends others here)
    if (L.mode == 3) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const __amdgpu_buffer_rsrc_t r = strip_rsrc((const char*)desc->digit_lut, 2048u);
      for (uint32_t i = threadIdx.x; i < 128u; i += NT)
        ((u32x4*)slut)[i] = __builtin_amdgcn_raw_buffer_load_b128(r, i * 16u, 0, 0);
      L.s = slut;
    }
    return L;
  }
  if (L.mode == 2) {  // key ranges: no table to stage
  } else if (L.mode == 3) {  // split table: 512 u32 entries (2 KB)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t r = strip_rsrc((const char*)desc->digit_lut, 2048u);
    for (uint32_t i = threadIdx.x; i < 128u; i += NT)
      ((u32x4*)slut)[i] = __builtin_amdgcn_raw_buffer_load_b128(r, i * 16u, 0, 0);
    L.s = slut;
  } else if (L.mode == 1) {
    const int n8 = (desc->lut_entries + 7) >> 3;  // 4096 + 16 per split bin (<= kLdsLutEntries)
    constexpr int K = (kLdsLutEntries / 8 + NT - 1) / NT;
    const __amdgpu_buffer_rsrc_t r = strip_rsrc((const char*)desc->digit_lut, (uint32_t)n8 * 16u);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v[K];
#pragma unroll
    for (int k = 0; k < K; k++)
      v[k] = __builtin_amdgcn_raw_buffer_load_b128(r, (threadIdx.x + (uint32_t)k * NT) * 16u, 0, 0);
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int i = threadIdx.x + k * NT;
      if (i < n8) ((u32x4*)slut)[i] = v[k];
    }
    L.s = slut;
  } else if (desc->lut_bits < 2) {
    for (int i = threadIdx.x; i < (1 << desc->lut_bits); i += NT)
      slut[i] = (uint16_t)gld<int32_t>(desc->digit_lut + i);
    L.s = slut;
  } else if (desc->lut_bits <= kLdsLutBits) {
    const int n4 = (1 << desc->lut_bits) >> 2;
    constexpr int K = ((1 << kLdsLutBits) / 4 + NT - 1) / NT;
    const __amdgpu_buffer_rsrc_t r = strip_rsrc((const char*)desc->digit_lut, (uint32_t)n4 * 16u);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v[K];
#pragma unroll
    for (int k = 0; k < K; k++)
      v[k] = __builtin_amdgcn_raw_buffer_load_b128(r, (threadIdx.x + (uint32_t)k * NT) * 16u, 0, 0);
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int i = threadIdx.x + k * NT;
      if (i < n4) {
        ((uint32_t*)slut)[2 * i] = (v[k][0] & 0xFFFFu) | (v[k][1] << 16);
        ((uint32_t*)slut)[2 * i + 1] = (v[k][2] & 0xFFFFu) | (v[k][3] << 16);
      }
    }
    L.s = slut;
  } else {
    L.g = desc->digit_lut;
  }
  return L;
}

// ---------------------------------------------------------------------------
// count: per-tile digit histogram (one tile-major row per tile) + varying bits
// ---------------------------------------------------------------------------
// A workgroup counts kCountTiles consecutive tiles; the next tile's loads go
// out before the current one is counted (two register sets, LDS-only
// barriers), so a workgroup's reads stay in flight across its tiles.
#ifndef SRS_COUNT_TILES
#define SRS_COUNT_TILES 1
#endif
constexpr int kCountTiles = SRS_COUNT_TILES;

struct CountTile {
  int64_t t;     // tile index (its histogram row)
  int32_t s;     // segment
  int32_t cnt;   // keys in the tile (0: none / past the last tile)
  bool vec;      // dense 4/8-byte keys read in 16-byte pieces
};

// element of item k: a dense 4/8-byte key column is read in 16-byte pieces
// (range-checked buffer loads; piece j of thread i holds elements
// (j * NT + i) * PER ...), anything else (1/2-byte keys, AoS records) one key
// per load. The histogram does not depend on the mapping.
template <typename KT>
__device__ __forceinline__ int count_elem(bool vec, int k) {
  constexpr int KB = (int)sizeof(KT);
  constexpr int PER = KB >= 4 ? 16 / KB : 1;
  return vec ? ((k / PER) * kCountThreads + (int)threadIdx.x) * PER + k % PER
             : k * kCountThreads + (int)threadIdx.x;
}

// Issues tile t's key loads (raw).
template <typename KT, typename U>
__device__ __forceinline__ CountTile count_load(const SortDesc* __restrict__ desc,
                                                const SegPlan* __restrict__ plan,
                                                const int32_t* __restrict__ tile_seg,
                                                const GTile* __restrict__ gt, int64_t t,
                                                int64_t ntiles, U (&raw)[kCountItems]) {
  CountTile T;
  T.t = t;
  T.cnt = 0;
  T.s = 0;
  T.vec = false;
  if (t >= ntiles) {
#pragma unroll
    for (int k = 0; k < kCountItems; k++) raw[k] = 0;
    return T;
  }
  T.s = tile_seg[t];
  const SegPlan P = plan[T.s];
  const char* kp = desc->key.base[P.buf];
  const uint32_t ks = desc->key.stride[P.buf];
  int64_t base;
  if (gt) {  // gathered level: the tile table says where the records are
    base = gt[t].src;
    T.cnt = gt[t].cnt;
  } else {
    const int64_t tl = t - P.tile_base;
    base = P.start + tl * kTile;
    const int64_t rem = P.len - tl * kTile;
    T.cnt = rem < kTile ? (int)rem : kTile;
  }
  constexpr int KB = (int)sizeof(KT);
  constexpr int PER = KB >= 4 ? 16 / KB : 1;
  static_assert(kCountItems % PER == 0, "whole 16-byte pieces per thread");
  T.vec = KB >= 4 && ks == (uint32_t)KB;
  const int cnt = T.cnt;
  if (T.vec) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t r =
        strip_rsrc(kp + base * (int64_t)KB, cnt > 0 ? (uint32_t)cnt * KB : 0u);
    u32x4 c[kCountItems / PER];
#pragma unroll
    for (int j = 0; j < kCountItems / PER; j++)
      c[j] = __builtin_amdgcn_raw_buffer_load_b128(
          r, (threadIdx.x + (uint32_t)j * kCountThreads) * 16u, 0, 0);
#pragma unroll
    for (int k = 0; k < kCountItems; k++) {
      const u32x4 v = c[k / PER];
      if constexpr (KB == 8)
        raw[k] = (U)((uint64_t)v[2 * (k % PER)] | ((uint64_t)v[2 * (k % PER) + 1] << 32));
      else
        raw[k] = (U)v[k % PER];
    }
  } else {
#pragma unroll
    for (int k = 0; k < kCountItems; k++) {
      const int e = count_elem<KT>(false, k);
      raw[k] = e < cnt ? (U)gld<KT>(kp + (base + e) * (int64_t)ks) : (U)0;
    }
  }
  return T;
}

// Counts a loaded tile into h (LDS, zeroed) and ORs its varying bits into *sor.
template <typename KT, typename U, int LUT, bool CZ>
__device__ __forceinline__ void count_add(const SortDesc* __restrict__ desc,
                                          const SegPlan* __restrict__ plan, const CountTile& T,
                                          const U (&raw)[kCountItems],
                                          uint32_t* h, unsigned long long* sor,
                                          const DigitLut& lut) {
  if (T.cnt == 0) return;
  const SegPlan P = plan[T.s];
  const uint32_t mask = (1u << P.bits) - 1;
  Xform<U, CZ> xf;
  xf.init(*desc);
  const int cnt = T.cnt;
  // the segment's varying bits are OR(keys) ^ AND(keys): no reference key
  // (loading the segment's first key put a dependent load in front of every
  // tile: C2's 4-byte counts 1.25 / 1.10 -> 0.85 ms without it)
  U vor = 0, vand = ~(U)0;
  // A wave holds 64 consecutive keys. Sorted or constant inputs give it one
  // digit, and 64 lanes adding into one LDS counter serialise (sorted C1
  // input: 3.6 ms per count launch against 1.45 uniform). A wave whose valid
  // lanes all share one digit adds once. Whether to look is decided once per
  // tile from the first item (the per-item check cost C2's 4-byte count 9 %).
  bool agg;
  {
    const uint32_t d = pass_digit<LUT>(xf(raw[0]), P.shift, mask, lut);
    const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
    const bool ok0 = count_elem<KT>(T.vec, 0) < cnt;
    agg = __ballot(ok0 && d == d0) == __ballot(ok0);
  }
  // No per-key branch or mask work: keys past the tile's end count into the
  // spare bin kMaxBins (an earlier loop with `if (ok)` around each add cost
  // C2's 4-byte count ~4x the VALU and ~8x the SALU instructions per key:
  // 1.26 ms per launch against 0.74 for the same bytes in
  // tools/probe/count_probe; SQ_INSTS_*, tools/prof_count.sh). `agg` is
  // uniform: the two loops are separate code (a per-item test of it left
  // ~20 scalar instructions per item in the mixed-digit loop).
  const bool full = cnt == kTile;
  auto digit_of = [&](int k, bool& ok) -> uint32_t {
    ok = full || count_elem<KT>(T.vec, k) < cnt;
    const U u = xf(raw[k]);
    vor |= ok ? u : (U)0;
    vand &= ok ? u : ~(U)0;
    return ok ? pass_digit<LUT>(u, P.shift, mask, lut) : (uint32_t)kMaxBins;
  };
  if (!agg) {
#pragma unroll
    for (int k = 0; k < kCountItems; k++) {
      bool ok;
      atomicAdd(&h[digit_of(k, ok)], 1u);
    }
  } else {
#pragma unroll
    for (int k = 0; k < kCountItems; k++) {
      bool ok;
      const uint32_t d = digit_of(k, ok);
      const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
      const uint64_t vm = __ballot(ok);  // (all lanes: a ballot inside `lane 0` sees one)
      if (__ballot(d != d0) == 0) {      // (one digit, or none valid: d0 = kMaxBins)
        if (lane_id() == 0) atomicAdd(&h[d0], (uint32_t)__popcll(vm));
      } else {
        atomicAdd(&h[d], 1u);
      }
    }
  }
  // one LDS atomic pair per wave (sor[0]: OR, sor[1]: AND; U's upper bits
  // are 0 in both, i.e. not varying)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    vor |= __shfl_xor(vor, o, 64);
    vand &= __shfl_xor(vand, o, 64);
  }
  if (lane_id() == 0) {
    atomicOr(&sor[0], (unsigned long long)vor);
    atomicAnd(&sor[1], (unsigned long long)vand);
  }
}

// After a barrier: the tile's row of u16 counts (a tile holds <= kTile = 4096
// keys; one coalesced 2*nb-byte write, packed pairs), h zeroed again for the
// tile after next, the varying bits published.
__device__ __forceinline__ void count_flush(const SegPlan* __restrict__ plan, const CountTile& T,
                                            uint32_t* h, unsigned long long* sor,
                                            uint16_t* __restrict__ hist,
                                            unsigned long long* __restrict__ var_or,
                                            unsigned long long* __restrict__ var_and) {
  static_assert(kTile < 65536, "u16 tile counts");
  if (T.cnt == 0) return;
  const uint32_t nb = 1u << plan[T.s].bits;
  uint32_t* row = (uint32_t*)(hist + T.t * kMaxBins);
  for (uint32_t i = threadIdx.x; i < nb / 2; i += kCountThreads) {
    row[i] = h[2 * i] | (h[2 * i + 1] << 16);
    h[2 * i] = 0;
    h[2 * i + 1] = 0;
  }
  if (threadIdx.x == 0) {
    const unsigned long long o = sor[0], a = sor[1];
    sor[0] = 0;
    sor[1] = ~0ull;
    // most tiles add nothing new: skip the (contended) atomics then
    const unsigned long long ko =
        __hip_atomic_load(&var_or[T.s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (o & ~ko) atomicOr(&var_or[T.s], o);
    const unsigned long long ka =
        __hip_atomic_load(&var_and[T.s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ka & ~a) atomicAnd(&var_and[T.s], a);
  }
}

// waves per SIMD the compiler must keep: 8 for the small-table passes of
// keys up to 4 bytes (C2's first level lands at 7 otherwise), no constraint
// elsewhere (forcing 8 on C1's plain pass spills 24 SGPRs it does not need
// to; on the 8-byte range level it spills VGPRs to scratch even at 7: that
// one runs at 6 waves, 73 VGPRs)
template <int LUT, int KB>
constexpr int kCountMinWaves = LUT == 2 && KB <= 4 ? 8 : 1;
template <typename KT, typename U, int LUT, bool CZ>
__global__ __launch_bounds__(kCountThreads, (kCountMinWaves<LUT, (int)sizeof(KT)>)) void count_kernel(
    const SortDesc* __restrict__ desc, const SegPlan* __restrict__ plan,
    const int32_t* __restrict__ tile_seg, uint16_t* __restrict__ hist,
    unsigned long long* __restrict__ var_or, unsigned long long* __restrict__ var_and,
    const GTile* __restrict__ gt, int64_t ntiles, const int32_t* __restrict__ torder) {
  constexpr int NH = kCountTiles > 1 ? 2 : 1;  // (one row when nothing is prefetched:
  __shared__ uint32_t h[NH][kMaxBins + 16];     //  the LUT pass keeps 6 workgroups per CU;
                                                //  bin kMaxBins: keys past the tile's end)
  __shared__ unsigned long long sh_or[NH][2];  // the tile's key OR and AND
  int64_t t0 = xcd_remap(blockIdx.x, gridDim.x) * kCountTiles;
  // gathered level: tiles in stripe order (each stripe's pieces lie back to
  // back, so the reads sweep memory); the rows do not depend on the order
  if (torder && kCountTiles == 1) t0 = torder[t0];
  __shared__ alignas(16) uint16_t slut[kLutLdsEntries<LUT>];
  U ra[kCountItems], rb[kCountItems];
  CountTile A = count_load<KT, U>(desc, plan, tile_seg, gt, t0, ntiles, ra);
  const DigitLut lut = stage_lut<LUT, kCountThreads>(desc, slut);
  for (uint32_t i = threadIdx.x; i < NH * (kMaxBins + 16); i += kCountThreads) (&h[0][0])[i] = 0;
  if (threadIdx.x < NH) {
    sh_or[threadIdx.x][0] = 0;
    sh_or[threadIdx.x][1] = ~0ull;
  }
  lds_barrier();
#pragma unroll
  for (int i = 0; i < kCountTiles; i += 2) {
    CountTile B;
    if (i + 1 < kCountTiles) B = count_load<KT, U>(desc, plan, tile_seg, gt, t0 + i + 1, ntiles, rb);
    count_add<KT, U, LUT, CZ>(desc, plan, A, ra, h[0], &sh_or[0][0], lut);
    lds_barrier();
    count_flush(plan, A, h[0], &sh_or[0][0], hist, var_or, var_and);
    if (i + 1 < kCountTiles) {
      if (i + 2 < kCountTiles) A = count_load<KT, U>(desc, plan, tile_seg, gt, t0 + i + 2, ntiles, ra);
      count_add<KT, U, LUT, CZ>(desc, plan, B, rb, h[NH - 1], &sh_or[NH - 1][0], lut);
      lds_barrier();
      count_flush(plan, B, h[NH - 1], &sh_or[NH - 1][0], hist, var_or, var_and);
    }
  }
}

// ---------------------------------------------------------------------------
// segmented column scan of the tile-major histograms:
//   offset(t, b) = sum_{b' < b} total(b') + sum_{t' < t in segment} H[t'][b]
// in three passes over groups of kScanGroup tiles (all row accesses coalesced)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kMaxBins) void group_sum_kernel(
    const SegPlan* __restrict__ plan, const int32_t* __restrict__ group_seg,
    const uint16_t* __restrict__ hist, uint32_t* __restrict__ gsum) {
  const int64_t g = blockIdx.x;
  const SegPlan P = plan[group_seg[g]];
  const uint32_t b = threadIdx.x;
  if (b >= (1u << P.bits)) return;
  const int64_t t0 = P.tile_base + (g - P.group_base) * kScanGroup;
  const int64_t t1 = min(t0 + kScanGroup, P.tile_base + P.ntiles);
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int64_t t = t0;
  for (; t + 4 <= t1; t += 4) {
    s0 += hist[(t + 0) * kMaxBins + b];
    s1 += hist[(t + 1) * kMaxBins + b];
    s2 += hist[(t + 2) * kMaxBins + b];
    s3 += hist[(t + 3) * kMaxBins + b];
  }
  for (; t < t1; t++) s0 += hist[t * kMaxBins + b];
  gsum[g * kMaxBins + b] = s0 + s1 + s2 + s3;
}

// ---------------------------------------------------------------------------
// device-wide exclusive scan of int64/uint64 (three small kernels)
// ---------------------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kScanChunk = kScanThreads * kScanItems;

__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(
    const uint64_t* __restrict__ x, int64_t n, uint64_t* __restrict__ bsum) {
  __shared__ uint64_t sh[kScanThreads / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanChunk;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    const int64_t i = base + k * kScanThreads + threadIdx.x;
    if (i < n) s += x[i];
  }
  uint64_t tot;
  block_excl_scan<kScanThreads>(s, sh, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void scan_bsums_kernel(uint64_t* __restrict__ bsum,
                                                          int64_t nb,
                                                          uint64_t* __restrict__ total) {
  __shared__ uint64_t sh[1024 / 64 + 1];
  uint64_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += 1024) {
    const int64_t i = b0 + threadIdx.x;
    const uint64_t v = i < nb ? bsum[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_scan<1024>(v, sh, &tot);
    if (i < nb) bsum[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

__global__ __launch_bounds__(kScanThreads) void scan_apply_kernel(
    const uint64_t* __restrict__ x, int64_t n, const uint64_t* __restrict__ bsum,
    uint64_t* __restrict__ y) {
  __shared__ uint64_t sh[kScanThreads / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanItems;
  uint64_t v[kScanItems];
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    const int64_t i = base + k;
    v[k] = i < n ? x[i] : 0;
    s += v[k];
  }
  uint64_t tot;
  uint64_t run = block_excl_scan<kScanThreads>(s, sh, &tot) + bsum[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    const int64_t i = base + k;
    if (i < n) y[i] = run;
    run += v[k];
  }
}

// ---------------------------------------------------------------------------
// children: turn each large segment's scanned histogram into child segments
// ---------------------------------------------------------------------------
struct Lists {
  Seg* big;
  Seg* local;    // segments of <= kLocalCapSmall keys
  Seg* local2;   // segments of <= kLocalCap keys
  Seg* copy;
  ListCounters* ctr;
};

__device__ __forceinline__ void emit_local(const Lists& L, const Seg& c) {
  if (c.len <= kLocalCapSmall) L.local[atomicAdd(&L.ctr->n_local, 1ull)] = c;
  else L.local2[atomicAdd(&L.ctr->n_local2, 1ull)] = c;
  atomicAdd(&L.ctr->local_elems, (unsigned long long)c.len);
}

__device__ __forceinline__ void emit_child(const Lists& L, Seg c) {
  if (c.len <= 0) return;
  if (c.rbits == 0 || c.len == 1) {
    if (c.buf == BUF_OUT) return;  // finished in place
    if (c.len <= kLocalCap) emit_local(L, c);
    else L.copy[atomicAdd(&L.ctr->n_copy, 1ull)] = c;
  } else if (c.len <= kLocalCap) {
    emit_local(L, c);
  } else {
    L.big[atomicAdd(&L.ctr->n_big, 1ull)] = c;
  }
}

// One block per large segment: exclusive scan over its groups (per bin),
// bin totals, bin bases, and the child segments of the next level.
// Every thread of the block offers at most one child (c.len == 0: none).
// Slots are reserved with one global atomic per list per block (a global
// atomic per child serialises on the counter).
__device__ __forceinline__ void emit_children_block(const Lists& L, const Seg& c) {
  enum { C_NONE = -1, C_BIG = 0, C_LOCAL = 1, C_LOCAL2 = 2, C_COPY = 3 };
  __shared__ unsigned int cnt[4];
  __shared__ unsigned long long basev[4];
  __shared__ unsigned long long lsum;
  int cls = C_NONE;
  if (c.len > 0) {
    if (c.rbits == 0 || c.len == 1) {
      if (c.buf != BUF_OUT)
        cls = c.len <= kLocalCapSmall ? C_LOCAL : c.len <= kLocalCap ? C_LOCAL2 : C_COPY;
    } else if (c.len <= kLocalCapSmall) {
      cls = C_LOCAL;
    } else if (c.len <= kLocalCap) {
      cls = C_LOCAL2;
    } else {
      cls = C_BIG;
    }
  }
  if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
  if (threadIdx.x == 0) lsum = 0;
  __syncthreads();
  unsigned int my = 0;
  if (cls != C_NONE) my = atomicAdd(&cnt[cls], 1u);
  if (cls == C_LOCAL || cls == C_LOCAL2) atomicAdd(&lsum, (unsigned long long)c.len);
  __syncthreads();
  if (threadIdx.x == 4 && lsum) atomicAdd(&L.ctr->local_elems, lsum);
  if (threadIdx.x < 4) {
    unsigned long long* ctrp = threadIdx.x == C_BIG ? &L.ctr->n_big
                             : threadIdx.x == C_LOCAL ? &L.ctr->n_local
                             : threadIdx.x == C_LOCAL2 ? &L.ctr->n_local2 : &L.ctr->n_copy;
    basev[threadIdx.x] = cnt[threadIdx.x] ? atomicAdd(ctrp, (unsigned long long)cnt[threadIdx.x]) : 0;
  }
  __syncthreads();
  if (cls == C_NONE) return;
  Seg* list = cls == C_BIG ? L.big : cls == C_LOCAL ? L.local : cls == C_LOCAL2 ? L.local2 : L.copy;
  list[basev[cls] + my] = c;
}

__global__ __launch_bounds__(kMaxBins) void seg_scan_kernel(
    SegPlan* __restrict__ plan, const uint32_t* __restrict__ gsum,
    uint64_t* __restrict__ gofs, uint64_t* __restrict__ sbase,
    const unsigned long long* __restrict__ var_or, Seg* big_next, Seg* local, Seg* local2,
    Seg* copy, ListCounters* ctr, const int32_t* __restrict__ lut_rbits, int mode,
    uint32_t* __restrict__ prun, int64_t rows) {
  // rows > 0: the one segment's scan over `rows` super-group rows (gsum /
  // gofs then hold the super sums / offsets; launch_offsets).
  // mode 0: a plain level. 1: a stripe level (every stripe is scattered, its
  // bucket sizes go to prun; the next level's segments come from
  // stripe_segs_kernel). 2: a gathered level (every segment is scattered:
  // its records are not where a skipped segment would have to be).
  __shared__ uint64_t scan_sh[kMaxBins / 64 + 1];
  __shared__ int single;
  const int64_t s = blockIdx.x;
  const SegPlan P = plan[s];
  const uint32_t nb = 1u << P.bits;
  const uint32_t b = threadIdx.x;
  if (b == 0) single = 0;
  uint64_t run = 0;
  if (b < nb) {
    const int64_t g0 = rows > 0 ? 0 : P.group_base;
    const int64_t g1 = rows > 0 ? rows : P.group_base + P.ngroups;
    int64_t g = g0;
    // One thread walks its bin's column serially, so a segment of many
    // groups is bound by load latency (one whole segment of 1e9 / 4 keys:
    // 2348 groups, 0.19-0.47 ms per launch at four loads per step): 32 group
    // sums in flight per step
    constexpr int U = 32;
    for (; g + U <= g1; g += U) {
      uint32_t a[U];
#pragma unroll
      for (int k = 0; k < U; k++) a[k] = gsum[(g + k) * kMaxBins + b];
#pragma unroll
      for (int k = 0; k < U; k++) {
        gofs[(g + k) * kMaxBins + b] = run;
        run += a[k];
      }
    }
    for (; g + 4 <= g1; g += 4) {
      const uint32_t a0 = gsum[(g + 0) * kMaxBins + b], a1 = gsum[(g + 1) * kMaxBins + b];
      const uint32_t a2 = gsum[(g + 2) * kMaxBins + b], a3 = gsum[(g + 3) * kMaxBins + b];
      gofs[(g + 0) * kMaxBins + b] = run;
      gofs[(g + 1) * kMaxBins + b] = run + a0;
      gofs[(g + 2) * kMaxBins + b] = run + a0 + a1;
      gofs[(g + 3) * kMaxBins + b] = run + a0 + a1 + a2;
      run += (uint64_t)a0 + a1 + a2 + a3;
    }
    for (; g < g1; g++) {
      gofs[g * kMaxBins + b] = run;
      run += gsum[g * kMaxBins + b];
    }
  }
  uint64_t tot;
  const uint64_t ex = block_excl_scan<kMaxBins>(run, scan_sh, &tot);
  if (b < nb) sbase[s * kMaxBins + b] = ex;
  if (b < nb && (int64_t)run == P.len && mode == 0) single = 1;
  if (mode == 1) {
    if (b < nb) prun[s * kMaxBins + b] = (uint32_t)run;
    return;
  }
  __syncthreads();
  Seg c;
  c.len = 0;
  if (single) {
    if (b == 0) {
      plan[s].skip = 1;
      const unsigned long long v = var_or[s] ^ var_or[gridDim.x + s];  // OR ^ AND of the keys
      c.start = P.start;
      c.len = P.len;
      c.rbits = v ? 64 - __clzll((long long)v) : 0;
      if (c.rbits > P.shift) c.rbits = P.shift;  // cannot happen; defensive
      c.buf = P.buf;
    }
  } else if (b < nb && run > 0) {
    c.start = P.start + (int64_t)ex;
    c.len = (int64_t)run;
    // a LUT level's group b is a key range whose keys share a known prefix
    c.rbits = (lut_rbits && lut_rbits[b] < P.shift) ? lut_rbits[b] : P.shift;
    c.buf = P.dst;
  }
  emit_children_block(Lists{big_next, local, local2, copy, ctr}, c);
}

// Per group: turn group offsets into every tile's bucket offsets.
// Tile offsets (bucket start of each tile inside its segment). offs32 != 0
// (every segment of the level < 2^32 keys): u32 rows, half the bytes of the
// u64 rows in `offs` for this kernel and the scatter that reads them.
__global__ __launch_bounds__(kMaxBins) void tile_offs_kernel(
    const SegPlan* __restrict__ plan, const int32_t* __restrict__ group_seg,
    const uint16_t* __restrict__ hist, const uint64_t* __restrict__ gofs,
    const uint64_t* __restrict__ sbase, uint64_t* __restrict__ offs,
    uint32_t* __restrict__ offs32) {
  const int64_t g = blockIdx.x;
  const int32_t s = group_seg[g];
  const SegPlan P = plan[s];
  const uint32_t b = threadIdx.x;
  if (P.skip || b >= (1u << P.bits)) return;
  const int64_t t0 = P.tile_base + (g - P.group_base) * kScanGroup;
  const int64_t t1 = min(t0 + kScanGroup, P.tile_base + P.ntiles);
  uint64_t run = sbase[s * kMaxBins + b] + gofs[g * kMaxBins + b];
  auto body = [&](auto* out) {
    using O = std::remove_pointer_t<decltype(out)>;
    int64_t t = t0;
    for (; t + 4 <= t1; t += 4) {
      const uint32_t a0 = hist[(t + 0) * kMaxBins + b], a1 = hist[(t + 1) * kMaxBins + b];
      const uint32_t a2 = hist[(t + 2) * kMaxBins + b], a3 = hist[(t + 3) * kMaxBins + b];
      out[(t + 0) * kMaxBins + b] = (O)run;
      out[(t + 1) * kMaxBins + b] = (O)(run + a0);
      out[(t + 2) * kMaxBins + b] = (O)(run + a0 + a1);
      out[(t + 3) * kMaxBins + b] = (O)(run + a0 + a1 + a2);
      run += (uint64_t)a0 + a1 + a2 + a3;
    }
    for (; t < t1; t++) {
      const uint32_t a = hist[t * kMaxBins + b];
      out[t * kMaxBins + b] = (O)run;
      run += a;
    }
  };
  if (offs32) body(offs32);
  else body(offs);
}

// ---------------------------------------------------------------------------
// stripe first level -> the second level's segments and gathered tiles
// ---------------------------------------------------------------------------
// Piece (s, b): stripe s's share of bucket b, prun[s][b] records at element
// plan[s].start + sbase[s][b] of the stripe level's destination buffer.
// Tiles never straddle a piece: piece (s, b) gives ceil(len / kTile) tiles.
// One block per bucket: per-piece tile prefix (ptile), the bucket's records
// and tiles (btot, bnt).
constexpr int kStripeThreads = 256;
__global__ __launch_bounds__(kStripeThreads) void stripe_tiles_kernel(
    const uint32_t* __restrict__ prun, int64_t nstripes, uint32_t* __restrict__ ptile,
    uint64_t* __restrict__ btot, uint32_t* __restrict__ bnt) {
  __shared__ uint64_t sh[kStripeThreads / 64 + 1];
  __shared__ uint64_t sh2[kStripeThreads / 64 + 1];
  const int b = blockIdx.x;
  uint64_t tiles = 0, keys = 0;
  for (int64_t s0 = 0; s0 < nstripes; s0 += kStripeThreads) {
    const int64_t s = s0 + threadIdx.x;
    const uint32_t len = s < nstripes ? prun[s * kMaxBins + b] : 0u;
    const uint64_t nt = (len + kTile - 1) / kTile;
    uint64_t tt, kt;
    const uint64_t ex = block_excl_scan<kStripeThreads>(nt, sh, &tt);
    block_excl_scan<kStripeThreads>((uint64_t)len, sh2, &kt);
    if (s < nstripes) ptile[s * kMaxBins + b] = (uint32_t)(tiles + ex);
    tiles += tt;
    keys += kt;
  }
  if (threadIdx.x == 0) {
    btot[b] = keys;
    bnt[b] = (uint32_t)tiles;
  }
}

// One block of kMaxBins threads (thread = bucket): the non-empty buckets
// become the next level's segments (logical start = records in lower
// buckets, still `rbits` bits to sort, living in `buf`), with their tile
// counts (nt_over) and first tiles (btile, per bucket); n_big is set.
__global__ __launch_bounds__(kMaxBins) void stripe_segs_kernel(
    const uint64_t* __restrict__ btot, const uint32_t* __restrict__ bnt, int nb, int rbits,
    int buf, Seg* __restrict__ big, int32_t* __restrict__ nt_over,
    uint32_t* __restrict__ btile, ListCounters* __restrict__ ctr,
    const int32_t* __restrict__ lut_rbits) {
  __shared__ uint64_t sh[3][kMaxBins / 64 + 1];
  const int b = threadIdx.x;
  const uint64_t len = b < nb ? btot[b] : 0;
  const uint64_t nt = b < nb ? bnt[b] : 0;
  const uint64_t used = len > 0 ? 1 : 0;
  uint64_t tot_len, tot_nt, tot_used;
  const uint64_t start = block_excl_scan<kMaxBins>(len, sh[0], &tot_len);
  const uint64_t tb = block_excl_scan<kMaxBins>(nt, sh[1], &tot_nt);
  const uint64_t idx = block_excl_scan<kMaxBins>(used, sh[2], &tot_used);
  if (b < nb) btile[b] = (uint32_t)tb;
  if (used) {
    // a digit-table level's group b is a key range whose keys share a prefix
    const int rb = (lut_rbits && lut_rbits[b] < rbits) ? lut_rbits[b] : rbits;
    big[idx] = Seg{(int64_t)start, (int64_t)len, rb, buf};
    nt_over[idx] = (int32_t)nt;
  }
  if (b == 0) ctr->n_big = tot_used;
}

// The gathered level's tiles in stripe-major order (stripe s's pieces of
// buckets 0, 1, ... lie back to back in memory), for its count. Block per
// stripe, thread per bucket: the stripe's tile total, then (second kernel)
// the stripe's first position and each piece's tiles.
__global__ __launch_bounds__(kMaxBins) void stripe_rows_kernel(const uint32_t* __restrict__ prun,
                                                               int nb,
                                                               uint32_t* __restrict__ rowtot) {
  __shared__ uint64_t sh[kMaxBins / 64 + 1];
  const int64_t s = blockIdx.x;
  const uint32_t b = threadIdx.x;
  const uint64_t my = b < (uint32_t)nb ? (prun[s * kMaxBins + b] + kTile - 1) / kTile : 0;
  uint64_t tot;
  block_excl_scan<kMaxBins>(my, sh, &tot);
  if (b == 0) rowtot[s] = (uint32_t)tot;
}

__global__ __launch_bounds__(kMaxBins) void stripe_order_kernel(
    const uint32_t* __restrict__ prun, const uint32_t* __restrict__ ptile,
    const uint32_t* __restrict__ btile, const uint32_t* __restrict__ rowtot, int nb,
    int32_t* __restrict__ torder) {
  __shared__ uint64_t sh[kMaxBins / 64 + 1];
  const int64_t s = blockIdx.x;
  const uint32_t b = threadIdx.x;
  uint64_t before = 0;  // tiles of the stripes before s
  for (int64_t i = b; i < s; i += kMaxBins) before += rowtot[i];
  uint64_t base;
  block_excl_scan<kMaxBins>(before, sh, &base);
  const uint32_t len = b < (uint32_t)nb ? prun[s * kMaxBins + b] : 0u;
  const uint64_t my = (len + kTile - 1) / kTile;
  uint64_t tot;
  uint64_t pos = base + block_excl_scan<kMaxBins>(my, sh, &tot);
  if (my) {
    const uint32_t t = btile[b] + ptile[s * kMaxBins + b];
    for (uint32_t c = 0; c < (uint32_t)my; c++) torder[pos + c] = (int32_t)(t + c);
  }
}

// One thread per piece: its tiles' table entries (bucket-major, then stripe
// order, so a bucket's tiles list its records in input order: stable).
__global__ void stripe_gtile_kernel(const uint32_t* __restrict__ prun,
                                    const uint32_t* __restrict__ ptile,
                                    const uint32_t* __restrict__ btile,
                                    const uint64_t* __restrict__ sbase,
                                    const SegPlan* __restrict__ plan, int64_t nstripes, int nb,
                                    GTile* __restrict__ gt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nstripes * nb) return;
  const int64_t s = i / nb;
  const int b = (int)(i % nb);
  const uint32_t len = prun[s * kMaxBins + b];
  if (len == 0) return;
  const int64_t src = plan[s].start + (int64_t)sbase[s * kMaxBins + b];
  GTile* out = gt + btile[b] + ptile[s * kMaxBins + b];
  for (uint32_t c = 0; c * (uint32_t)kTile < len; c++) {
    const uint32_t rem = len - c * (uint32_t)kTile;
    out[c] = GTile{src + (int64_t)c * kTile, (int32_t)(rem < (uint32_t)kTile ? rem : kTile), 0};
  }
}

// ---------------------------------------------------------------------------
// scatter: rank one tile by digit, stage in LDS, write coalesced runs
// ---------------------------------------------------------------------------
// Column 0 holds the key in its low bytes (SoA: the key column; AoS: the
// record's first <=8-byte slice). A tile's loads (column 0, the first payload
// column, its row of bucket offsets) are issued together; stores are never
// waited for (LDS-only barriers between columns). One tile per workgroup,
// two 16-wave workgroups per CU (<= 64 VGPRs); persistent variants that
// prefetch the next tile measured slower.
template <int LUT>
struct ScatterLds {
  uint64_t sval[kTile];
  // digit of each staged slot (big-table passes recompute it instead: their 24 KB
  // table must leave room for two workgroups per CU)
  uint16_t sdig[(LUT == 1 || !SRS_SCATTER_SDIG) ? 1 : kTile];
  alignas(8) uint16_t wc[kScatterThreads / 64][kMaxBins];  // zeroed as u64
  uint16_t bin_start[kMaxBins];  // tile offsets <= kTile fit 16 bits
  int64_t gdst[kMaxBins];
  uint32_t scan_sh[kScatterThreads / 64 + 1];
};

struct TileInfo {
  int64_t base;   // first element of the tile
  int32_t cnt;    // elements in the tile (0: skip)
  int32_t s;      // segment
  int64_t t;      // tile index in the level
};

#ifdef SRS_DIAG_LOOKBACK
// Diagnostic: a decoupled look-back over the tiles of a
// segment, per digit, as a one-pass scatter would need it instead of the
// count pass + scans: publish the tile's digit count (flag 1), walk back
// over the predecessors' words (flag 1: add and continue, flag 2: an
// inclusive prefix, add and stop), publish the inclusive prefix (flag 2).
// Status words are single 4-byte sc1 stores / sc1 loads (self-contained
// {flag, value} granules). The result is only compared with the offsets
// the count pass produced (lb_err[0] counts mismatches); spins are bounded.
__device__ __forceinline__ void diag_lookback(const SortDesc* __restrict__ desc,
                                              const SegPlan& P, int64_t t, uint32_t d,
                                              uint32_t tb, int64_t my_off,
                                              const uint64_t* __restrict__ offs,
                                              const uint32_t* __restrict__ offs32) {
  uint32_t* st = desc->lb_status;
  const uint64_t first = offs32 ? offs32[P.tile_base * kMaxBins + d] : offs[P.tile_base * kMaxBins + d];
  uint32_t pre = 0;
  if (t == P.tile_base) {
    __hip_atomic_store(&st[t * kMaxBins + d], (2u << 30) | tb, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_store(&st[t * kMaxBins + d], (1u << 30) | tb, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    int64_t j = t - 1;
    uint32_t spins = 0, hops = 0;
    while (true) {
      const uint32_t v = __hip_atomic_load(&st[j * kMaxBins + d], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t f = v >> 30;
      if (f == 0) {
        if (++spins > (1u << 22)) {
          atomicAdd(&desc->lb_err[1], 1ull);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      pre += v & 0x3FFFFFFFu;
      hops++;
      if (f == 2 || j == P.tile_base) break;
      j--;
    }
    __hip_atomic_store(&st[t * kMaxBins + d], (2u << 30) | (pre + tb), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    if (d == 0) atomicAdd(&desc->lb_err[2], (unsigned long long)hops);
  }
  if ((uint64_t)my_off - first != pre) atomicAdd(&desc->lb_err[0], 1ull);
}
#endif

template <typename KT, typename U, bool PRE3>
__device__ __forceinline__ TileInfo scatter_load_tile(
    const SortDesc* __restrict__ desc, const SegPlan* __restrict__ plan,
    const int32_t* __restrict__ tile_seg, const uint64_t* __restrict__ offs,
    const uint32_t* __restrict__ offs32, const GTile* __restrict__ gt, int64_t t, int ncols,
    uint64_t (&v0)[kScatterItems], uint64_t (&v1)[kScatterItems],
    uint64_t (&v2)[kScatterItems], int64_t& my_off) {
  constexpr int IT = kScatterItems;
  TileInfo ti;
  ti.t = t;
  ti.s = tile_seg[t];
  const SegPlan P = plan[ti.s];
  if (gt) {  // gathered level (never skipped)
    ti.base = gt[t].src;
    ti.cnt = gt[t].cnt;
  } else {
    const int64_t tl = t - P.tile_base;
    ti.base = P.start + tl * kTile;
    const int64_t rem = P.len - tl * kTile;
    ti.cnt = P.skip ? 0 : (rem < kTile ? (int)rem : kTile);
  }
  const int ebase = (int)(threadIdx.x >> 6) * IT * 64 + (int)lane_id();
  constexpr int LA = SRS_SCATTER_LOAD_AUX;
  load_strip<IT, false, 0, LA>(v0, desc->cols[0].base[P.buf], desc->cols[0].width,
                               desc->cols[0].stride[P.buf], ti.base, ebase, ti.cnt);
  // (desc->pair: in TMP / TMP2 columns 1 and 2 are one 8-byte word column,
  // loaded whole into v1)
  const bool pair_src = PRE3 && desc->pair && (P.buf == BUF_TMP || P.buf == BUF_TMP2);
  if (ncols > 1)
    load_strip<IT, false, 0, LA>(v1, desc->cols[1].base[P.buf], pair_src ? 8u : desc->cols[1].width,
                                 desc->cols[1].stride[P.buf], ti.base, ebase, ti.cnt);
  if (PRE3 && ncols > 2 && !pair_src)
    load_strip<IT, false, 0, LA>(v2, desc->cols[2].base[P.buf], desc->cols[2].width,
                                 desc->cols[2].stride[P.buf], ti.base, ebase, ti.cnt);
  my_off = 0;
  if (ti.cnt > 0 && threadIdx.x < (1u << P.bits))
    my_off = offs32 ? (int64_t)offs32[t * kMaxBins + threadIdx.x]
                    : (int64_t)offs[t * kMaxBins + threadIdx.x];
  return ti;
}

template <typename KT, typename U, int LUT, bool CZ, bool PRE3>
__device__ __forceinline__ void scatter_process_tile(
    const SortDesc* __restrict__ desc, const SegPlan* __restrict__ plan, ScatterLds<LUT>& L,
    const TileInfo& ti, int ncols, const uint64_t (&v0)[kScatterItems],
    uint64_t (&v1)[kScatterItems], uint64_t (&v2)[kScatterItems], int64_t my_off,
    const DigitLut& lut, const uint64_t* __restrict__ lb_offs = nullptr,
    const uint32_t* __restrict__ lb_offs32 = nullptr) {
  constexpr int NT = kScatterThreads;
  constexpr int IT = kScatterItems;
  constexpr int NW = NT / 64;
  const SegPlan P = plan[ti.s];
  const uint32_t nb = 1u << P.bits;
  const uint32_t mask = nb - 1;
  const uint32_t wave = threadIdx.x >> 6;
  const int ebase = (int)wave * IT * 64 + (int)lane_id();
  const int cnt = ti.cnt;
  Xform<U, CZ> xf;
  xf.init(*desc);
  const int kbytes = desc->key_bits >> 3;
  const uint64_t kmask = kbytes == 8 ? ~0ull : ((1ull << (8 * kbytes)) - 1);
  STAMP_DECL
  STAMP();

  if constexpr (LUT) lds_barrier();  // publishes the staged digit table
  // each wave zeroes its own counter row (no barrier: a wave's LDS accesses
  // execute in order, and the rank touches only the wave's row), so a wave
  // starts ranking as soon as its own loads have landed
  static_assert(kMaxBins % 256 == 0, "row zeroing: 64 lanes x u64");
#pragma unroll
  for (int i = 0; i < kMaxBins / 256; i++)
    ((uint64_t*)&L.wc[wave][0])[i * 64 + lane_id()] = 0;
  auto valid = [&](int k) -> bool { return ebase + k * 64 < cnt; };
  // each key's digit, computed once (transform + digit cost ~15 VALU per key)
  uint32_t dg[IT];
#pragma unroll
  for (int k = 0; k < IT; k++) dg[k] = pass_digit<LUT>(xf((U)(v0[k] & kmask)), P.shift, mask, lut);
  STAMP();  // 1: loads returned

  uint32_t pos[IT];
  // digits are < 2^kMaxDigitBits: every ballot unconditionally (no per-bit
  // predication); bits above P.bits are zero in every lane
  wlms_rank_fn<IT, kMaxDigitBits, true>([&](int k) { return dg[k]; }, valid, P.bits,
                                        &L.wc[wave][0], pos);
  lds_barrier();
  STAMP();  // 2: ranked

  {  // per-bin totals over waves -> per-wave exclusive offsets; tile scan
    const uint32_t my_bin = threadIdx.x;
    uint32_t tb = 0;
    if (my_bin < nb) {
#pragma unroll
      for (int w = 0; w < NW; w++) {
        const uint32_t c = L.wc[w][my_bin];
        L.wc[w][my_bin] = (uint16_t)tb;
        tb += c;
      }
    }
    const uint32_t ex = block_excl_scan_1b<NT>(tb, L.scan_sh);
    if (my_bin < nb) {
      L.bin_start[my_bin] = ex;
      L.gdst[my_bin] = P.start + my_off - (int64_t)ex;
    }
#ifdef SRS_DIAG_LOOKBACK
    if (my_bin < nb && desc->lb_status)
      diag_lookback(desc, P, ti.t, my_bin, tb, my_off, lb_offs, lb_offs32);
#endif
  }
  lds_barrier();
  STAMP();  // 3: tile scan

#pragma unroll
  for (int k = 0; k < IT; k++) {
    if (valid(k)) {
      const uint32_t d = dg[k];
      pos[k] = L.bin_start[d] + L.wc[wave][d] + pos[k];
      L.sval[pos[k]] = v0[k];
      if constexpr (LUT != 1 && SRS_SCATTER_SDIG) L.sdig[pos[k]] = (uint16_t)d;
    }
  }
  lds_barrier();
  STAMP();  // 4: column 0 staged

#ifdef SRS_DIAG_WIN
  // diagnostic (wrong result): each window of SRS_DIAG_WIN consecutive tiles
  // of a segment is its own little bucket array, so the scattered runs land
  // in a window of SRS_DIAG_WIN * kTile records instead of the whole segment
  auto diag_win = [&](int j, uint32_t d) -> int64_t {
    constexpr int S = SRS_DIAG_WIN;
    const int64_t tl = (ti.base - P.start) / kTile;
    const int64_t wb = P.start + (tl / S) * S * kTile;
    const int64_t per = (int64_t)S * kTile >> P.bits;
    const int64_t r = ((tl % S) * (per / S) + (j - (int)L.bin_start[d])) % per;
    const int64_t a = wb + (int64_t)d * per + r;
    return a < P.start + P.len ? a : ti.base + j;
  };
#endif
  // column 0: output slot j's bucket was staged with it
  uint16_t dout[IT];
  {
    char* out = desc->cols[0].base[P.dst];
    const uint32_t w = desc->cols[0].width, st = desc->cols[0].stride[P.dst];
    with_width(w, [&](auto W_) {
#pragma unroll
      for (int i = 0; i < IT; i++) {
        const int j = i * NT + (int)threadIdx.x;
        dout[i] = 0;
        if (j < cnt) {
          const uint64_t x = L.sval[j];
          uint32_t d;
          if constexpr (LUT == 1 || !SRS_SCATTER_SDIG) d = pass_digit<LUT>(xf((U)(x & kmask)), P.shift, mask, lut);
          else d = L.sdig[j];
          dout[i] = (uint16_t)d;
          #ifdef SRS_DIAG_SEQW
          stw<decltype(W_)::value>(out + ((int64_t)j + ti.base) * (int64_t)st, x);
#elif defined(SRS_DIAG_WIN)
          stw<decltype(W_)::value>(out + diag_win(j, d) * (int64_t)st, x);
#else
          stw<decltype(W_)::value>(out + ((int64_t)j + L.gdst[d]) * (int64_t)st, x);
#endif
        }
      }
    });
  }
  // Columns 1..: column c's registers are staged in LDS, then the next
  // column's loads that use them go out before column c's stores: column
  // c + 1 (PRE3 = false: one payload register set) or c + 2 (PRE3: three
  // columns loaded up front, v0, v1, v2). A wave's loads complete in issue
  // order with its stores (vmcnt counts both), so a load issued after a
  // store cannot be used before that store is acknowledged; with one set,
  // column c + 1's loads follow column c - 1's stores and their latency is
  // partly exposed (C2, three columns: PRE3 scatter 3.53-3.62 -> 3.48 ms).
  // PRE3 costs 9 VGPRs, which slowed the two-column C3 scatter: it is an
  // instantiation of its own.
  constexpr int STEP = PRE3 ? 2 : 1;
  auto move_col = [&](int c, uint64_t (&v)[IT]) {
    const uint32_t cw = desc->cols[c].width, cst = desc->cols[c].stride[P.dst];
    lds_barrier();  // every slot of the previous column has been read
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (valid(k)) L.sval[pos[k]] = v[k];
    lds_barrier();
    if (c + STEP < ncols)
      load_strip<IT, false, 0, SRS_SCATTER_LOAD_AUX>(
          v, desc->cols[c + STEP].base[P.buf], desc->cols[c + STEP].width,
          desc->cols[c + STEP].stride[P.buf], ti.base, ebase, cnt);
    char* out = desc->cols[c].base[P.dst];
    with_width(cw, [&](auto W_) {
#pragma unroll
      for (int i = 0; i < IT; i++) {
        const int j = i * NT + (int)threadIdx.x;
        if (j < cnt)
          #ifdef SRS_DIAG_SEQW
          stw<decltype(W_)::value>(out + ((int64_t)j + ti.base) * (int64_t)cst, L.sval[j]);
#elif defined(SRS_DIAG_WIN)
          stw<decltype(W_)::value>(out + diag_win(j, dout[i]) * (int64_t)cst, L.sval[j]);
#else
          stw<decltype(W_)::value>(out + ((int64_t)j + L.gdst[dout[i]]) * (int64_t)cst,
                                   L.sval[j]);
#endif
      }
    });
  };
  if constexpr (PRE3) {
    if (desc->pair) {
      // key + two 4-byte payloads whose destination (TMP / TMP2) holds them as
      // one interleaved word per record: one staging pass and 8-byte stores
      // (from IN / OUT, the caller's arrays, the two columns were loaded apart
      // and are joined here)
      if (P.buf != BUF_TMP && P.buf != BUF_TMP2) {
#pragma unroll
        for (int k = 0; k < IT; k++) v1[k] = (v1[k] & 0xFFFFFFFFull) | (v2[k] << 32);
      }
      lds_barrier();
#pragma unroll
      for (int k = 0; k < IT; k++)
        if (valid(k)) L.sval[pos[k]] = v1[k];
      lds_barrier();
      char* out = desc->cols[1].base[P.dst];
#pragma unroll
      for (int i = 0; i < IT; i++) {
        const int j = i * NT + (int)threadIdx.x;
        if (j < cnt) stw<8>(out + ((int64_t)j + L.gdst[dout[i]]) * 8, L.sval[j]);
      }
    } else {
      for (int c = 1; c < ncols; c += 2) {
        move_col(c, v1);
        if (c + 1 < ncols) move_col(c + 1, v2);
      }
    }
  } else {
    for (int c = 1; c < ncols; c++) move_col(c, v1);
  }
  STAMP();  // 5: all stores issued (and, in stamp builds, drained)
  STAMP_FLUSH(0);
}

// One tile per workgroup (XCD-aware order).
template <typename KT, typename U, int LUT, bool CZ, bool PRE3>
__global__ __launch_bounds__(kScatterThreads, SRS_SCATTER_WAVES_PER_EU) void scatter_kernel(
    const SortDesc* __restrict__ desc, const SegPlan* __restrict__ plan,
    const int32_t* __restrict__ tile_seg, const uint64_t* __restrict__ offs,
    const uint32_t* __restrict__ offs32, const GTile* __restrict__ gt) {
  __shared__ ScatterLds<LUT> L;
  __shared__ alignas(16) uint16_t slut[kLutLdsEntries<LUT>];
  const int64_t t = xcd_remap(blockIdx.x, gridDim.x);
  const int ncols = desc->ncols;
  uint64_t v0[kScatterItems], v1[kScatterItems], v2[kScatterItems];
  int64_t my_off;
  const TileInfo ti = scatter_load_tile<KT, U, PRE3>(desc, plan, tile_seg, offs, offs32, gt, t,
                                                     ncols, v0, v1, v2, my_off);
  if (ti.cnt == 0) return;
  // (the table is published by the barrier at the top of the tile)
  const DigitLut lut = stage_lut<LUT, kScatterThreads>(desc, slut);
  scatter_process_tile<KT, U, LUT, CZ, PRE3>(desc, plan, L, ti, ncols, v0, v1, v2, my_off, lut,
                                             offs, offs32);
}

// ---------------------------------------------------------------------------
// scatter of two count tiles per workgroup ("tile pairs", 8192 records)
// ---------------------------------------------------------------------------
// The scatter's cost follows the number of partially written 64-byte blocks
// (the runs per digit and tile, not the bytes). Two
// consecutive count tiles of one segment ranked together write each
// bucket's run per workgroup twice as long: C2's 4-byte keys 64-byte runs
// instead of 32, its payload words 128 instead of 64. The count pass and
// the scans are unchanged: tile b's offsets are tile a's plus a's counts, so
// ranking a's records before b's (waves 0-3 hold tile a, waves 4-7 tile b)
// and adding tile a's offsets gives the same stable result. 512 threads x 16
// records; the LDS holds one 8-byte slot per record (the 4-byte keys use
// half of it), 8 per-wave counter rows and the bucket bases: 79 KB with the
// small digit table, two workgroups per CU. 8-byte keys recompute each
// slot's digit from the staged key; 4-byte keys stage it in the half of the
// slot area they leave free. Columns: the key plus one column, or the key
// plus C2's pair word (SortDesc::pair).
constexpr int kPairThreads = 512;
constexpr int kPairItems = 16;
constexpr int kPairTile = 2 * kTile;
static_assert(kPairThreads * kPairItems == kPairTile, "tile pair shape");
static_assert(kPairThreads >= kMaxBins, "the pair scan gives one bin per thread");

struct PairLds {
  uint64_t sval[kPairTile];
  alignas(8) uint16_t wc[kPairThreads / 64][kMaxBins];
  uint16_t bin_start[kMaxBins];  // tile-pair offsets <= 8192 fit 16 bits
  int64_t gdst[kMaxBins];
  uint32_t scan_sh[kPairThreads / 64 + 1];
};

// a strip of IT slots into registers of type T (load_strip's layout)
template <int IT, typename T>
__device__ __forceinline__ void load_strip_t(T (&dst)[IT], const char* src, uint32_t w,
                                             uint32_t st, int64_t first, int ebase, int cnt) {
  uint64_t tmp[IT];
  load_strip<IT>(tmp, src, w, st, first, ebase, cnt);
#pragma unroll
  for (int k = 0; k < IT; k++) dst[k] = (T)tmp[k];
}

template <typename KT, typename U, int LUT>
__device__ __forceinline__ void scatter_pair_tiles(
    const SortDesc* __restrict__ desc, const SegPlan* __restrict__ plan, PairLds& L,
    const int32_t* __restrict__ tile_seg, const uint64_t* __restrict__ offs,
    const uint32_t* __restrict__ offs32, const GTile* __restrict__ gt, int64_t ta, int64_t tb,
    const DigitLut& lut) {
  constexpr int NT = kPairThreads;
  constexpr int IT = kPairItems;
  constexpr int NW = NT / 64;
  constexpr int KW = sizeof(KT) >= 8 ? 8 : 4;  // (key register width)
  typedef typename std::conditional<KW == 8, uint64_t, uint32_t>::type KR;
  const SegPlan P = plan[tile_seg[ta]];
  int64_t base[2] = {0, 0};
  int cnt[2] = {0, 0};
  for (int h = 0; h < 2; h++) {
    const int64_t t = h ? tb : ta;
    if (t < 0) continue;
    if (gt) {
      base[h] = gt[t].src;
      cnt[h] = gt[t].cnt;
    } else {
      const int64_t tl = t - P.tile_base;
      base[h] = P.start + tl * kTile;
      const int64_t rem = P.len - tl * kTile;
      cnt[h] = P.skip ? 0 : (int)std::min<int64_t>(rem, kTile);
    }
  }
  const int total = cnt[0] + cnt[1];
  if (total == 0) return;
  const uint32_t wave = threadIdx.x >> 6;
  const int half = (int)(wave >> 2);
  const int64_t mybase = half ? base[1] : base[0];
  const int mycnt = half ? cnt[1] : cnt[0];
  const int ebase = (int)(wave & 3) * IT * 64 + (int)lane_id();
  const int ncols = desc->ncols;
  const bool pair = desc->pair != 0;
  const bool pair_src = pair && (P.buf == BUF_TMP || P.buf == BUF_TMP2);

  // loads: the key column, then the payload column (or the pair word)
  KR v0[IT];
  uint64_t v1[IT];
  load_strip_t<IT>(v0, desc->cols[0].base[P.buf], desc->cols[0].width,
                   desc->cols[0].stride[P.buf], mybase, ebase, mycnt);
  if (ncols > 1)
    load_strip<IT>(v1, desc->cols[1].base[P.buf], pair_src ? 8u : desc->cols[1].width,
                   desc->cols[1].stride[P.buf], mybase, ebase, mycnt);
  if (pair && !pair_src) {  // two 4-byte columns from the caller's arrays: joined here
    uint32_t v2[IT];
    load_strip_t<IT>(v2, desc->cols[2].base[P.buf], 4u, desc->cols[2].stride[P.buf], mybase,
                     ebase, mycnt);
#pragma unroll
    for (int k = 0; k < IT; k++) v1[k] = (v1[k] & 0xFFFFFFFFull) | ((uint64_t)v2[k] << 32);
  }
  int64_t my_off = 0;
  const uint32_t nb = 1u << P.bits;
  if (threadIdx.x < nb)
    my_off = offs32 ? (int64_t)offs32[ta * kMaxBins + threadIdx.x]
                    : (int64_t)offs[ta * kMaxBins + threadIdx.x];

  const uint32_t mask = nb - 1;
  Xform<U, false> xf;
  xf.init(*desc);
  const int kbytes = desc->key_bits >> 3;
  const U kmask = kbytes >= (int)sizeof(U) ? (U)~(U)0 : (U)(((uint64_t)1 << (8 * kbytes)) - 1);
#pragma unroll
  for (int i = 0; i < kMaxBins / 256; i++)
    ((uint64_t*)&L.wc[wave][0])[i * 64 + lane_id()] = 0;
  auto valid = [&](int k) -> bool { return ebase + k * 64 < mycnt; };
  uint32_t dg[IT];
#pragma unroll
  for (int k = 0; k < IT; k++) dg[k] = pass_digit<LUT>(xf((U)v0[k] & kmask), P.shift, mask, lut);
  uint32_t pos[IT];
  wlms_rank_fn<IT, kMaxDigitBits, true>([&](int k) { return dg[k]; }, valid, P.bits,
                                        &L.wc[wave][0], pos);
  lds_barrier();
  {  // per-bin totals over the waves (tile a's waves first) -> wave offsets; scan
    const uint32_t my_bin = threadIdx.x;
    uint32_t tsum = 0;
    if (my_bin < nb) {
#pragma unroll
      for (int w = 0; w < NW; w++) {
        const uint32_t c = L.wc[w][my_bin];
        L.wc[w][my_bin] = (uint16_t)tsum;
        tsum += c;
      }
    }
    const uint32_t ex = block_excl_scan_1b<NT>(tsum, L.scan_sh);
    if (my_bin < nb) {
      L.bin_start[my_bin] = (uint16_t)ex;
      L.gdst[my_bin] = P.start + my_off - (int64_t)ex;
    }
  }
  lds_barrier();
  KR* skey = (KR*)L.sval;
  // 4-byte keys fill half of the slot area: the other half holds each slot's
  // digit (no table lookup again at the stores; the word column overwrites
  // both afterwards)
  uint16_t* sdig = (uint16_t*)((char*)L.sval + (size_t)kPairTile * 4);
#pragma unroll
  for (int k = 0; k < IT; k++)
    if (valid(k)) {
      const uint32_t d = dg[k];
      pos[k] = L.bin_start[d] + L.wc[wave][d] + pos[k];
      skey[pos[k]] = v0[k];
      if constexpr (KW == 4) sdig[pos[k]] = (uint16_t)d;
    }
  lds_barrier();
  // the key column: slot j's bucket from its staged key
  uint16_t dout[IT];
  {
    char* out = desc->cols[0].base[P.dst];
    const uint32_t st = desc->cols[0].stride[P.dst];
    with_width(desc->cols[0].width, [&](auto W_) {
#pragma unroll
      for (int i = 0; i < IT; i++) {
        const int j = i * NT + (int)threadIdx.x;
        dout[i] = 0;
        if (j < total) {
          const KR x = skey[j];
          uint32_t d;
          if constexpr (KW == 4) d = sdig[j];
          else d = pass_digit<LUT>(xf((U)x & kmask), P.shift, mask, lut);
          dout[i] = (uint16_t)d;
          stw<decltype(W_)::value>(out + ((int64_t)j + L.gdst[d]) * (int64_t)st, (uint64_t)x);
        }
      }
    });
  }
  if (ncols < 2) return;
  lds_barrier();  // every key slot has been read
#pragma unroll
  for (int k = 0; k < IT; k++)
    if (valid(k)) L.sval[pos[k]] = v1[k];
  lds_barrier();
  {
    char* out = desc->cols[1].base[P.dst];
    const bool pair_dst = pair && (P.dst == BUF_TMP || P.dst == BUF_TMP2);
    const uint32_t w1 = pair_dst ? 8u : desc->cols[1].width;
    const uint32_t st = pair_dst ? 8u : desc->cols[1].stride[P.dst];
    with_width(w1, [&](auto W_) {
#pragma unroll
      for (int i = 0; i < IT; i++) {
        const int j = i * NT + (int)threadIdx.x;
        if (j < total)
          stw<decltype(W_)::value>(out + ((int64_t)j + L.gdst[dout[i]]) * (int64_t)st, L.sval[j]);
      }
    });
  }
}

// One pair of count tiles (2w, 2w + 1) per workgroup, XCD-aware order; a
// pair that straddles two segments is scattered as two single tiles.
template <typename KT, typename U, int LUT>
__global__ __launch_bounds__(kPairThreads, 4) void scatter_pair_kernel(
    const SortDesc* __restrict__ desc, const SegPlan* __restrict__ plan,
    const int32_t* __restrict__ tile_seg, const uint64_t* __restrict__ offs,
    const uint32_t* __restrict__ offs32, const GTile* __restrict__ gt, int64_t ntiles) {
  __shared__ PairLds L;
  __shared__ alignas(16) uint16_t slut[kLutLdsEntries<LUT>];
  const int64_t ta = 2 * xcd_remap(blockIdx.x, gridDim.x);
  const int64_t tb = ta + 1;
  const DigitLut lut = stage_lut<LUT, kPairThreads>(desc, slut);
  if (LUT) lds_barrier();  // publishes the staged digit table
  if (tb < ntiles && tile_seg[tb] == tile_seg[ta]) {
    scatter_pair_tiles<KT, U, LUT>(desc, plan, L, tile_seg, offs, offs32, gt, ta, tb, lut);
  } else {
    scatter_pair_tiles<KT, U, LUT>(desc, plan, L, tile_seg, offs, offs32, gt, ta, -1, lut);
    if (tb < ntiles) {
      lds_barrier();  // (the first tile's slots have all been read)
      scatter_pair_tiles<KT, U, LUT>(desc, plan, L, tile_seg, offs, offs32, gt, tb, -1, lut);
    }
  }
}

// ---------------------------------------------------------------------------
// local: one workgroup sorts one segment (<= CAP keys) in LDS
// ---------------------------------------------------------------------------
// Finishes the recursion for a segment that fits in LDS (the reference's
// leaf, CmpSorterInsertionSort radixSort.hpp:159-178, plus every bit level
// below it):
//   1. keys and the first two columns are loaded once, coalesced;
//   2. bucket pass on the top kLocalBits varying bits with LDS atomics
//      (order inside a bucket is arbitrary here);
//   3. if every bucket holds <= kRankSortMax keys: each key's final slot is
//      bucket start + #(keys in its bucket ordered before it by
//      (key, original index)) -> a stable order, computed in lockstep over
//      the bucket so that LDS reads overlap;
//      otherwise (skewed data): stable LSD digit passes (ballot ranks) over
//      all varying bits;
//   4. every column is staged in LDS in input order and written in output
//      order: coalesced both ways, and safe in place.
constexpr int kLocalBits = 9;      // digit of the LSD fallback passes
#ifndef SRS_LOCAL_TOP_BITS
#define SRS_LOCAL_TOP_BITS 11
#endif
constexpr int kLocalTopBits = SRS_LOCAL_TOP_BITS;  // bucket digit of the fast local kernel
constexpr int kLocalStableTopBits = 10;            // bucket digit of the stable fallback
constexpr int kRankSortMax = 64;   // largest bucket the rank step takes

// Stable ballot-ranked digit pass (fallback path): writes (u, id) in digit
// order to su / sidx.
template <int NT, int IT, typename U>
__device__ __forceinline__ void local_digit_pass(
    const U (&u)[IT], const uint32_t (&id)[IT], const bool (&valid)[IT], int sh, int nbits,
    U* su, uint16_t* sidx, uint16_t (*wc)[1 << kLocalBits], uint32_t* bin_start,
    uint32_t* scan_sh) {
  constexpr int NW = NT / 64;
  constexpr int BPT = (1 << kLocalBits) >= NT ? (1 << kLocalBits) / NT : 1;  // bins per thread
  static_assert(BPT * NT >= (1 << kLocalBits), "bins per thread");
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t nb = 1u << nbits, mask = nb - 1;
  for (uint32_t i = threadIdx.x; i < (uint32_t)(NW << kLocalBits); i += NT) (&wc[0][0])[i] = 0;
  uint32_t dig[IT];
#pragma unroll
  for (int k = 0; k < IT; k++) dig[k] = (uint32_t)(u[k] >> sh) & mask;
  lds_barrier();
  uint32_t rank[IT];
  wlms_rank<IT>(dig, valid, nbits, &wc[wave][0], rank);
  lds_barrier();
  {
    uint32_t tb[BPT], tsum = 0;
#pragma unroll
    for (int q = 0; q < BPT; q++) {
      const uint32_t b = threadIdx.x * BPT + q;
      tb[q] = 0;
      if (b < nb) {
#pragma unroll
        for (int w = 0; w < NW; w++) {
          const uint32_t c = wc[w][b];
          wc[w][b] = (uint16_t)tb[q];
          tb[q] += c;
        }
      }
      tsum += tb[q];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan_lds<NT>(tsum, scan_sh, &tot);
#pragma unroll
    for (int q = 0; q < BPT; q++) {
      const uint32_t b = threadIdx.x * BPT + q;
      if (b < nb) bin_start[b] = ex;
      ex += tb[q];
    }
  }
  lds_barrier();
#pragma unroll
  for (int k = 0; k < IT; k++) {
    if (valid[k]) {
      const uint32_t p = bin_start[dig[k]] + wc[wave][dig[k]] + rank[k];
      su[p] = u[k];
      sidx[p] = (uint16_t)id[k];
    }
  }
  lds_barrier();
}

// Fast path: bucket pass with LDS atomics (order inside a bucket arbitrary);
// the rank step then restores the stable order from the packed
// (key bits, original index) words.
// TB: the atomic bucket pass's digit bits (the exact pass keeps
// kLocalTopBits). The small sorts take one or two more: a whole small sort of
// full-range 64-bit keys then packs (the 52 / 51 key bits below a 12 / 13-bit
// digit, index) into a word, where 11 bits left it to the stable kernel at
// twice the time
template <int NT, int IT, int TB = kLocalTopBits>
struct FastLds {
  // sbuf: packed sort words (+ rank sentinels) during the sort, column
  // staging afterwards
  // (field order: the layout the compiler gave the former separate
  // __shared__ arrays)
  uint64_t sbuf[NT * IT + kRankSortMax];
  uint16_t perm[NT * IT];                      // output slot -> original index
  uint16_t bin_start[(1 << TB) + 2];
  int maxlen;
  unsigned long long wor[NT / 64];             // varying-bit OR, one slot per wave (wave_or)
  uint32_t hist2[(1 << TB) / 2];               // 16-bit bucket sizes, then cursors (pairs)
  uint32_t scan_sh[NT / 64 + 1];
};

// One segment g (<= NT * IT records) by one workgroup. Returns true when the
// segment goes to the stable path instead (nothing written to global memory
// then); block-uniform.
// bail() runs (every thread) right where the segment is handed over: the
// grid kernel appends it to its fallback list there.
template <typename KT, typename U, int NT, int IT, bool CZ, bool REC16 = false, typename Bail,
          int TB>
__device__ __forceinline__ bool local_fast_body(const SortDesc* __restrict__ desc, const Seg g,
                                                FastLds<NT, IT, TB>& Ls, Bail bail) {
  constexpr int NW = NT / 64;
  constexpr int CAP = NT * IT;
  constexpr int IDXB = CAP <= 4096 ? 12 : 13;  // bits of an index inside the segment
  static_assert((1 << IDXB) >= CAP, "index bits");
  static_assert(TB >= kLocalTopBits, "the exact pass's counters live in the bucket arrays' shape");
  constexpr int NB = 1 << TB;
  constexpr int BPT = NB / NT;  // bins per thread (an even count: packed pairs)
  static_assert(BPT * NT == NB && BPT % 2 == 0, "bins per thread");
  static_assert(CAP < 65536, "16-bit bucket counters");
  auto& sbuf = Ls.sbuf;
  auto& perm = Ls.perm;
  auto& hist2 = Ls.hist2;
  auto& bin_start = Ls.bin_start;
  auto& scan_sh = Ls.scan_sh;
  auto& maxlen = Ls.maxlen;
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
  const int ebase = (int)wave * IT * 64 + (int)lane;  // element of slot k: ebase + 64 k
  Xform<U, CZ> xf;
  xf.init(*desc);
  const int cnt = (int)g.len;
  const int64_t base = g.start;
  const int ncols = desc->ncols;
  const int kbytes = desc->key_bits >> 3;
  const uint64_t kmask = kbytes == 8 ? ~0ull : ((1ull << (8 * kbytes)) - 1);
  STAMP_DECL
  STAMP();

  if (threadIdx.x == 0) maxlen = 0;  // (first used after several barriers)
  for (uint32_t i = threadIdx.x; i < (uint32_t)(NB / 2); i += NT) hist2[i] = 0;

  // ---- 1. keys (column 0 holds the key in its low bytes) -------------------
  uint64_t v0[IT];
  load_strip<IT>(v0, desc->cols[0].base[g.buf], desc->cols[0].width,
                 desc->cols[0].stride[g.buf], base, ebase, cnt);
  const U uref = xf((U)(load_w(desc->cols[0].base[g.buf] +
                                   base * (int64_t)desc->cols[0].stride[g.buf],
                               desc->cols[0].width) & kmask));
  // keys are recomputed from v0 when needed (holding them costs occupancy)
  auto ukey = [&](int k) -> U { return xf((U)(v0[k] & kmask)); };
  auto valid = [&](int k) -> bool { return ebase + k * 64 < cnt; };
  auto load_col = [&](int c, uint64_t (&dst)[IT]) {
    load_strip<IT>(dst, desc->cols[c].base[g.buf], desc->cols[c].width,
                   desc->cols[c].stride[g.buf], base, ebase, cnt);
  };
  auto load_col_dense = [&](int c, uint64_t (&dst)[IT]) {  // SoA (DIRECT path)
    load_strip<IT, true>(dst, desc->cols[c].base[g.buf], desc->cols[c].width,
                         desc->cols[c].stride[g.buf], base, ebase, cnt);
  };
  uint64_t vn[IT];
  U vor = 0;
#pragma unroll
  for (int k = 0; k < IT; k++)
    if (valid(k)) vor |= ukey(k) ^ uref;
  STAMP();  // 1: keys loaded
  wave_or_add(Ls.wor, wave, lane, (unsigned long long)vor);
  STAMP();  // (diag) or reduced
  lds_barrier();
  STAMP();  // (diag) barrier passed
  const unsigned long long var = wave_or_read(Ls.wor);
  STAMP();  // (diag) var

  if (var != 0) {
    const int lo = __ffsll((long long)var) - 1;
    const int hi = 63 - __clzll((long long)var);
    const bool exact = hi - lo + 1 <= kLocalTopBits;
    const int nbits = (hi - lo + 1) < TB ? (hi - lo + 1) : TB;
    const int sh = hi - nbits + 1;
    // The sort word packs (key bits 0..hi, original index) when that fits
    // in 64 bits. Wide segments (hi+1+IDXB > 64: mid-size sorts of 64-bit
    // keys) pack only the bits lo..sh-1 below the bucket digit (equal inside
    // a bucket) and rank element-mapped with a masked loop; wider still goes
    // to the stable kernel.
    const bool wide = !exact && hi + 1 + IDXB > 64;
    // (too wide for a rank word: the stable kernel takes it, unless the
    // CmpSorterNoSort leaves need no rank, decided after the bucket pass)
    const bool too_wide = wide && sh - lo + IDXB > 64;
    if (too_wide && desc->leaf_skip == 0) {
      bail();
      return true;
    }
    const uint64_t below = (sh - lo >= 64) ? ~0ull : ((1ull << (sh - lo)) - 1);
    const uint32_t mask = (1u << nbits) - 1;
    const uint64_t keep = (hi == 63) ? ~0ull : ((1ull << (hi + 1)) - 1);
    if (exact) {
      // ---- exact: the digit covers every varying bit, so a bucket holds one
      // key value and a STABLE bucket pass (ballot ranks, input order inside
      // a bucket) is the final order. Duplicate-heavy data (C2's floats) lands
      // here; no bucket-size limit. Per-wave counters [NW][nb] live in sbuf.
      constexpr bool kWcFits =
          NW * (1 << kLocalTopBits) * sizeof(uint16_t) <= CAP * sizeof(uint64_t);
      if constexpr (!kWcFits) {  // (tuning shapes only) the stable kernel takes it
        bail();
        return true;
      }
      uint16_t* wc = (uint16_t*)sbuf;
      const uint32_t nb = kWcFits ? 1u << nbits : 1u;
      for (uint32_t i = threadIdx.x; i < NW * nb / 2; i += NT) ((uint32_t*)wc)[i] = 0;
      auto digit = [&](int k) -> uint32_t { return (uint32_t)(ukey(k) >> lo) & mask; };
      lds_barrier();
      uint32_t rank[IT];
      wlms_rank_fn<IT, kLocalTopBits>(digit, valid, nbits, &wc[wave * nb], rank);
      lds_barrier();
      {
        uint32_t tb[BPT], tsum = 0;
#pragma unroll
        for (int q = 0; q < BPT; q++) {
          const uint32_t b = threadIdx.x * BPT + q;
          tb[q] = 0;
          if (b < nb) {
            for (int w = 0; w < NW; w++) {
              const uint32_t c = wc[w * nb + b];
              wc[w * nb + b] = (uint16_t)tb[q];
              tb[q] += c;
            }
          }
          tsum += tb[q];
        }
        uint32_t tot;
        uint32_t ex = block_excl_scan_1b<NT>(tsum, scan_sh, &tot);
#pragma unroll
        for (int q = 0; q < BPT; q++) {
          const uint32_t b = threadIdx.x * BPT + q;
          if (b < nb) bin_start[b] = (uint16_t)ex;
          ex += tb[q];
        }
      }
      lds_barrier();
#pragma unroll
      for (int k = 0; k < IT; k++) {
        if (valid(k)) {
          const uint32_t d = digit(k);
          perm[bin_start[d] + wc[wave * nb + d] + rank[k]] = (uint16_t)(ebase + k * 64);
        }
      }
      lds_barrier();
      STAMP();  // 2: stable bucket pass
      STAMP();
      STAMP();
    } else {
    // DIRECT: column 0 is exactly the key and the sort word holds every key
    // bit that varies, so the sorted keys are rebuilt from the words (no
    // staging pass and one barrier fewer for column 0; C1 local 6.88 -> 6.62
    // ms). Column 1's loads go out right after the rank (issuing them before
    // it, in the registers v0 frees, forces the rank into quarters: slower).
    // (SoA only: for AoS records the key slice's stores run ahead of the
    // other slices' and C3 measured 11 % slower)
    // (SoA columns are dense in every buffer: the DIRECT code has no strided
    // load or store path)
    const bool direct = !CZ && !wide && desc->cols[0].width == (uint32_t)kbytes &&
                        desc->cols[0].stride[BUF_OUT] == (uint32_t)kbytes &&
                        (!desc->tmp2 || desc->pair ||
                         desc->cols[0].stride[BUF_TMP2] == (uint32_t)kbytes) &&
                        desc->cols[0].stride[BUF_IN] == (uint32_t)kbytes;
    auto bucket_rank = [&](auto DIRECT_) -> bool {
    constexpr bool DIRECT = decltype(DIRECT_)::value;
    STAMP();  // (diag) direct decided
    // ---- 2. bucket pass on the top varying bits (LDS atomics on 16-bit
    // counters packed in pairs: 2^11 buckets in the LDS of 2^10 u32 ones) ----
#pragma unroll
    for (int k = 0; k < IT; k++) {
      if (valid(k)) {
        const uint32_t d = (uint32_t)(ukey(k) >> sh) & mask;
        atomicAdd(&hist2[d >> 1], 1u << ((d & 1) << 4));
      }
    }
    STAMP();  // (diag) atomics issued
    lds_barrier();
    STAMP();  // (diag) barrier
    {
      uint32_t tb[BPT], tsum = 0;
#pragma unroll
      for (int q = 0; q < BPT; q += 2) {
        const uint32_t w2 = hist2[(threadIdx.x * BPT + q) >> 1];
        tb[q] = w2 & 0xFFFFu;
        tb[q + 1] = w2 >> 16;
        tsum += tb[q] + tb[q + 1];
      }
      uint32_t tot;
      uint32_t ex = block_excl_scan_1b<NT>(tsum, scan_sh, &tot);
      STAMP();  // (diag) scanned
      int mymax = 0;
#pragma unroll
      for (int q = 0; q < BPT; q += 2) {
        const uint32_t b = threadIdx.x * BPT + q;
        const uint32_t e0 = ex, e1 = ex + tb[q];
        bin_start[b] = (uint16_t)e0;
        bin_start[b + 1] = (uint16_t)e1;
        hist2[b >> 1] = e0 | (e1 << 16);  // insertion cursors
        ex = e1 + tb[q + 1];
        mymax = max(mymax, (int)max(tb[q], tb[q + 1]));
      }
      if (threadIdx.x == 0) bin_start[NB] = (uint16_t)tot;
      block_max_into(&maxlen, mymax);
    }
    lds_barrier();
    STAMP();  // 2: bucket histogram
    // CmpSorterNoSort: when every bucket (a node of the reference's bit
    // recursion, all keys sharing the bits above sh) holds <= leaf_skip keys,
    // the buckets are the leaves and stay in bucket-pass order
    const bool skip_rank = maxlen <= desc->leaf_skip;
    if ((maxlen > kRankSortMax || too_wide) && !skip_rank) {
      // a large bucket (duplicates or skew): local_stable_kernel takes the
      // segment (nothing has been written to global memory yet)
      bail();
      return true;
    }
#pragma unroll
    for (int k = 0; k < IT; k++) {
      if (valid(k)) {
        const U uk = ukey(k);
        const uint32_t d = (uint32_t)(uk >> sh) & mask;
        const uint32_t hs = (d & 1) << 4;
        const uint32_t p = (atomicAdd(&hist2[d >> 1], 1u << hs) >> hs) & 0xFFFFu;
        const uint64_t kw = wide ? (((uint64_t)uk >> lo) & below) : ((uint64_t)uk & keep);
        sbuf[p] = (kw << IDXB) | (uint64_t)(ebase + k * 64);
      }
    }
    if (threadIdx.x < (uint32_t)kRankSortMax) sbuf[cnt + threadIdx.x] = ~0ull;  // sentinels
    lds_barrier();
    STAMP();  // 3: bucket scatter
    if (skip_rank) {  // the leaves unsorted: output slot p takes word p
      for (int p = (int)threadIdx.x; p < cnt; p += NT)
        perm[p] = DIRECT ? (uint16_t)p : (uint16_t)(sbuf[p] & ((1u << IDXB) - 1));
      lds_barrier();
      return false;
    }
    // ---- 3. rank inside each bucket: #(words of the bucket below mine) ----
    // The word orders by (key, original index), so the result is stable.
    // Slots in two halves bound register use; a wave-uniform trip count
    // keeps several LDS reads in flight.
    constexpr int NH = SRS_LOCAL_RANK_SPLIT;
    constexpr int H = IT / NH;
    if (DIRECT || !wide) {
#pragma unroll
    for (int half = 0; half < NH; half++) {
      uint64_t x[H];
      uint32_t bs[H], bl[H], r[H];
      int wmax = 0;
#pragma unroll
      for (int i = 0; i < H; i++) {
        const int p = (half * H + i) * NT + (int)threadIdx.x;
        bl[i] = 0;
        bs[i] = 0;
        x[i] = 0;
        r[i] = 0;
        if (p < cnt) {
          x[i] = sbuf[p];
          const uint32_t d = (uint32_t)(x[i] >> (sh + IDXB)) & mask;
          bs[i] = bin_start[d];
          bl[i] = bin_start[d + 1] - bs[i];
          wmax = (int)bl[i] > wmax ? (int)bl[i] : wmax;
        }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const int t2 = __shfl_xor(wmax, o, 64);
        wmax = t2 > wmax ? t2 : wmax;
      }
      // Branch-free and unmasked: sbuf is in bucket order, so a word read
      // past the end of my bucket belongs to a higher bucket (a larger key)
      // or is a ~0 sentinel (slots [cnt, cnt + kRankSortMax)); neither is
      // below x. The H reads of a step issue back to back under one wait.
      for (int j = 0; j < wmax; j++) {
        uint64_t w[H];
#pragma unroll
        for (int i = 0; i < H; i++) w[i] = sbuf[bs[i] + (uint32_t)j];
#pragma unroll
        for (int i = 0; i < H; i++) r[i] += w[i] < x[i];
      }
#pragma unroll
      for (int i = 0; i < H; i++) {
        const int p = (half * H + i) * NT + (int)threadIdx.x;
        if (p < cnt)  // DIRECT: the word's slot (its key and index are in the word)
          perm[bs[i] + r[i]] = DIRECT ? (uint16_t)p : (uint16_t)(x[i] & ((1u << IDXB) - 1));
      }
    }
    } else {
      // element-mapped: my own keys, their buckets recomputed; words past a
      // bucket's end are not ordered against mine, so the loop is masked
#pragma unroll
      for (int half = 0; half < NH; half++) {
        uint64_t x[H];
        uint32_t bs[H], bl[H], r[H];
        int wmax = 0;
#pragma unroll
        for (int i = 0; i < H; i++) {
          const int k = half * H + i;
          bl[i] = 0;
          bs[i] = 0;
          x[i] = 0;
          r[i] = 0;
          if (valid(k)) {
            const U uk = ukey(k);
            const uint32_t d = (uint32_t)(uk >> sh) & mask;
            x[i] = ((((uint64_t)uk >> lo) & below) << IDXB) | (uint64_t)(ebase + k * 64);
            bs[i] = bin_start[d];
            bl[i] = bin_start[d + 1] - bs[i];
            wmax = (int)bl[i] > wmax ? (int)bl[i] : wmax;
          }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
          const int t2 = __shfl_xor(wmax, o, 64);
          wmax = t2 > wmax ? t2 : wmax;
        }
        for (int j = 0; j < wmax; j++) {
          uint64_t w[H];
#pragma unroll
          for (int i = 0; i < H; i++) w[i] = sbuf[bs[i] + (uint32_t)j];  // < CAP + kRankSortMax
#pragma unroll
          for (int i = 0; i < H; i++) r[i] += ((uint32_t)j < bl[i]) & (w[i] < x[i]);
        }
#pragma unroll
        for (int i = 0; i < H; i++)
          if (valid(half * H + i)) perm[bs[i] + r[i]] = (uint16_t)(ebase + (half * H + i) * 64);
      }
    }
    lds_barrier();
    STAMP();  // 4: ranked
    return false;
    };  // bucket_rank
    if (direct) {
      if (bucket_rank(std::true_type{})) return true;
      // ---- 4'. column 0 from the words; the rank left each output slot's
      // word slot in perm. u = known top bits | word bits, then the inverse
      // key transform. The other columns staged, written in order. FW: the
      // payload width as a compile-time fact for the common one-column case.
      // FW: the payload width when there is exactly one payload column (0:
      // any columns, staged one by one; -1: desc->pair's two 4-byte payloads
      // read as one 8-byte word column from TMP / TMP2)
      auto direct_out = [&](auto FW_) {
        constexpr int FW = decltype(FW_)::value;
        if (ncols > 1) {
          if constexpr (FW > 0) load_strip<IT, true, FW>(vn, desc->cols[1].base[g.buf], FW, FW,
                                                         base, ebase, cnt);
          else if constexpr (FW < 0) load_strip<IT, true, 8>(vn, desc->cols[1].base[g.buf], 8, 8,
                                                             base, ebase, cnt);
          else load_col_dense(1, vn);
        }
        uint32_t id[IT];
        const uint64_t top = (uint64_t)uref & ~keep;
        const uint64_t imask = (1u << IDXB) - 1;
        // (column 0 is the key column: its width is sizeof(KT))
        store_strip<IT, true, (int)sizeof(KT)>(desc->cols[0].base[BUF_OUT], desc->cols[0].width,
                              desc->cols[0].stride[BUF_OUT], base, ebase, cnt,
                              [&](int k) -> uint64_t {
                                const int e = ebase + k * 64;
                                const uint64_t w = sbuf[perm[e < cnt ? e : 0]];
                                id[k] = (uint32_t)(w & imask);
                                return (uint64_t)xf.inv((U)(top | (w >> IDXB)));
                              });
        STAMP();  // 5: column 0 moved
        if constexpr (FW != 0) {  // exactly one payload column (or word pair)
          lds_barrier();  // every read of the words is done
#pragma unroll
          for (int k = 0; k < IT; k++)
            if (valid(k)) sbuf[ebase + k * 64] = vn[k];
          lds_barrier();
          if constexpr (FW > 0) {
            store_strip<IT, true, FW>(desc->cols[1].base[BUF_OUT], FW, FW, base, ebase, cnt,
                                      [&](int k) { return sbuf[id[k]]; });
          } else {  // the two halves of each word to their own OUT arrays
            store_strip<IT, true, 4>(desc->cols[1].base[BUF_OUT], 4, 4, base, ebase, cnt,
                                     [&](int k) { return sbuf[id[k]] & 0xFFFFFFFFull; });
            store_strip<IT, true, 4>(desc->cols[2].base[BUF_OUT], 4, 4, base, ebase, cnt,
                                     [&](int k) { return sbuf[id[k]] >> 32; });
          }
        } else {
          // column c is staged straight from vn, whose registers then take
          // column c + 1's loads before column c's stores (no register
          // copies: a copy of in-flight load results costs a vmcnt(0) wait)
          for (int c = 1; c < ncols; c++) {
            lds_barrier();  // every read of sbuf (words, or the previous column) is done
#pragma unroll
            for (int k = 0; k < IT; k++)
              if (valid(k)) sbuf[ebase + k * 64] = vn[k];
            if (c + 1 < ncols) load_col_dense(c + 1, vn);
            lds_barrier();
            store_strip<IT, true>(desc->cols[c].base[BUF_OUT], desc->cols[c].width,
                                  desc->cols[c].stride[BUF_OUT], base, ebase, cnt,
                                  [&](int k) { return sbuf[id[k]]; });
          }
        }
      };
      if (ncols == 2 && desc->cols[1].width == 8) direct_out(std::integral_constant<int, 8>{});
      else if (desc->pair && (g.buf == BUF_TMP || g.buf == BUF_TMP2))
        direct_out(std::integral_constant<int, -1>{});
      else direct_out(std::integral_constant<int, 0>{});
      STAMP();  // 6
      STAMP_FLUSH(1);
      return false;
    }
    if (bucket_rank(std::false_type{})) return true;
    }  // atomic bucket pass + rank
  } else if (g.buf == BUF_OUT) {
    return false;  // all keys equal and already home
  } else {
#pragma unroll
    for (int k = 0; k < IT; k++) perm[ebase + k * 64] = (uint16_t)(ebase + k * 64);
    lds_barrier();
  }
  // ---- 4'. 16-byte records (AoS records of 16 bytes that travelled as two
  // dense 8-byte slice columns through TMP / TMP2, C3): both slices staged in
  // turn, each output slot's key slice held in registers across the second
  // staging, then one 16-byte store per record instead of two 8-byte stores
  // at stride 16 into half-written lines.
  // (an instantiation of its own, REC16: the extra path measurably slowed
  // C1's kernel, 6.43 -> 6.51 ms, when compiled into it)
  if (REC16 && ncols == 2 && desc->tmp2 && !desc->pair &&
      (g.buf == BUF_TMP || g.buf == BUF_TMP2) &&
      desc->cols[0].width == 8 && desc->cols[1].width == 8 &&
      desc->cols[0].stride[BUF_OUT] == 16 && desc->cols[1].stride[BUF_OUT] == 16 &&
      desc->cols[1].base[BUF_OUT] == desc->cols[0].base[BUF_OUT] + 8) {
    load_strip<IT, true, 8>(vn, desc->cols[1].base[g.buf], 8, 8, base, ebase, cnt);
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (valid(k)) sbuf[ebase + k * 64] = v0[k];
    lds_barrier();
    uint64_t ko[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) ko[k] = sbuf[valid(k) ? perm[ebase + k * 64] : 0];
    lds_barrier();
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (valid(k)) sbuf[ebase + k * 64] = vn[k];
    lds_barrier();
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t r = strip_rsrc(desc->cols[0].base[BUF_OUT] + base * 16,
                                                cnt > 0 ? (uint32_t)cnt * 16u : 0u);
#pragma unroll
    for (int k = 0; k < IT; k++) {
      const uint64_t pv = sbuf[valid(k) ? perm[ebase + k * 64] : 0];
      u32x4 x;
      x[0] = (uint32_t)ko[k];
      x[1] = (uint32_t)(ko[k] >> 32);
      x[2] = (uint32_t)pv;
      x[3] = (uint32_t)(pv >> 32);
      __builtin_amdgcn_raw_buffer_store_b128(x, r, (uint32_t)(ebase + k * 64) * 16u, 0, 0);
    }
    STAMP();
    STAMP();
    STAMP_FLUSH(1);
    return false;
  }

  // output slot e takes input element perm[e]
  uint32_t id[IT];
#pragma unroll
  for (int k = 0; k < IT; k++) id[k] = valid(k) ? perm[ebase + k * 64] : 0u;  // store_strip reads every slot

  // ---- 4. columns: stage in input order, write in output order --------------
  // Software-pipelined: column c+1's loads are issued before column c is
  // staged and stored, so their latency hides behind that work. In place is
  // safe: a column's loads complete before the barrier that precedes its own
  // stores, and different columns never share bytes.
  // desc->pair with the segment in TMP / TMP2: columns 1 and 2 are one word
  // column there (one load and staging pass, two half-word store passes)
  const bool pw = desc->pair && (g.buf == BUF_TMP || g.buf == BUF_TMP2);
  if (pw) load_strip<IT>(vn, desc->cols[1].base[g.buf], 8, 8, base, ebase, cnt);
  else if (ncols > 1) load_col(1, vn);
  // column 0 from v0 (the barrier after the perm writes already ordered
  // every earlier sbuf access), then each column c >= 1 staged straight from
  // vn, whose registers take column c + 1's loads before column c's stores
  // (no register copies: a copy of in-flight load results waits vmcnt(0))
#pragma unroll
  for (int k = 0; k < IT; k++)
    if (valid(k)) sbuf[ebase + k * 64] = v0[k];
  lds_barrier();
  store_strip<IT>(desc->cols[0].base[BUF_OUT], desc->cols[0].width,
                  desc->cols[0].stride[BUF_OUT], base, ebase, cnt,
                  [&](int k) { return sbuf[id[k]]; });
  STAMP();  // 5: column 0 moved
  if (pw) {
    lds_barrier();
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (valid(k)) sbuf[ebase + k * 64] = vn[k];
    lds_barrier();
    store_strip<IT>(desc->cols[1].base[BUF_OUT], 4, desc->cols[1].stride[BUF_OUT], base, ebase,
                    cnt, [&](int k) { return sbuf[id[k]] & 0xFFFFFFFFull; });
    store_strip<IT>(desc->cols[2].base[BUF_OUT], 4, desc->cols[2].stride[BUF_OUT], base, ebase,
                    cnt, [&](int k) { return sbuf[id[k]] >> 32; });
  }
  for (int c = pw ? ncols : 1; c < ncols; c++) {
    lds_barrier();
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (valid(k)) sbuf[ebase + k * 64] = vn[k];
    if (c + 1 < ncols) load_col(c + 1, vn);
    lds_barrier();
    store_strip<IT>(desc->cols[c].base[BUF_OUT], desc->cols[c].width,
                    desc->cols[c].stride[BUF_OUT], base, ebase, cnt,
                    [&](int k) { return sbuf[id[k]]; });
  }
  STAMP();  // 6: columns moved
  STAMP_FLUSH(1);
  return false;
}

template <typename KT, typename U, int NT, int IT, int WPE, bool CZ, bool REC16 = false>
__global__ __launch_bounds__(NT, WPE) void local_kernel(const SortDesc* __restrict__ desc,
                                                   const Seg* __restrict__ segs,
                                                   Seg* __restrict__ fallback,
                                                   unsigned long long* fallback_count) {
  __shared__ FastLds<NT, IT> Ls;
  const Seg g = segs[blockIdx.x];
  local_fast_body<KT, U, NT, IT, CZ, REC16>(desc, g, Ls, [&] {
    if (threadIdx.x == 0) fallback[atomicAdd(fallback_count, 1ull)] = g;
  });
}

// The fast kernel over a list whose length is known on device only
// (segments the direct kernel below handed over): grid-stride, so an empty
// list costs a few microseconds.
template <typename KT, typename U, int NT, int IT, int WPE>
__global__ __launch_bounds__(NT, WPE) void local_list_kernel(const SortDesc* __restrict__ desc,
                                                        const Seg* __restrict__ segs,
                                                        const unsigned long long* nsegs,
                                                        Seg* __restrict__ fallback,
                                                        unsigned long long* fallback_count) {
  __shared__ FastLds<NT, IT> Ls;
  const int64_t m = (int64_t)*nsegs;
  for (int64_t i = blockIdx.x; i < m; i += gridDim.x) {
    const Seg g = segs[i];
    local_fast_body<KT, U, NT, IT, false>(desc, g, Ls, [&] {
      if (threadIdx.x == 0) fallback[atomicAdd(fallback_count, 1ull)] = g;
    });
    __syncthreads();  // the next segment reuses the LDS
  }
}

// ---- Direct local kernel (round 3): the common shapes -- a dense 4/8-byte
// key column with one dense 8-byte payload column (C1), a key with a pair of
// 4-byte payloads travelling as one word (C2), 16-byte AoS records travelling
// as two slices (C3); no canon-zero -- at four workgroups of 256 x 16 per CU
// instead of three of 512 x 8.
// The fast kernel's LDS holds the sort words, a u16 permutation (8 KB) and a
// bucket-start table (4 KB) beside the packed bucket counters: 49.5 KB, three
// workgroups per CU. Here every word (key bits lo..hi, index) is written to
// its sorted slot (each thread keeps its 16 words and their slots in
// registers across one barrier), so no permutation table is needed, and the
// key column is rebuilt from the sorted words; the bucket starts are read
// from the advanced insertion cursors (bucket b's cursor ends at the start
// of bucket b + 1; cursor word 0 stays 0): 37.4 KB. 16 items per thread at
// four waves per SIMD leave 128 VGPRs.
//   exact segments (<= kLocalTopBits varying bits, so a bucket is one key
//   value; pair mode only): the stable ballot-ranked bucket pass gives every
//   word its slot;
//   others: the atomic bucket pass, then the rank inside each bucket by word.
// Handed to the fast kernel (`redo`): all keys equal, more than 52 varying
// bits, exact segments outside the pair mode, and (PM 1/2) segments outside
// TMP / TMP2; large buckets of a non-exact segment go to the stable kernel's
// list as from the fast kernel. The host runs this kernel only from
// direct_min_segs() local segments on (srs_api.hip).
// PM (payload mode): 0 one dense 8-byte payload column; 1 AoS 16-byte
// records as two slices in TMP / TMP2, written back as one 16-byte store per
// record; 2 desc->pair's word column (two 4-byte payloads) in TMP / TMP2,
// written to the two OUT arrays.
template <int NT, int IT>
struct DirectLds {
  uint64_t sbuf[NT * IT + kRankSortMax];      // sort words (+ sentinels), then the payloads
  uint32_t cur[(1 << kLocalTopBits) / 2 + 1];  // [0] = 0; bucket b: cur[1 + b/2], half b & 1
  uint32_t scan_sh[NT / 64 + 1];
  unsigned long long wor[NT / 64];  // varying-bit OR, one slot per wave (wave_or_add)
  int maxlen;
};

template <typename KT, typename U, int NT, int IT, int WPE, int PM>
__global__ __launch_bounds__(NT, WPE) void local_direct_kernel(
    const SortDesc* __restrict__ desc, const Seg* __restrict__ segs, Seg* __restrict__ redo,
    unsigned long long* redo_count, Seg* __restrict__ fallback,
    unsigned long long* fallback_count, int xcd) {
  constexpr int CAP = NT * IT;
  constexpr int IDXB = CAP <= 4096 ? 12 : 13;  // bits of an index inside the segment
  static_assert(CAP <= (1 << IDXB) && CAP <= 65536, "index bits, u16 cursors");
  constexpr int NB = 1 << kLocalTopBits;
  constexpr int NW = NT / 64;
  constexpr int BPT = NB / NT;  // bins per thread (an even count: packed pairs)
  static_assert(BPT * NT == NB && BPT % 2 == 0, "bins per thread");
  static_assert(NW * NB * sizeof(uint16_t) <= CAP * sizeof(uint64_t), "per-wave counters");
  constexpr int KB = (int)sizeof(KT);
  static_assert(PM != 1 || KB == 8, "16-byte records: the key slice is the key");
  __shared__ DirectLds<NT, IT> Ls;
  auto& sbuf = Ls.sbuf;
  auto& cur = Ls.cur;
  // (xcd: consecutive list entries on one XCD)
  const Seg g = segs[xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x];
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
  const int ebase = (int)wave * IT * 64 + (int)lane;  // element of slot k: ebase + 64 k
  const int cnt = (int)g.len;
  const int64_t base = g.start;
  auto hand_over = [&](Seg* list, unsigned long long* n) {
    if (threadIdx.x == 0) list[atomicAdd(n, 1ull)] = g;
  };
  if (PM != 0 && g.buf != BUF_TMP && g.buf != BUF_TMP2) {  // (block-uniform)
    hand_over(redo, redo_count);
    return;
  }
  Xform<U, false> xf;
  xf.init(*desc);
  if (threadIdx.x == 0) Ls.maxlen = 0;  // (first used after several barriers)
  for (uint32_t i = threadIdx.x; i < (uint32_t)(NB / 2 + 1); i += NT) cur[i] = 0;

  // ---- 1. keys ---------------------------------------------------------------
  uint64_t v0[IT];
  load_strip<IT, true, KB, SRS_LOCAL_LOAD_AUX>(v0, desc->cols[0].base[g.buf], KB, KB, base, ebase,
                                               cnt);
  const U uref = xf((U)ldw<KB>(desc->cols[0].base[g.buf] + base * KB));
  auto ukey = [&](int k) -> U { return xf((U)v0[k]); };
  auto valid = [&](int k) -> bool { return ebase + k * 64 < cnt; };
  U vor = 0;
#pragma unroll
  for (int k = 0; k < IT; k++)
    if (valid(k)) vor |= ukey(k) ^ uref;
  wave_or_add(Ls.wor, wave, lane, (unsigned long long)vor);
  lds_barrier();
  // (LDS values made provably uniform: everything derived from them then
  // lives in SGPRs, not in the 128 VGPRs)
  const unsigned long long var_l = wave_or_read(Ls.wor);
  const unsigned long long var =
      ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(var_l >> 32))
       << 32) |
      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)var_l);  // (int results: no sign extension)
  const int lo = var ? __ffsll((long long)var) - 1 : 0;
  const int hi = var ? 63 - __clzll((long long)var) : 0;
  const int vbits = hi - lo + 1;
#if SRS_DIRECT_WORD_DIGIT
  // The bucket digit is the top kLocalTopBits bits of the sort word (key bits
  // lo..hi above the 12-bit element index). With more varying key bits than
  // that, these are the top varying key bits; with fewer (an "exact"
  // segment: few distinct values, many copies each) the digit takes the top
  // index bits too, which spreads each value's copies over buckets by input
  // position, so buckets stay small and the rank by word (key, index) is the
  // stable order: no separate exact pass.
  constexpr bool EX = false;
  if (var == 0 || vbits + IDXB > 64) {
    hand_over(redo, redo_count);
    return;
  }
  const bool exact = false;
  const int nbits = kLocalTopBits;
  const int dsh = vbits + IDXB - kLocalTopBits;  // the digit's position in a word
#else
  // (EX: the exact pass is compiled in; it costs the other modes their
  // spill-free 128 VGPRs, and only the pair mode (C2's float keys with ~60
  // copies of each value) meets exact segments in bulk)
  constexpr bool EX = PM == 2;
  if (var == 0 || vbits + IDXB > 64 || (!EX && vbits <= kLocalTopBits)) {
    hand_over(redo, redo_count);
    return;
  }
  const bool exact = vbits <= kLocalTopBits;
  const int nbits = exact ? vbits : kLocalTopBits;
  const int dsh = hi - nbits + 1 - lo + IDXB;  // the digit's position in a word
#endif
  const uint32_t mask = (1u << nbits) - 1;
  const uint64_t vmask = vbits == 64 ? ~0ull : ((1ull << vbits) - 1);
  // sort word: the varying key bits lo..hi above the element index (the bits
  // below lo and above hi are uref's)
  auto word = [&](int k) -> uint64_t {
    return ((((uint64_t)ukey(k) >> lo) & vmask) << IDXB) | (uint64_t)(ebase + k * 64);
  };
  auto digit = [&](int k) -> uint32_t { return (uint32_t)(word(k) >> dsh) & mask; };
  // both paths end with word i of this thread (xs) going to its sorted slot
  // (dst) after one barrier; slot kDump takes the words of empty slots
  constexpr uint32_t kDump = CAP + kRankSortMax - 1;
  uint64_t xs[IT];
  uint32_t dst[IT];
  bool place = true;

  if (EX && exact) {
    // ---- 2e. stable bucket pass (ballot ranks, input order inside a bucket):
    // per-wave counters [NW][nb] in sbuf, bucket starts (u16) in cur; each
    // word then goes straight to its final slot
    // (the words are 32-bit here: vbits <= kLocalTopBits, and the digit is
    // the word's key field; the keys' registers are free from here on)
    uint16_t* wc = (uint16_t*)sbuf;
    uint16_t* bstart = (uint16_t*)cur;
    const uint32_t nb = 1u << nbits;
    uint32_t w32[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) w32[k] = (uint32_t)word(k);
    auto edigit = [&](int k) -> uint32_t { return w32[k] >> IDXB; };
    for (uint32_t i = threadIdx.x; i < NW * nb / 2; i += NT) ((uint32_t*)wc)[i] = 0;
    lds_barrier();
    uint32_t rank[IT];
    wlms_rank_fn<IT, kLocalTopBits>(edigit, valid, nbits, &wc[wave * nb], rank);
    lds_barrier();
    {
      uint32_t tb[BPT], tsum = 0;
#pragma unroll
      for (int q = 0; q < BPT; q++) {
        const uint32_t b = threadIdx.x * BPT + q;
        tb[q] = 0;
        if (b < nb) {
#pragma unroll
          for (int w = 0; w < NW; w++) {
            const uint32_t c = wc[w * nb + b];
            wc[w * nb + b] = (uint16_t)tb[q];
            tb[q] += c;
          }
        }
        tsum += tb[q];
      }
      uint32_t ex = block_excl_scan_1b<NT>(tsum, Ls.scan_sh);
#pragma unroll
      for (int q = 0; q < BPT; q++) {
        const uint32_t b = threadIdx.x * BPT + q;
        if (b < nb) bstart[b] = (uint16_t)ex;
        ex += tb[q];
      }
    }
    lds_barrier();
#pragma unroll
    for (int k = 0; k < IT; k++) {
      dst[k] = valid(k) ? rank[k] + bstart[edigit(k)] + wc[wave * nb + edigit(k)] : kDump;
      xs[k] = w32[k];
    }
  } else {
    // ---- 2. bucket histogram (packed 16-bit counters), insertion cursors ----
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (valid(k)) {
        const uint32_t d = digit(k);
        atomicAdd(&cur[1 + (d >> 1)], 1u << ((d & 1) << 4));
      }
    lds_barrier();
    {
      uint32_t tb[BPT], tsum = 0;
#pragma unroll
      for (int q = 0; q < BPT; q += 2) {
        const uint32_t w2 = cur[1 + ((threadIdx.x * BPT + q) >> 1)];
        tb[q] = w2 & 0xFFFFu;
        tb[q + 1] = w2 >> 16;
        tsum += tb[q] + tb[q + 1];
      }
      uint32_t ex = block_excl_scan_1b<NT>(tsum, Ls.scan_sh);
      int mymax = 0;
#pragma unroll
      for (int q = 0; q < BPT; q += 2) {
        const uint32_t e0 = ex, e1 = ex + tb[q];
        cur[1 + ((threadIdx.x * BPT + q) >> 1)] = e0 | (e1 << 16);
        ex = e1 + tb[q + 1];
        mymax = max(mymax, (int)max(tb[q], tb[q + 1]));
      }
      block_max_into(&Ls.maxlen, mymax);
    }
    lds_barrier();
    const int maxlen = __builtin_amdgcn_readfirstlane(Ls.maxlen);
    // CmpSorterNoSort leaves (see the fast kernel): buckets of <= leaf_skip
    // keys stay in bucket-pass order
    const bool skip_rank = maxlen <= desc->leaf_skip;
    if (maxlen > kRankSortMax && !skip_rank) {  // (block-uniform)
      hand_over(fallback, fallback_count);
      return;
    }
    // ---- 3. bucket scatter of the words ----------------------------------------
#pragma unroll
    for (int k = 0; k < IT; k++) {
      if (valid(k)) {
        const uint32_t d = digit(k);
        const uint32_t hs = (d & 1) << 4;
        const uint32_t p = (atomicAdd(&cur[1 + (d >> 1)], 1u << hs) >> hs) & 0xFFFFu;
        sbuf[p] = word(k);
      }
    }
    if (threadIdx.x < (uint32_t)kRankSortMax) sbuf[cnt + threadIdx.x] = ~0ull;  // sentinels
    lds_barrier();
    // ---- 4. rank inside each bucket, then every word to its sorted slot ------
    place = !skip_rank;
    if (!skip_rank) {
      constexpr int NH = SRS_DIRECT_RANK_SPLIT;
      constexpr int H = IT / NH;
#pragma unroll
      for (int half = 0; half < NH; half++) {
        uint32_t bs[H], r[H];
        int wmax = 0;
#pragma unroll
        for (int i = 0; i < H; i++) {
          const int p = (half * H + i) * NT + (int)threadIdx.x;
          xs[half * H + i] = 0;
          bs[i] = 0;
          r[i] = 0;
          if (p < cnt) {
            const uint64_t x = sbuf[p];
            xs[half * H + i] = x;
            const uint32_t d = (uint32_t)(x >> dsh) & mask;
            const uint32_t i1 = 1 + (d >> 1);
            const uint32_t w0 = cur[i1 - 1], w1 = cur[i1];  // (bucket d - 1's end, d's end)
            const uint32_t s = (d & 1) ? (w1 & 0xFFFFu) : (w0 >> 16);
            const uint32_t e = (d & 1) ? (w1 >> 16) : (w1 & 0xFFFFu);
            bs[i] = s;
            wmax = (int)(e - s) > wmax ? (int)(e - s) : wmax;
          }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
          const int t2 = __shfl_xor(wmax, o, 64);
          wmax = t2 > wmax ? t2 : wmax;
        }
        // (branch-free and unmasked as in the fast kernel: a word past my
        // bucket's end is a larger key or a ~0 sentinel)
        for (int j = 0; j < wmax; j++) {
          uint64_t w[H];
#pragma unroll
          for (int i = 0; i < H; i++) w[i] = sbuf[bs[i] + (uint32_t)j];
#pragma unroll
          for (int i = 0; i < H; i++) r[i] += w[i] < xs[half * H + i];
        }
#pragma unroll
        for (int i = 0; i < H; i++)
          dst[half * H + i] = (half * H + i) * NT + (int)threadIdx.x < cnt ? bs[i] + r[i] : kDump;
      }
    }
  }
  if (place) {  // (block-uniform)
    lds_barrier();  // every read of the counters / bucket-ordered words is done
#pragma unroll
    for (int i = 0; i < IT; i++) sbuf[dst[i]] = xs[i];
  }
  // the payloads (dense 8-byte words in every mode)
  uint64_t vn[IT];
  load_strip<IT, true, 8, SRS_LOCAL_LOAD_AUX>(vn, desc->cols[1].base[g.buf], 8, 8, base, ebase,
                                              cnt);
  lds_barrier();

  // ---- 5. keys rebuilt from the sorted words, payloads staged ----------------
  uint32_t id[IT];
  const uint64_t ubase = (uint64_t)uref & ~(vmask << lo);
  const uint64_t imask = (1u << IDXB) - 1;
  auto key_of = [&](int k) -> uint64_t {
    const uint64_t w = sbuf[ebase + k * 64];  // (< CAP + sentinels; past cnt: dropped)
    id[k] = (uint32_t)(w & imask);
    return (uint64_t)xf.inv((U)(ubase | ((w >> IDXB) << lo)));
  };
  uint64_t ko[IT];
  if constexpr (PM == 1) {
#pragma unroll
    for (int k = 0; k < IT; k++) ko[k] = key_of(k);
  } else {
    store_strip<IT, true, KB>(desc->cols[0].base[BUF_OUT], KB, KB, base, ebase, cnt,
                              [&](int k) { return key_of(k); });
  }
  lds_barrier();  // every read of the words is done
#pragma unroll
  for (int k = 0; k < IT; k++)
    if (valid(k)) sbuf[ebase + k * 64] = vn[k];
  lds_barrier();
  if constexpr (PM == 0) {
    store_strip<IT, true, 8>(desc->cols[1].base[BUF_OUT], 8, 8, base, ebase, cnt,
                             [&](int k) { return sbuf[id[k]]; });
  } else if constexpr (PM == 2) {  // the two halves of each word to their own OUT arrays
    store_strip<IT, true, 4>(desc->cols[1].base[BUF_OUT], 4, 4, base, ebase, cnt,
                             [&](int k) { return sbuf[id[k]] & 0xFFFFFFFFull; });
    store_strip<IT, true, 4>(desc->cols[2].base[BUF_OUT], 4, 4, base, ebase, cnt,
                             [&](int k) { return sbuf[id[k]] >> 32; });
  } else {  // {key, payload} records, one 16-byte store each
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t r = strip_rsrc(desc->cols[0].base[BUF_OUT] + base * 16,
                                                cnt > 0 ? (uint32_t)cnt * 16u : 0u);
#pragma unroll
    for (int k = 0; k < IT; k++) {
      const uint64_t pv = sbuf[id[k]];
      u32x4 x;
      x[0] = (uint32_t)ko[k];
      x[1] = (uint32_t)(ko[k] >> 32);
      x[2] = (uint32_t)pv;
      x[3] = (uint32_t)(pv >> 32);
      __builtin_amdgcn_raw_buffer_store_b128(x, r, (uint32_t)(ebase + k * 64) * 16u, 0, 0);
    }
  }
}

// Stable path for segments the fast kernel handed over (a top-digit bucket
// larger than kRankSortMax): the bucket pass ranks with ballots (stable), so
// buckets whose keys are all equal are final; only mixed buckets are ranked.
// Grid-stride over a device-side list whose length is read on device.
template <int NT>
struct StableLds {
  static constexpr int CAP = NT * kLocalStableItems;
  static constexpr int NB = 1 << kLocalStableTopBits;
  static constexpr int WCP = (NT / 64) * NB > CAP ? (NT / 64) * NB : CAP;
  // sbuf: packed sort words during the sort, column staging afterwards
  uint64_t sbuf[CAP];
  uint16_t wc_perm[WCP];       // ballot counters [NW][NB], then perm[CAP]
  uint32_t bflag[NB];          // bucket holds differing keys
  uint16_t sorig[CAP];         // wide words: original index by slot
  uint32_t bin_start[NB + 1];
  uint32_t scan_sh[NT / 64 + 1];
  unsigned long long sh_or;
  int maxlen;
};

// One segment g by one workgroup; true: the segment goes on to the LSD path
// (nothing written to global memory then). Block-uniform.
template <typename KT, typename U, int NT, bool CZ>
__device__ __forceinline__ bool local_stable_body(const SortDesc* __restrict__ desc, const Seg g,
                                                  StableLds<NT>& Ls) {
  constexpr int IT = kLocalStableItems;
  constexpr int NW = NT / 64;
  constexpr int CAP = NT * IT;
  constexpr int IDXB = CAP <= 4096 ? 12 : 13;  // bits of an index inside the segment
  static_assert((1 << IDXB) >= CAP, "index bits");
  constexpr int NB = 1 << kLocalStableTopBits;
  constexpr int BPT = NB >= NT ? NB / NT : 1;  // bins per thread (threads >= NB idle)
  static_assert(BPT * NT >= NB, "bins per thread");
  constexpr int WCP = StableLds<NT>::WCP;
  auto& sbuf = Ls.sbuf;
  auto& wc_perm = Ls.wc_perm;
  auto& bflag = Ls.bflag;
  auto& sorig = Ls.sorig;
  auto& bin_start = Ls.bin_start;
  auto& scan_sh = Ls.scan_sh;
  auto& sh_or = Ls.sh_or;
  auto& maxlen = Ls.maxlen;
  uint16_t* perm = wc_perm;               // output slot -> original index

  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
  const int ebase = (int)wave * IT * 64 + (int)lane;  // element of slot k: ebase + 64 k
  Xform<U, CZ> xf;
  xf.init(*desc);
  const int ncols = desc->ncols;
  const int kbytes = desc->key_bits >> 3;
  const uint64_t kmask = kbytes == 8 ? ~0ull : ((1ull << (8 * kbytes)) - 1);
  const int cnt = (int)g.len;
  const int64_t base = g.start;
  // (reset before the barrier: the previous segment read them long before
  // its last barrier, and this segment's atomics come after this one)
  if (threadIdx.x == 0) {
    sh_or = 0;
    maxlen = 0;
  }
  __syncthreads();  // the previous segment is done with the shared arrays

  for (uint32_t i = threadIdx.x; i < (uint32_t)WCP; i += NT) wc_perm[i] = 0;
  for (uint32_t i = threadIdx.x; i < (uint32_t)NB; i += NT) bflag[i] = 0;

  // ---- 1. keys (column 0 holds the key in its low bytes) -------------------
  uint64_t v0[IT];
  {
    const char* src = desc->cols[0].base[g.buf];
    const uint32_t w = desc->cols[0].width, st = desc->cols[0].stride[g.buf];
with_width(w, [&](auto W_) {
#pragma unroll
  for (int k = 0; k < IT; k++) {
    const int e = ebase + k * 64;
    v0[k] = e < cnt ? ldw<decltype(W_)::value>(src + (base + e) * (int64_t)st) : 0;
  }
});
  }
  const U uref = xf((U)(load_w(desc->cols[0].base[g.buf] +
                                   base * (int64_t)desc->cols[0].stride[g.buf],
                               desc->cols[0].width) & kmask));
  // keys are recomputed from v0 when needed (holding them costs occupancy)
  auto ukey = [&](int k) -> U { return xf((U)(v0[k] & kmask)); };
  auto valid = [&](int k) -> bool { return ebase + k * 64 < cnt; };
  U vor = 0;
#pragma unroll
  for (int k = 0; k < IT; k++)
    if (valid(k)) vor |= ukey(k) ^ uref;
  {
    const unsigned long long wv = wave_or((unsigned long long)vor);  // (one atomic per wave)
    if (lane == 0 && wv) atomicOr(&sh_or, wv);
  }
  lds_barrier();
  const unsigned long long var = sh_or;

  // exact: the bucket digit covers every varying bit, so each bucket holds a
  // single key value and the stable bucket pass alone is the sorted order
  bool exact = false;
  uint16_t* sidx = (uint16_t*)sbuf;  // exact case: original index by output slot
  if (var != 0) {
    const int lo = __ffsll((long long)var) - 1;
    const int hi = 63 - __clzll((long long)var);
    exact = hi - lo + 1 <= kLocalStableTopBits;
    // The sort word packs (key bits 0..hi, original index) when that fits
    // in 64 bits. Otherwise (wide: e.g. a whole small sort of 64-bit keys)
    // the word is the key alone and ties break by slot: the bucket pass is
    // stable, so slot order inside a bucket is input order; the original
    // index goes to sorig.
    const bool wide = hi + 1 + IDXB > 64;
    const int dsh = wide ? 0 : IDXB;  // key bits start here in a word
    const int nbits = (hi - lo + 1) < kLocalStableTopBits ? (hi - lo + 1) : kLocalStableTopBits;
    const int sh = hi - nbits + 1;
    const uint32_t mask = (1u << nbits) - 1;
    const uint64_t keep = (hi == 63) ? ~0ull : ((1ull << (hi + 1)) - 1);
    // ---- 2. stable bucket pass on the top varying bits (ballot ranks) -----
    auto digit = [&](int k) -> uint32_t { return (uint32_t)(ukey(k) >> sh) & mask; };
    uint32_t rank[IT];
    wlms_rank_fn<IT, kLocalStableTopBits>(digit, valid, nbits, &wc_perm[wave * NB], rank);
    lds_barrier();
    {
      uint32_t tb[BPT], tsum = 0;
#pragma unroll
      for (int q = 0; q < BPT; q++) {
        const uint32_t b = threadIdx.x * BPT + q;
        tb[q] = 0;
        if (b < (uint32_t)NB) {
#pragma unroll
          for (int w = 0; w < NW; w++) {
            const uint32_t c = wc_perm[w * NB + b];
            wc_perm[w * NB + b] = (uint16_t)tb[q];
            tb[q] += c;
          }
        }
        tsum += tb[q];
      }
      uint32_t tot;
      uint32_t ex = block_excl_scan_lds<NT>(tsum, scan_sh, &tot);
#pragma unroll
      for (int q = 0; q < BPT; q++) {
        const uint32_t b = threadIdx.x * BPT + q;
        if (b < (uint32_t)NB) bin_start[b] = ex;
        ex += tb[q];
      }
      if (threadIdx.x == 0) bin_start[NB] = tot;
    }
    lds_barrier();
#pragma unroll
    for (int k = 0; k < IT; k++) {
      if (valid(k)) {
        const uint32_t d = digit(k);
        const uint32_t p = bin_start[d] + wc_perm[wave * NB + d] + rank[k];
        if (exact) {
          sidx[p] = (uint16_t)(ebase + k * 64);
        } else if (wide) {
          sbuf[p] = (uint64_t)ukey(k) & keep;
          sorig[p] = (uint16_t)(ebase + k * 64);
        } else {
          sbuf[p] = (((uint64_t)ukey(k) & keep) << IDXB) | (uint64_t)(ebase + k * 64);
        }
      }
    }
    lds_barrier();
    if (!exact) {
    // ---- 3. buckets whose keys all equal are final (the pass was stable) --
#pragma unroll
    for (int i = 0; i < IT; i++) {
      const int p = i * NT + (int)threadIdx.x;
      if (p < cnt) {
        const uint64_t x = sbuf[p];
        const uint32_t d = (uint32_t)(x >> (sh + dsh)) & mask;
        if (((x ^ sbuf[bin_start[d]]) >> dsh) != 0) bflag[d] = 1;
      }
    }
    lds_barrier();
    {
      int mymax = 0;
#pragma unroll
      for (int q = 0; q < BPT; q++) {
        const uint32_t b = threadIdx.x * BPT + q;
        if (b >= (uint32_t)NB) continue;
        const int len = (int)(bin_start[b + 1] - bin_start[b]);
        if (bflag[b] && len > mymax) mymax = len;
      }
      block_max_into(&maxlen, mymax);
    }
    lds_barrier();
    if (maxlen > kRankSortMax) {
      // a large bucket of differing keys: local_lsd_kernel takes the segment
      // (nothing has been written to global memory yet)
      return true;
    }
    // ---- 4. rank inside mixed buckets: #(words of the bucket below mine) --
    // The word orders by (key, original index): stable. Slots in two halves
    // bound register use; a wave-uniform trip count keeps LDS reads in flight.
    constexpr int H = IT / 2;
#pragma unroll
    for (int half = 0; half < 2; half++) {
      uint64_t x[H];
      uint32_t bs[H], bl[H], r[H];
      int wmax = 0;
#pragma unroll
      for (int i = 0; i < H; i++) {
        const int p = (half * H + i) * NT + (int)threadIdx.x;
        bl[i] = 0;
        bs[i] = (uint32_t)p;
        x[i] = 0;
        r[i] = 0;
        if (p < cnt) {
          x[i] = sbuf[p];
          const uint32_t d = (uint32_t)(x[i] >> (sh + dsh)) & mask;
          if (bflag[d]) {
            bs[i] = bin_start[d];
            bl[i] = bin_start[d + 1] - bs[i];
            wmax = (int)bl[i] > wmax ? (int)bl[i] : wmax;
          }
        }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const int t2 = __shfl_xor(wmax, o, 64);
        wmax = t2 > wmax ? t2 : wmax;
      }
      if (!wide) {
        for (int j = 0; j < wmax; j++) {
#pragma unroll
          for (int i = 0; i < H; i++)
            if ((uint32_t)j < bl[i]) r[i] += sbuf[bs[i] + j] < x[i];
        }
      } else {
        for (int j = 0; j < wmax; j++) {
#pragma unroll
          for (int i = 0; i < H; i++) {
            const uint32_t q = bs[i] + (uint32_t)j;
            const int p = (half * H + i) * NT + (int)threadIdx.x;
            if ((uint32_t)j < bl[i]) {
              const uint64_t w = sbuf[q];
              r[i] += (w < x[i]) | ((w == x[i]) & ((int)q < p));
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < H; i++) {
        const int p = (half * H + i) * NT + (int)threadIdx.x;
        if (p < cnt)
          perm[bs[i] + r[i]] = wide ? sorig[p] : (uint16_t)(x[i] & ((1u << IDXB) - 1));
      }
    }
    lds_barrier();
    }  // !exact
  } else if (g.buf == BUF_OUT) {
    return false;  // all keys equal and already home
  } else {
#pragma unroll
    for (int k = 0; k < IT; k++) perm[ebase + k * 64] = (uint16_t)(ebase + k * 64);
    lds_barrier();
  }
  // output slot e takes input element perm[e]
  uint32_t id[IT];
#pragma unroll
  for (int k = 0; k < IT; k++) id[k] = exact ? sidx[ebase + k * 64] : perm[ebase + k * 64];

  // ---- 5. columns, software-pipelined as in local_kernel -------------------
  auto load_col = [&](int c, uint64_t (&dst)[IT]) {
    const char* src = desc->cols[c].base[g.buf];
    const uint32_t st = desc->cols[c].stride[g.buf];
    with_width(desc->cols[c].width, [&](auto W_) {
#pragma unroll
      for (int k = 0; k < IT; k++) {
        const int e = ebase + k * 64;
        dst[k] = e < cnt ? ldw<decltype(W_)::value>(src + (base + e) * (int64_t)st) : 0;
      }
    });
  };
  uint64_t vn[IT];
  load_col(0, vn);  // (the keys are reloaded: keeping them costs occupancy)
  for (int c = 0; c < ncols; c++) {
    char* out = desc->cols[c].base[BUF_OUT];
    const uint32_t st = desc->cols[c].stride[BUF_OUT];
    uint64_t v[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) v[k] = vn[k];
    if (c + 1 < ncols) load_col(c + 1, vn);
    lds_barrier();  // previous users of sbuf are done
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (valid(k)) sbuf[ebase + k * 64] = v[k];
    lds_barrier();
    with_width(desc->cols[c].width, [&](auto W_) {
#pragma unroll
      for (int k = 0; k < IT; k++) {
        const int e = ebase + k * 64;
        if (valid(k)) stw<decltype(W_)::value>(out + (base + e) * (int64_t)st, sbuf[id[k]]);
      }
    });
  }
  return false;
}

template <typename KT, typename U, int NT, bool CZ>
__global__ __launch_bounds__(NT) void local_stable_kernel(
    const SortDesc* __restrict__ desc, const Seg* __restrict__ segs,
    const unsigned long long* __restrict__ nsegs, Seg* __restrict__ fallback,
    unsigned long long* fallback_count) {
  __shared__ StableLds<NT> Ls;
  const unsigned long long total = *nsegs;
  for (unsigned long long si = blockIdx.x; si < total; si += gridDim.x) {
    const Seg g = segs[si];
    if (local_stable_body<KT, U, NT, CZ>(desc, g, Ls) && threadIdx.x == 0)
      fallback[atomicAdd(fallback_count, 1ull)] = g;
  }
}


// Fallback for segments whose top-digit buckets are too large for the rank
// step (skewed keys): stable LSD passes (ballot ranks) over every varying
// bit. Grid-stride over a device-side list whose length is read on device.
template <int NT>
struct LsdLds {
  static constexpr int CAP = NT * kLocalStableItems;
  uint64_t sbuf[CAP];
  uint16_t sidx[CAP];
  uint16_t wc[NT / 64][1 << kLocalBits];
  uint32_t bin_start[(1 << kLocalBits) + 1];
  uint32_t scan_sh[NT / 64 + 1];
  unsigned long long sh_or;
};

// One segment g (<= NT * kLocalStableItems records) by one workgroup of NT
// threads (always finishes it).
template <typename KT, typename U, bool CZ, int NT = kLocalStableThreads>
__device__ __forceinline__ void local_lsd_body(const SortDesc* __restrict__ desc, const Seg g,
                                               LsdLds<NT>& Ls) {
  constexpr int IT = kLocalStableItems;
  auto& sbuf = Ls.sbuf;
  auto& sidx = Ls.sidx;
  auto& wc = Ls.wc;
  auto& bin_start = Ls.bin_start;
  auto& scan_sh = Ls.scan_sh;
  auto& sh_or = Ls.sh_or;
  U* su = (U*)sbuf;
  const uint32_t wave = threadIdx.x >> 6;
  const int ebase = (int)wave * IT * 64 + (int)lane_id();
  Xform<U, CZ> xf;
  xf.init(*desc);
  const int ncols = desc->ncols;
  const int kbytes = desc->key_bits >> 3;
  const uint64_t kmask = kbytes == 8 ? ~0ull : ((1ull << (8 * kbytes)) - 1);
  {
    const int cnt = (int)g.len;
    const int64_t base = g.start;
    if (threadIdx.x == 0) sh_or = 0;  // (before the barrier, as in local_stable_body)
    __syncthreads();
    U u[IT];
    uint32_t id[IT];
    bool valid[IT];
    {
      const char* src = desc->cols[0].base[g.buf];
      const uint32_t w = desc->cols[0].width, st = desc->cols[0].stride[g.buf];
      with_width(w, [&](auto W_) {
#pragma unroll
        for (int k = 0; k < IT; k++) {
          const int e = ebase + k * 64;
          valid[k] = e < cnt;
          id[k] = (uint32_t)e;
          u[k] = valid[k] ? xf((U)(ldw<decltype(W_)::value>(src + (base + e) * (int64_t)st) & kmask))
                          : (U)0;
        }
      });
    }
    __syncthreads();
    const U uref = xf((U)(load_w(desc->cols[0].base[g.buf] +
                                     base * (int64_t)desc->cols[0].stride[g.buf],
                                 desc->cols[0].width) & kmask));
    U vor = 0;
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (valid[k]) vor |= u[k] ^ uref;
    {
      const unsigned long long wv = wave_or((unsigned long long)vor);  // (one atomic per wave)
      if (lane_id() == 0 && wv) atomicOr(&sh_or, wv);
    }
    __syncthreads();
    const unsigned long long var = sh_or;
    if (var != 0) {
      const int lo = __ffsll((long long)var) - 1;
      const int hi = 63 - __clzll((long long)var);
      for (int s0 = lo; s0 <= hi; s0 += kLocalBits) {
        const int nb2 = (hi - s0 + 1) < kLocalBits ? (hi - s0 + 1) : kLocalBits;
        local_digit_pass<NT, IT, U>(u, id, valid, s0, nb2, su, sidx, wc, bin_start, scan_sh);
#pragma unroll
        for (int k = 0; k < IT; k++) {
          const int e = ebase + k * 64;
          if (valid[k]) {
            u[k] = su[e];
            id[k] = sidx[e];
          }
        }
        __syncthreads();
      }
    }
    // register gather, barrier between all loads and all stores (in place safe)
    for (int c = 0; c < ncols; c++) {
      const char* src = desc->cols[c].base[g.buf];
      char* out = desc->cols[c].base[BUF_OUT];
      const uint32_t w = desc->cols[c].width, st = desc->cols[c].stride[BUF_OUT];
      const uint32_t sti = desc->cols[c].stride[g.buf];
      uint64_t v[IT];
      with_width(w, [&](auto W_) {
#pragma unroll
        for (int k = 0; k < IT; k++)
          v[k] = valid[k] ? ldw<decltype(W_)::value>(src + (base + (int64_t)id[k]) * sti) : 0;
      });
      __syncthreads();
      with_width(w, [&](auto W_) {
#pragma unroll
        for (int k = 0; k < IT; k++) {
          const int e = ebase + k * 64;
          if (valid[k]) stw<decltype(W_)::value>(out + (base + e) * (int64_t)st, v[k]);
        }
      });
    }
  }
}

template <typename KT, typename U, bool CZ>
__global__ __launch_bounds__(kLocalStableThreads) void local_lsd_kernel(
    const SortDesc* __restrict__ desc, const Seg* __restrict__ segs,
    const unsigned long long* __restrict__ nsegs) {
  __shared__ LsdLds<kLocalStableThreads> Ls;
  const unsigned long long total = *nsegs;
  for (unsigned long long si = blockIdx.x; si < total; si += gridDim.x)
    local_lsd_body<KT, U, CZ>(desc, segs[si], Ls);
}

// ---------------------------------------------------------------------------
// small sorts: n <= kLocalCap in ONE launch
// ---------------------------------------------------------------------------
// The whole input is one local segment. Instead of start kernel + segment
// list + fast / stable / LSD launches (four launches, ~40 us per call), one
// workgroup runs the three bodies in turn over a union of their LDS, with
// the descriptor as a kernel argument. taken[0] / taken[1] record whether the
// stable / LSD body ran (srs_debug_last_fallbacks).
static_assert(kLocalStableThreads == kLocalThreads, "the three bodies share one workgroup");
static_assert(sizeof(SortDesc) + sizeof(Seg) + sizeof(int64_t*) <= 4096,
              "small_sort_kernel's arguments fit the 4 KB kernel-argument segment");
static_assert(kLocalItems == kLocalStableItems, "the three bodies hold the same records per thread");
template <int NT>
union SmallLdsT {
  FastLds<NT, kLocalItems, (NT <= 512 ? 12 : 13)> fast;  // (see FastLds: TB)
  StableLds<NT> stable;
  LsdLds<NT> lsd;
};
using SmallLds = SmallLdsT<kLocalThreads>;

// NT threads for n <= NT * 8 records: a 1024-thread workgroup puts four
// waves on each SIMD, and every wave issues every (predicated) instruction of
// the bodies whether it holds records or not, so a small sort's time follows
// the waves, not the records (1024 keys: 11 us with 16 waves)
// The three bodies in turn over one segment; returns 0 (fast), 1 (stable)
// or 2 (LSD): the last body that ran.
template <typename KT, typename U, bool CZ, int NT>
__device__ __forceinline__ int small_bodies(const SortDesc* __restrict__ desc, const Seg g,
                                            SmallLdsT<NT>& Ls) {
  int path = 0;
  if (local_fast_body<KT, U, NT, kLocalItems, CZ>(desc, g, Ls.fast, [] {})) {
    __syncthreads();  // the fast body's LDS is reused
    path = 1;
    if (local_stable_body<KT, U, NT, CZ>(desc, g, Ls.stable)) {
      __syncthreads();
      path = 2;
      local_lsd_body<KT, U, CZ, NT>(desc, g, Ls.lsd);
    }
  }
  return path;
}

template <typename KT, typename U, bool CZ, int NT>
__global__ __launch_bounds__(NT) void small_sort_kernel(const SortDesc d, const Seg g,
                                                        int64_t* taken) {
  __shared__ SmallLdsT<NT> Ls;
  const SortDesc* desc = &d;
  const int path = small_bodies<KT, U, CZ, NT>(desc, g, Ls);
  if (threadIdx.x == 0 && taken) {
    taken[0] = path >= 1;
    taken[1] = path >= 2;
  }
#ifdef SRS_DIAG_TWICE
  // diagnostic (timing only): the sort again over its own output, so that a
  // kernel trace shows what a second, warm pass through the same code costs
  __syncthreads();
  small_bodies<KT, U, CZ, NT>(desc, Seg{g.start, g.len, g.rbits, BUF_OUT}, Ls);
#endif
}

// ---------------------------------------------------------------------------
// mid-size sorts (kLocalCap < n <= kMidMaxTiles * kTile) in ONE launch
// ---------------------------------------------------------------------------
// Between one workgroup's small sort and the general path (a plan, a count,
// three offset kernels and a scatter per level, then the local kernels:
// about twelve dependent launches, ~85 us of GPU-side span at 8K-64K keys,
// almost all of it launch gaps) one launch of G = ceil(n / 4096)
// workgroups does it all, with grid barriers between the phases:
//   1. every workgroup loads its tile and reduces the keys' OR / AND;
//   2. the global varying bits give the digit (choose_bits, as a level
//      would), each tile counts its digits;
//   3. each tile's bucket offsets follow from the T x 2^bits counts (every
//      workgroup scans them itself) and the tile is scattered, stably, to
//      TMP (scatter_process_tile, the global levels' code);
//   4. workgroup b sorts bucket b in LDS with the small sort's bodies (fast,
//      stable, LSD) into OUT; a bucket larger than kLocalCap (skewed keys)
//      goes to the big list for the host's general levels (ctr->n_big, read
//      back once).
// G = max(T tiles, 2^mid_bits(n)) workgroups (<= 256 at kMidMaxKeys): one
// bucket each, no loop -- a loop over buckets had the compiler hoist the
// bodies' per-thread invariants out of it and spill 55 VGPRs. One
// workgroup per CU (129 KB of LDS), so G must fit the chip for the
// launch (its grid barriers need every workgroup resident). Round 6: up to
// 2^20 keys (256 tiles, the digit capped at 8 bits: 256 buckets of ~4K);
// when the T x 2^bits count matrix exceeds the LDS share (kMidMat) the
// column scans are spread over the grid (phase 2b, one more barrier).
constexpr int kMidMaxTiles = 256;  // n <= 2^20
constexpr int kMidMaxBits = 8;     // (G <= 256: every bucket its workgroup)
constexpr int kMidMat = 8192;      // tiles x buckets scanned in LDS (64 x 128)
static_assert(kMidMat % kScatterThreads == 0, "count matrix: whole rounds of loads");

struct MidLevelLds {
  ScatterLds<0> sc;
  SegPlan plan;
  unsigned long long wor[kScatterThreads / 64], wand[kScatterThreads / 64];
  uint32_t hist[kMaxBins];
  uint32_t mat[kMidMat];  // every tile's bucket counts (phase 3)
};

// A grid barrier of the mid-size launch. Every workgroup is resident (the
// host launches G <= CUs x resident workgroups per CU, one per CU at 123 KB
// of LDS), so a plain launch replaces the cooperative launch (VERDICT r05:
// processes that had made a cooperative launch crashed in the runtime's
// teardown at exit under rocprofv3). A central counter with a generation
// word (sense reversal): each workgroup notes the generation, arrives with
// one atomic add, and the last to arrive resets the counter and bumps the
// generation, which releases the others; the words are left ready for the
// next barrier and the next call (no per-call state in the kernel's
// arguments: every argument costs SGPRs, and this kernel is at its limit).
// A compare-and-swap arrival (tagged words) serialised 128 workgroups'
// retries at 0.6 ms per call. The agent-scope fences write this workgroup's
// stores back to the shared point of coherence before it arrives (and make
// the generation read complete first) and invalidate stale lines after the
// wait (workgroups sit on different XCDs, each with its own L2). The wait is
// bounded: a barrier that never fills (it cannot, short of a broken
// residency assumption) posts the call's seq to MidFlag::err and lets the
// grid drain instead of hanging the GPU; the host checks it.
// FULL = false ("light"): the phases before it exchange only small words
// (tile OR / AND, count rows, column scans), and those move with agent-scope
// atomic stores and loads (mid_st / mid_ld: sc1, coherent at the device
// level without the L2), so the barrier needs no L2 write-back or
// invalidate, only every store acknowledged before the arrival
// (tools/probe/mid_barrier: 3.9 instead of 9.4 us per barrier at 256
// workgroups). The barrier before the bucket sorts, which read the scattered
// tiles (ordinary stores), is FULL.
constexpr int kMidBarWords = 32;  // u64: the counter and the generation 128 bytes apart
template <bool FULL>
__device__ __forceinline__ void mid_grid_barrier(unsigned long long* bar, unsigned long long seq,
                                                 MidFlag* flag) {
  if (!FULL) __builtin_amdgcn_s_waitcnt(0);  // (this thread's sc1 stores acknowledged)
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* cnt = (unsigned*)bar;
    unsigned* gen = (unsigned*)(bar + 16);
    const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // (release: this workgroup's writes; and g0 is read before arriving)
    if (FULL) __threadfence();
    else __builtin_amdgcn_s_waitcnt(0);
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {  // the last arrival: reset, then release everyone
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0);
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      for (uint32_t spin = 0;
           __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0; spin++) {
        __builtin_amdgcn_s_sleep(2);
        if (spin > (1u << 24)) {  // (seconds: never in a correct run)
          __hip_atomic_store(&flag->err, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
    if (FULL) __threadfence();  // (acquire: the other workgroups' writes)
  }
  __syncthreads();
}
// the words the light barriers order (see above)
template <typename T>
__device__ __forceinline__ void mid_st(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T mid_ld(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void mid_tell_host(MidFlag* f, unsigned long long n_big,
                                              unsigned long long seq) {
  __hip_atomic_store(&f->n_big, n_big, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&f->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
union MidLds {
  SmallLds local;
  MidLevelLds level;
};

template <typename KT, typename U, bool CZ>
__global__ __launch_bounds__(kLocalThreads) void mid_sort_kernel(
    const SortDesc d, int64_t n, int32_t src, unsigned long long* __restrict__ part,
    uint32_t* __restrict__ hist, ListCounters* __restrict__ ctr, Seg* __restrict__ big,
    unsigned long long* __restrict__ taken, MidFlag* __restrict__ flag, unsigned long long seq,
    unsigned long long* __restrict__ bar, int wide) {
  static_assert(kLocalThreads == kScatterThreads, "the level phases use the scatter's shape");
  __shared__ MidLds Ls;
  __shared__ int64_t my_start;
  __shared__ int32_t my_len;
  const SortDesc* desc = &d;
  constexpr int IT = kScatterItems;
  const int G = (int)gridDim.x;
  const int T = (int)((n + kTile - 1) / kTile);  // tiles (workgroups [0, T))
  const int w = (int)blockIdx.x;
  const bool has_tile = w < T;
  const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
  const int64_t tbase = (int64_t)w * kTile;
  const int cnt = has_tile ? (int)std::min<int64_t>(kTile, n - tbase) : 0;
  const int ebase = (int)wave * IT * 64 + (int)lane;
  const int ncols = desc->ncols;
  Xform<U, CZ> xf;
  xf.init(*desc);
  const int kbytes = desc->key_bits >> 3;
  const uint64_t kmask = kbytes == 8 ? ~0ull : ((1ull << (8 * kbytes)) - 1);
  auto valid = [&](int k) -> bool { return ebase + k * 64 < cnt; };

  // ---- 1. the tile in registers; the keys' OR / AND
  uint64_t v0[IT], v1[IT], v2[IT];
  if (has_tile) {
    load_strip<IT>(v0, desc->cols[0].base[src], desc->cols[0].width, desc->cols[0].stride[src],
                   tbase, ebase, cnt);
    if (ncols > 1)
      load_strip<IT>(v1, desc->cols[1].base[src], desc->cols[1].width,
                     desc->cols[1].stride[src], tbase, ebase, cnt);
    unsigned long long kor = 0, kand = ~0ull;
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (valid(k)) {
        const unsigned long long u = (unsigned long long)xf((U)(v0[k] & kmask));
        kor |= u;
        kand &= u;
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      kor |= __shfl_xor(kor, o, 64);
      kand &= __shfl_xor(kand, o, 64);
    }
    if (lane == 0) {
      Ls.level.wor[wave] = kor;
      Ls.level.wand[wave] = kand;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long o = 0, a = ~0ull;
      for (int i = 0; i < kScatterThreads / 64; i++) {
        o |= Ls.level.wor[i];
        a &= Ls.level.wand[i];
      }
      mid_st(&part[2 * w], o);
      mid_st(&part[2 * w + 1], a);
    }
  }
  if (w == 0 && threadIdx.x == 0) {  // (every counter: a skewed sort continues on the general path)
    *ctr = ListCounters{};
    taken[0] = taken[1] = 0;
  }
  mid_grid_barrier<false>(bar, seq, flag);

  // ---- 2. the digit; this tile's counts
  // (the T pairs in one round of loads: a loop over them paid a cross-XCD
  // round trip per tile)
  unsigned long long gor = 0, gand = ~0ull;
  {
    unsigned long long o = 0, a = ~0ull;
    if (threadIdx.x < (uint32_t)T) {
      o = mid_ld(&part[2 * threadIdx.x]);
      a = mid_ld(&part[2 * threadIdx.x + 1]);
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
      o |= __shfl_xor(o, s, 64);
      a &= __shfl_xor(a, s, 64);
    }
    __syncthreads();  // (phase 1's reads of wor / wand are over)
    if (lane == 0) {
      Ls.level.wor[wave] = o;
      Ls.level.wand[wave] = a;
    }
    __syncthreads();
    for (int i = 0; i < kScatterThreads / 64; i++) {
      gor |= Ls.level.wor[i];
      gand &= Ls.level.wand[i];
    }
  }
  const unsigned long long var = gor ^ gand;
  if (var == 0) {  // every key equal: the input is the output (stable)
    if (w == 0 && threadIdx.x == 0) mid_tell_host(flag, 0, seq);
    if (src != BUF_OUT && has_tile)
      for (int c = 0; c < ncols; c++) {
        uint64_t t[IT];
        load_strip<IT>(t, desc->cols[c].base[src], desc->cols[c].width,
                       desc->cols[c].stride[src], tbase, ebase, cnt);
        store_strip<IT>(desc->cols[c].base[BUF_OUT], desc->cols[c].width,
                        desc->cols[c].stride[BUF_OUT], tbase, ebase, cnt,
                        [&](int k) { return t[k]; });
      }
    return;  // (uniform over the grid: no barrier follows)
  }
  const int rbits = 64 - __clzll((long long)var);
  const int bits = min(choose_bits(n, rbits), kMidMaxBits);
  const int shift = rbits - bits;
  const uint32_t nb = 1u << bits, mask = nb - 1;
  if (has_tile) {
    for (uint32_t b = threadIdx.x; b < kMaxBins; b += kScatterThreads) Ls.level.hist[b] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (valid(k))
        atomicAdd(&Ls.level.hist[(uint32_t)(xf((U)(v0[k] & kmask)) >> shift) & mask], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += kScatterThreads)
      mid_st(&hist[(size_t)w * kMaxBins + b], Ls.level.hist[b]);
  }
  mid_grid_barrier<false>(bar, seq, flag);
  const int TN = T * (int)nb;
  if (wide) {
    // ---- 2b. (the count matrix does not fit one workgroup's LDS) workgroup
    // j < nb scans bucket j's column over the tiles: its tiles' offsets
    // inside the bucket in place of their counts, the bucket's total in
    // part[j] (phase 1's words are read: phase 2 is over)
    const uint32_t i = threadIdx.x;  // (kScatterThreads >= kMidMaxTiles: one tile per thread)
    if (w < (int)nb) {
      const uint32_t c = i < (uint32_t)T ? mid_ld(&hist[(size_t)i * kMaxBins + w]) : 0u;
      uint32_t all;
      const uint32_t ex = block_excl_scan<kScatterThreads, uint32_t>(c, Ls.level.sc.scan_sh, &all);
      if (i < (uint32_t)T) mid_st(&hist[(size_t)i * kMaxBins + w], ex);
      if (i == 0) mid_st(&part[w], (unsigned long long)all);
    }
    mid_grid_barrier<false>(bar, seq, flag);
  }

  // ---- 3. offsets; the stable scatter of the tile into TMP
  {
    const uint32_t b = threadIdx.x;  // (kScatterThreads >= kMaxBins: one bin per thread)
    uint32_t tot = 0, pre = 0;
    if (wide) {  // (phase 2b's bucket totals and this tile's row of offsets)
      if (b < nb) {
        tot = (uint32_t)mid_ld(&part[b]);
        pre = has_tile ? mid_ld(&hist[(size_t)w * kMaxBins + b]) : 0u;
      }
    } else {
      // the T x nb counts into LDS in one round of loads, then summed per bucket
      uint32_t cv[kMidMat / kScatterThreads];
#pragma unroll
      for (int k = 0; k < kMidMat / kScatterThreads; k++) {
        const int e = (int)threadIdx.x + k * kScatterThreads;
        cv[k] = e < TN ? mid_ld(&hist[(size_t)(e >> bits) * kMaxBins + (e & mask)]) : 0u;
      }
#pragma unroll
      for (int k = 0; k < kMidMat / kScatterThreads; k++) {
        const int e = (int)threadIdx.x + k * kScatterThreads;
        if (e < TN) Ls.level.mat[e] = cv[k];
      }
      __syncthreads();
      if (b < nb)
        for (int i = 0; i < T; i++) {
          const uint32_t c = Ls.level.mat[i * nb + b];
          tot += c;
          pre += i < w ? c : 0u;
        }
    }
    uint32_t all;
    const uint32_t bs = block_excl_scan<kScatterThreads, uint32_t>(tot, Ls.level.sc.scan_sh, &all);
    if (b == (uint32_t)w) {  // (this workgroup's bucket, for phase 4)
      my_start = b < nb ? (int64_t)bs : 0;
      my_len = b < nb ? (int32_t)tot : 0;
    }
    // the host learns now how many buckets come back to it, not at the end
    const int nbig = __syncthreads_count(b < nb && tot > (uint32_t)kLocalCap && shift > 0);
    if (w == 0 && threadIdx.x == 0)
      mid_tell_host(flag, (unsigned long long)nbig |
                              (nb > (uint32_t)G || (!wide && TN > kMidMat) ? 1ull << 63 : 0), seq);
    if (has_tile) {
      if (threadIdx.x == 0) {
        SegPlan& P = Ls.level.plan;
        P.start = 0;
        P.len = n;
        P.tile_base = 0;
        P.group_base = 0;
        P.ntiles = T;
        P.ngroups = 1;
        P.shift = shift;
        P.bits = bits;
        P.buf = src;
        P.dst = BUF_TMP;
        P.skip = 0;
      }
      __syncthreads();
      TileInfo ti;
      ti.base = tbase;
      ti.cnt = cnt;
      ti.s = 0;
      ti.t = w;
      const int64_t my_off = b < nb ? (int64_t)bs + pre : 0;
      scatter_process_tile<KT, U, 0, CZ, false>(desc, &Ls.level.plan, Ls.level.sc, ti, ncols, v0,
                                                 v1, v2, my_off, DigitLut{});
    }
  }
  mid_grid_barrier<true>(bar, seq, flag);

  // ---- 4. bucket w, into OUT
  const int32_t len = my_len;
  if (len == 0) return;
  const Seg g{my_start, (int64_t)len, shift, BUF_TMP};
  if (len > kLocalCap && shift > 0) {  // (skewed keys: the host's general levels take it)
    if (threadIdx.x == 0) big[atomicAdd(&ctr->n_big, 1ull)] = g;
    return;
  }
  if (len > kLocalCap) {  // one key value (no bits below the digit): TMP holds it in order
    for (int c = 0; c < ncols; c++) {
      const Col& C = desc->cols[c];
      with_width(C.width, [&](auto W_) {
        constexpr int WB = decltype(W_)::value;
        for (int64_t i = threadIdx.x; i < len; i += kLocalThreads) {
          const int64_t r = my_start + i;
          stw<WB>(C.base[BUF_OUT] + r * C.stride[BUF_OUT], ldw<WB>(C.base[BUF_TMP] + r * C.stride[BUF_TMP]));
        }
      });
    }
    return;
  }
  // (a bucket of <= 4096 records by the first 512 threads: waves 8-15 end
  // here, and the bodies' barriers wait for the surviving waves only; eight
  // waves instead of sixteen issue the bodies' instructions, as in the small
  // sort's shapes)
  int path;
  if (len <= 512 * kLocalItems) {
    if (threadIdx.x >= 512) return;
    path = small_bodies<KT, U, CZ, 512>(desc, g, *reinterpret_cast<SmallLdsT<512>*>(&Ls.local));
  } else {
    path = small_bodies<KT, U, CZ, kLocalThreads>(desc, g, Ls.local);
  }
  if (threadIdx.x == 0 && path) {
    atomicMax(&taken[0], 1ull);
    if (path >= 2) atomicMax(&taken[1], 1ull);
  }
}

// ---------------------------------------------------------------------------
// the first level of a kMidMaxKeys < n <= kMidLevelMaxKeys sort in ONE launch
// ---------------------------------------------------------------------------
// Past the mid-size launch (one bucket per resident workgroup) the general
// path's first level costs a start kernel, a plan, a tile map, the count,
// three scan kernels, the scatter and a list read-back before the LDS pass
// can be enqueued: ~60 us of launch gaps and host wait around ~15 us of
// memory work at 2^21 keys. Here one launch of G = min(T, resident)
// workgroups, each looping over tiles w, w + G, ..., does it with two grid
// barriers (mid_grid_barrier, light: only count words cross them):
//   A. every tile's digit counts at the full key width (a level's digit:
//      choose_bits), and each workgroup's key OR / AND;
//   -- barrier; the keys' varying bits: when the digit lies above them
//      (every key in one bucket) A runs again below them (uniform decision,
//      at most once: the recount's digit holds the top varying bit);
//   B. workgroup j scans bucket j's column over the tiles (<= 1024: one per
//      thread), the tiles' offsets in place, the bucket's total;
//   -- barrier;
//   C. bucket bases (one scan per workgroup); workgroup 0 appends the
//      buckets to the work lists with a level's classes (emit_child) and
//      posts the lists' lengths to the host (MidFlag) -- the host enqueues the
//      LDS pass while the scatter runs; every tile is scattered into TMP with
//      the global levels' code (scatter_process_tile).
// The host continues exactly as after a general first level (skewed keys:
// big buckets take the general levels). Keys equal throughout: copied to OUT.
constexpr int kMidLevelMaxTiles = kMidLevelMaxKeys / kTile;
static_assert(kMidLevelMaxTiles <= kScatterThreads, "column scans: one tile per thread");
static_assert(kMaxBins <= kScatterThreads, "bucket scan: one bucket per thread");

__device__ __forceinline__ void copy_desc(const SortDesc& d, SortDesc* out);

struct MidLevel1Lds {
  ScatterLds<0> sc;
  SegPlan plan;
  unsigned long long wor[kScatterThreads / 64], wand[kScatterThreads / 64];
  uint32_t hist[kMaxBins];
  uint32_t cls[5];  // list lengths (big, local, local2, copy) and the local lists' records
};

template <typename KT, typename U, bool CZ>
__global__ __launch_bounds__(kScatterThreads) void mid_level_kernel(
    const SortDesc d, int64_t n, int32_t src, unsigned long long* __restrict__ part,
    uint32_t* __restrict__ hist, ListCounters* __restrict__ ctr, Seg* __restrict__ big,
    Seg* __restrict__ local, Seg* __restrict__ local2, Seg* __restrict__ copy,
    SortDesc* __restrict__ d_out, MidFlag* __restrict__ flag, unsigned long long seq,
    unsigned long long* __restrict__ bar) {
  __shared__ MidLevel1Lds L;
  const SortDesc* desc = &d;
  constexpr int IT = kScatterItems;
  constexpr int NT = kScatterThreads;
  const int G = (int)gridDim.x;
  const int T = (int)((n + kTile - 1) / kTile);
  const int w = (int)blockIdx.x;
  const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
  const int ebase = (int)wave * IT * 64 + (int)lane;
  const int ncols = desc->ncols;
  Xform<U, CZ> xf;
  xf.init(*desc);
  const int kbytes = desc->key_bits >> 3;
  const uint64_t kmask = kbytes == 8 ? ~0ull : ((1ull << (8 * kbytes)) - 1);
  auto tile_cnt = [&](int t) { return (int)std::min<int64_t>(kTile, n - (int64_t)t * kTile); };
  unsigned long long* tot_w = part;             // [kMaxBins] bucket totals (B)
  unsigned long long* var_w = part + kMaxBins;  // [2 G] the workgroups' key OR / AND (A)
  if (w == 0) {
    copy_desc(d, d_out);  // (for the kernels that follow)
    if (threadIdx.x == 0) *ctr = ListCounters{};
  }

  int rbits = desc->key_bits, bits = 0, shift = 0;
  uint32_t nb = 0;
  for (int pass = 0;; pass++) {
    bits = min(choose_bits(n, rbits), kMaxDigitBits);
    shift = rbits - bits;
    nb = 1u << bits;
    const uint32_t mask = nb - 1;
    // ---- A. the tiles' digit counts; the keys' OR / AND
    unsigned long long kor = 0, kand = ~0ull;
    // (the next tile's keys are loaded while this one is counted)
    uint64_t nv[IT];
    if (w < T)
      load_strip<IT>(nv, desc->cols[0].base[src], desc->cols[0].width, desc->cols[0].stride[src],
                     (int64_t)w * kTile, ebase, tile_cnt(w));
    for (int t = w; t < T; t += G) {
      const int cnt = tile_cnt(t);
      uint64_t v[IT];
#pragma unroll
      for (int k = 0; k < IT; k++) v[k] = nv[k];
      if (t + G < T)
        load_strip<IT>(nv, desc->cols[0].base[src], desc->cols[0].width,
                       desc->cols[0].stride[src], (int64_t)(t + G) * kTile, ebase, tile_cnt(t + G));
      __syncthreads();  // (the previous tile's row has been read out)
      if (threadIdx.x < (uint32_t)kMaxBins) L.hist[threadIdx.x] = 0;
      __syncthreads();
#pragma unroll
      for (int k = 0; k < IT; k++)
        if (ebase + k * 64 < cnt) {
          const unsigned long long u = (unsigned long long)xf((U)(v[k] & kmask));
          kor |= u;
          kand &= u;
          atomicAdd(&L.hist[(uint32_t)(u >> shift) & mask], 1u);
        }
      __syncthreads();
      if (threadIdx.x < nb) mid_st(&hist[(size_t)t * kMaxBins + threadIdx.x], L.hist[threadIdx.x]);
    }
    if (pass == 0) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        kor |= __shfl_xor(kor, o, 64);
        kand &= __shfl_xor(kand, o, 64);
      }
      if (lane == 0) {
        L.wor[wave] = kor;
        L.wand[wave] = kand;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned long long o = 0, a = ~0ull;
        for (int i = 0; i < NT / 64; i++) {
          o |= L.wor[i];
          a &= L.wand[i];
        }
        mid_st(&var_w[2 * w], o);
        mid_st(&var_w[2 * w + 1], a);
      }
    }
    mid_grid_barrier<false>(bar, seq, flag);
    if (pass == 0) {
      // the varying bits (G <= NT pairs: one round of loads)
      unsigned long long o = 0, a = ~0ull;
      if (threadIdx.x < (uint32_t)G) {
        o = mid_ld(&var_w[2 * threadIdx.x]);
        a = mid_ld(&var_w[2 * threadIdx.x + 1]);
      }
#pragma unroll
      for (int s = 32; s > 0; s >>= 1) {
        o |= __shfl_xor(o, s, 64);
        a &= __shfl_xor(a, s, 64);
      }
      __syncthreads();  // (the reads of wor / wand above are over)
      if (lane == 0) {
        L.wor[wave] = o;
        L.wand[wave] = a;
      }
      __syncthreads();
      unsigned long long gor = 0, gand = ~0ull;
      for (int i = 0; i < NT / 64; i++) {
        gor |= L.wor[i];
        gand &= L.wand[i];
      }
      const unsigned long long var = gor ^ gand;
      if (var == 0) {  // every key equal: the input is the output (stable)
        if (w == 0) {
          __syncthreads();  // (copy_desc above; nothing follows on the device)
          if (threadIdx.x == 0) {
            __hip_atomic_store(&flag->n_local, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&flag->n_local2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&flag->n_copy, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            mid_tell_host(flag, 0, seq);
          }
        }
        if (src != BUF_OUT)
          for (int t = w; t < T; t += G) {
            const int cnt = tile_cnt(t);
            for (int c = 0; c < ncols; c++) {
              uint64_t tv[IT];
              load_strip<IT>(tv, desc->cols[c].base[src], desc->cols[c].width,
                             desc->cols[c].stride[src], (int64_t)t * kTile, ebase, cnt);
              store_strip<IT>(desc->cols[c].base[BUF_OUT], desc->cols[c].width,
                              desc->cols[c].stride[BUF_OUT], (int64_t)t * kTile, ebase, cnt,
                              [&](int k) { return tv[k]; });
            }
          }
        return;  // (uniform over the grid: no barrier follows)
      }
      const int vb = 64 - __clzll((long long)var);
      if (vb <= shift) {  // (every key in one bucket: count again below the shared bits)
        rbits = vb;
        continue;
      }
    }
    // ---- B. bucket j's column: the tiles' offsets inside it, its total
    for (uint32_t j = (uint32_t)w; j < nb; j += (uint32_t)G) {
      const uint32_t i = threadIdx.x;
      const uint32_t c = i < (uint32_t)T ? mid_ld(&hist[(size_t)i * kMaxBins + j]) : 0u;
      uint32_t all;
      const uint32_t ex = block_excl_scan<NT, uint32_t>(c, L.sc.scan_sh, &all);
      if (i < (uint32_t)T) mid_st(&hist[(size_t)i * kMaxBins + j], ex);
      if (i == 0) mid_st(&tot_w[j], (unsigned long long)all);
      __syncthreads();  // (scan_sh is reused)
    }
    mid_grid_barrier<false>(bar, seq, flag);
    break;
  }

  // ---- C. bucket bases; the work lists; the scatter into TMP
  const uint32_t b = threadIdx.x;
  const uint32_t tot = b < nb ? (uint32_t)mid_ld(&tot_w[b]) : 0u;
  uint32_t all;
  const uint32_t bs = block_excl_scan<NT, uint32_t>(tot, L.sc.scan_sh, &all);
  if (w == 0) {
    // a level's classes (emit_child): final buckets (no bits left, or one
    // record) are copied by the LDS pass or, past its capacity, the copy list
    int cls = -1;
    if (tot > 0) {
      const bool fin = shift == 0 || tot == 1;
      cls = tot <= (uint32_t)kLocalCapSmall ? 1 : tot <= (uint32_t)kLocalCap ? 2 : fin ? 3 : 0;
    }
    if (threadIdx.x < 5) L.cls[threadIdx.x] = 0;
    __syncthreads();
    uint32_t my = 0;
    if (cls >= 0) my = atomicAdd(&L.cls[cls], 1u);
    if (cls == 1 || cls == 2) atomicAdd(&L.cls[4], tot);
    __syncthreads();
    if (cls >= 0) {
      Seg* list = cls == 0 ? big : cls == 1 ? local : cls == 2 ? local2 : copy;
      list[my] = Seg{(int64_t)bs, (int64_t)tot, shift, BUF_TMP};
    }
    if (threadIdx.x == 0) {
      ctr->n_big = L.cls[0];
      ctr->n_local = L.cls[1];
      ctr->n_local2 = L.cls[2];
      ctr->n_copy = L.cls[3];
      ctr->local_elems = L.cls[4];
      __hip_atomic_store(&flag->n_local, (unsigned long long)L.cls[1], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&flag->n_local2, (unsigned long long)L.cls[2], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&flag->n_copy, (unsigned long long)L.cls[3], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&flag->local_elems, (unsigned long long)L.cls[4], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      mid_tell_host(flag, L.cls[0], seq);
    }
  }
  if (threadIdx.x == 0) {
    SegPlan& P = L.plan;
    P.start = 0;
    P.len = n;
    P.tile_base = 0;
    P.group_base = 0;
    P.ntiles = T;
    P.ngroups = 1;
    P.shift = shift;
    P.bits = bits;
    P.buf = src;
    P.dst = BUF_TMP;
    P.skip = 0;
  }
  // (the next tile's first two columns are loaded while this one is scattered)
  uint64_t n0[IT], n1[IT];
  auto load_next = [&](int t) {
    const int64_t tbase = (int64_t)t * kTile;
    const int cnt = tile_cnt(t);
    load_strip<IT>(n0, desc->cols[0].base[src], desc->cols[0].width, desc->cols[0].stride[src],
                   tbase, ebase, cnt);
    if (ncols > 1)
      load_strip<IT>(n1, desc->cols[1].base[src], desc->cols[1].width,
                     desc->cols[1].stride[src], tbase, ebase, cnt);
  };
  if (w < T) load_next(w);
  for (int t = w; t < T; t += G) {
    const int cnt = tile_cnt(t);
    const int64_t tbase = (int64_t)t * kTile;
    uint64_t v0[IT], v1[IT], v2[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) {
      v0[k] = n0[k];
      v1[k] = n1[k];
    }
    const int64_t my_off = b < nb ? (int64_t)bs + mid_ld(&hist[(size_t)t * kMaxBins + b]) : 0;
    if (t + G < T) load_next(t + G);  // (after the offsets' load: its wait skips these)
    __syncthreads();  // (the plan is published; the previous tile's LDS use is over)
    TileInfo ti;
    ti.base = tbase;
    ti.cnt = cnt;
    ti.s = 0;
    ti.t = t;
    scatter_process_tile<KT, U, 0, CZ, false>(desc, &L.plan, L.sc, ti, ncols, v0, v1, v2, my_off,
                                               DigitLut{});
  }
}

// ---------------------------------------------------------------------------
// sampled 16-bit key histogram (balanced first level): chunk c
// = keys [c*stride, c*stride + chunk). Each of kSampleWGs workgroups counts
// its share of the chunks into LDS-private u16 bins (64K bins packed in
// pairs: 128 KB of LDS; a workgroup counts < 65536 keys) and stores them as
// one partial row; a second kernel sums the rows. Global atomics per key
// (the previous form) took 0.16 ms for 4M keys.
constexpr int kSampleThreads = 1024;

__global__ __launch_bounds__(kSampleThreads) void sample_hist16_kernel(
    const char* __restrict__ keys, int key_bytes, int elem_bytes, int64_t n, int64_t stride,
    int chunk, int64_t nchunks, uint64_t mpos, uint64_t mneg, uint32_t* __restrict__ partial) {
  __shared__ uint32_t h2[32768];
  for (uint32_t i = threadIdx.x; i < 32768u; i += kSampleThreads) h2[i] = 0;
  __syncthreads();
  const int kb = 8 * key_bytes;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t a = c * stride;
    const int64_t e = min(n, a + chunk);
    for (int64_t i = a + threadIdx.x; i < e; i += kSampleThreads) {
      const uint64_t bits = load_w(keys + i * elem_bytes, key_bytes);  // (AoS: record stride)
      const uint64_t u = bits ^ (((bits >> (kb - 1)) & 1) ? mneg : mpos);
      const uint32_t d = (uint32_t)(u >> (kb - 16)) & 0xFFFFu;
      atomicAdd(&h2[d >> 1], 1u << ((d & 1) << 4));
    }
  }
  __syncthreads();
  uint32_t* row = partial + (int64_t)blockIdx.x * 32768;
  for (uint32_t i = threadIdx.x; i < 32768u; i += kSampleThreads) row[i] = h2[i];
}

__global__ __launch_bounds__(256) void sample_reduce_kernel(const uint32_t* __restrict__ partial,
                                                            int rows, uint32_t* __restrict__ hist) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;  // a pair of bins
  uint32_t lo = 0, hi = 0;
  for (int r = 0; r < rows; r++) {
    const uint32_t v = partial[(int64_t)r * 32768 + i];
    lo += v & 0xFFFFu;
    hi += v >> 16;
  }
  hist[2 * i] = lo;
  hist[2 * i + 1] = hi;
}

int64_t sample_partial_bytes() { return (int64_t)kSampleWGs * 32768 * 4; }

// Exact smallest and largest transformed key of each of up to kMaxRanges
// key clusters (range c = #{k : u > hi[k]}): the range level's plan
// (DESIGN.md §2). mm[2c] / mm[2c + 1] must hold ~0 / 0 before the launch.
constexpr int kMinMaxThreads = 256;
__global__ __launch_bounds__(kMinMaxThreads) void key_minmax_kernel(
    const char* __restrict__ keys, int key_bytes, int elem_bytes, int64_t n, uint64_t mpos,
    uint64_t mneg, uint64_t hi0, uint64_t hi1, uint64_t hi2, unsigned long long* __restrict__ mm) {
  constexpr int R = kMaxRanges;
  __shared__ unsigned long long sh[2 * R][kMinMaxThreads / 64];
  const int kb = 8 * key_bytes;
  uint64_t lo[R], hi[R];
#pragma unroll
  for (int c = 0; c < R; c++) {
    lo[c] = ~0ull;
    hi[c] = 0;
  }
  auto add = [&](uint64_t bits) {
    const uint64_t u = bits ^ (((bits >> (kb - 1)) & 1) ? mneg : mpos);
    const int c = (u > hi0) + (u > hi1) + (u > hi2);
#pragma unroll
    for (int k = 0; k < R; k++) {
      if (c == k) {
        lo[k] = u < lo[k] ? u : lo[k];
        hi[k] = u > hi[k] ? u : hi[k];
      }
    }
  };
  const int64_t step = (int64_t)gridDim.x * kMinMaxThreads;
  int64_t i = (int64_t)blockIdx.x * kMinMaxThreads + threadIdx.x;
  for (; i + 3 * step < n; i += 4 * step) {  // four loads in flight per thread
    uint64_t b[4];
#pragma unroll
    for (int k = 0; k < 4; k++) b[k] = load_w(keys + (i + k * step) * elem_bytes, key_bytes);
#pragma unroll
    for (int k = 0; k < 4; k++) add(b[k]);
  }
  for (; i < n; i += step) add(load_w(keys + i * elem_bytes, key_bytes));
#pragma unroll
  for (int c = 0; c < R; c++) {
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t l2 = __shfl_xor(lo[c], o), h2 = __shfl_xor(hi[c], o);
      lo[c] = l2 < lo[c] ? l2 : lo[c];
      hi[c] = h2 > hi[c] ? h2 : hi[c];
    }
  }
  const uint32_t wave = threadIdx.x >> 6;
  if (lane_id() == 0) {
#pragma unroll
    for (int c = 0; c < R; c++) {
      sh[2 * c][wave] = lo[c];
      sh[2 * c + 1][wave] = hi[c];
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * R) {
    const int j = threadIdx.x;
    unsigned long long v = sh[j][0];
    for (int w = 1; w < kMinMaxThreads / 64; w++) {
      const unsigned long long x = sh[j][w];
      v = (j & 1) ? (x > v ? x : v) : (x < v ? x : v);
    }
    if (j & 1) {
      if (v) atomicMax(&mm[j], v);
    } else if (v != ~0ull) {
      atomicMin(&mm[j], v);
    }
  }
}

void launch_key_minmax(const void* keys, int key_bytes, int elem_bytes, int64_t n, uint64_t mpos,
                       uint64_t mneg, const uint64_t* hi, unsigned long long* mm, hipStream_t st) {
  const int64_t blocks = std::min<int64_t>(2048, (n + kMinMaxThreads - 1) / kMinMaxThreads);
  key_minmax_kernel<<<(unsigned)std::max<int64_t>(1, blocks), kMinMaxThreads, 0, st>>>(
      (const char*)keys, key_bytes, elem_bytes, n, mpos, mneg, hi[0], hi[1], hi[2], mm);
}

bool launch_sample_hist16(const void* keys, int key_bytes, int elem_bytes, int64_t n,
                          int64_t stride, int chunk, int64_t blocks, uint64_t mpos, uint64_t mneg,
                          uint32_t* partial, uint32_t* hist, hipStream_t st) {
  const int wgs = (int)std::min<int64_t>(kSampleWGs, std::max<int64_t>(1, blocks));
  // the packed u16 bins of one workgroup must not carry into their neighbour
  if ((blocks + wgs - 1) / wgs * (int64_t)chunk >= 65536) return false;
  sample_hist16_kernel<<<(unsigned)wgs, kSampleThreads, 0, st>>>(
      (const char*)keys, key_bytes, elem_bytes, n, stride, chunk, blocks, mpos, mneg, partial);
  sample_reduce_kernel<<<32768 / 256, 256, 0, st>>>(partial, wgs, hist);
  return true;
}

// ---------------------------------------------------------------------------
// synthetic data (bench / tests): splitmix64 of the global index
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void fill_kernel(int64_t n, int kind, uint64_t seed, uint64_t first,
                            char* keys, int npay, const Col* __restrict__ pays) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = splitmix64(seed + first + (uint64_t)i);
  uint64_t bits;
  uint32_t ksz;
  switch (kind) {
    case 0: case 1: bits = h & 0xFF; ksz = 1; break;
    case 2: case 3: bits = h & 0xFFFF; ksz = 2; break;
    case 4: case 5: bits = h & 0xFFFFFFFFull; ksz = 4; break;
    case 8: {  // uniform [-1, 1) on a 2^-23 grid (24 random bits)
      const float f = (float)(int32_t)(h >> 40) * (1.0f / 8388608.0f) - 1.0f;
      bits = __float_as_uint(f);
      ksz = 4;
    } break;
    case 9: {  // uniform [-1, 1) on a 2^-52 grid
      const double f = (double)(int64_t)(h >> 11) * (1.0 / 4503599627370496.0) - 1.0;
      bits = (uint64_t)__double_as_longlong(f);
      ksz = 8;
    } break;
    default: bits = h; ksz = 8; break;
  }
  store_w(keys + i * ksz, ksz, bits);
  for (int c = 0; c < npay; c++) {
    const uint64_t p = splitmix64(bits ^ ((uint64_t)c * 0xD1B54A32D192ED03ull));
    store_w(pays[c].base[0] + i * pays[c].width, pays[c].width, p);
  }
}

// ---------------------------------------------------------------------------
// launch wrappers (host side, called from srs_api.hip)
// ---------------------------------------------------------------------------
// KSZ: key size in bytes, | SRS_KS_CANON for the canon-zero float case
#define SRS_KEY_DISPATCH(KSZ, CALL)                              \
  switch (KSZ) {                                                  \
    case 1: CALL(uint8_t, uint32_t, false); break;                \
    case 2: CALL(uint16_t, uint32_t, false); break;               \
    case 4: CALL(uint32_t, uint32_t, false); break;               \
    case 4 | SRS_KS_CANON: CALL(uint32_t, uint32_t, true); break; \
    case 8 | SRS_KS_CANON: CALL(uint64_t, uint64_t, true); break; \
    default: CALL(uint64_t, uint64_t, false); break;              \
  }

void launch_plan(const Seg* big, int64_t nbig, SegPlan* plan, int64_t* tcount,
                 int64_t* gcount, unsigned long long* var_or, uint64_t* elems, int force_bits,
                 int tmp2, hipStream_t st, const int32_t* nt_over) {
  plan_kernel<<<(unsigned)((nbig + 255) / 256), 256, 0, st>>>(
      big, nbig, plan, tcount, gcount, var_or, elems, force_bits, tmp2, nt_over);
}

void launch_plan_small(const Seg* big, int64_t nbig, SegPlan* plan, int64_t* tbase,
                       int64_t* gbase, unsigned long long* var_or, uint64_t* totals,
                       unsigned long long* n_big_next, int force_bits, int tmp2,
                       hipStream_t st, const int32_t* nt_over) {
  plan_small_kernel<<<1, kPlanSmallThreads, 0, st>>>(big, nbig, plan, tbase, gbase, var_or,
                                                     totals, n_big_next, force_bits, tmp2,
                                                     nt_over);
}

void launch_plan_bases(SegPlan* plan, int64_t nbig, const int64_t* tbase,
                       const int64_t* gbase, hipStream_t st) {
  plan_bases_kernel<<<(unsigned)((nbig + 255) / 256), 256, 0, st>>>(plan, nbig, tbase,
                                                                    gbase);
}

void launch_seg_map2(const int64_t* tbase, int64_t ntiles, int32_t* tile_seg,
                     const int64_t* gbase, int64_t ngroups, int32_t* group_seg, int64_t nbig,
                     hipStream_t st) {
  const int64_t n = ntiles + ngroups;
  if (n > 0)
    seg_map2_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(tbase, ntiles, tile_seg, gbase,
                                                                 ngroups, group_seg, nbig);
}

void launch_count(int key_size, const SortDesc* d, const SegPlan* plan,
                  const int32_t* tile_seg, int64_t ntiles, uint16_t* hist,
                  unsigned long long* var_or, unsigned long long* var_and, int lut,
                  hipStream_t st, const GTile* gt, const int32_t* torder) {
  const unsigned grid = (unsigned)((ntiles + kCountTiles - 1) / kCountTiles);
#define CALL(KT, U, CZ)                                                                 \
  if (lut == 2)                                                                         \
    count_kernel<KT, U, 2, CZ><<<grid, kCountThreads, 0, st>>>(                          \
        d, plan, tile_seg, hist, var_or, var_and, gt, ntiles, torder);                           \
  else if (lut)                                                                         \
    count_kernel<KT, U, 1, CZ><<<grid, kCountThreads, 0, st>>>(                          \
        d, plan, tile_seg, hist, var_or, var_and, gt, ntiles, torder);                           \
  else                                                                                  \
    count_kernel<KT, U, 0, CZ><<<grid, kCountThreads, 0, st>>>(                          \
        d, plan, tile_seg, hist, var_or, var_and, gt, ntiles, torder)
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
}

int64_t scan_temp_elems(int64_t n) { return (n + kScanChunk - 1) / kScanChunk + 1; }

void launch_excl_scan(const uint64_t* x, uint64_t* y, int64_t n, uint64_t* temp,
                      uint64_t* total, hipStream_t st) {
  const int64_t nb = (n + kScanChunk - 1) / kScanChunk;
  if (nb > 0) scan_reduce_kernel<<<(unsigned)nb, kScanThreads, 0, st>>>(x, n, temp);
  scan_bsums_kernel<<<1, 1024, 0, st>>>(temp, nb, total);
  if (nb > 0) scan_apply_kernel<<<(unsigned)nb, kScanThreads, 0, st>>>(x, n, temp, y);
}

// SRS_SUPER_SCAN=0: the one-workgroup column scan for every segment (A/B)
bool super_scan_enabled() {
  static const bool on = [] {
    const char* e = getenv("SRS_SUPER_SCAN");
    return !(e && *e == '0');
  }();
  return on;
}

// One large segment (a shard's partition chunk or round sort, any level of
// a single big segment): its column scan is one workgroup, i.e. one CU
// moving ngroups x 6 KB of rows (2348 groups of a 250 M-key chunk: 14 MB,
// 0.17-0.47 ms). Above kSuperMinGroups groups the scan runs
// over sums of kSuperGroups groups instead, and a grid-wide pass turns the
// super offsets back into group offsets.
constexpr int64_t kSuperGroups = 64;
constexpr int64_t kSuperMinGroups = 256;
int64_t g_super_min_groups = kSuperMinGroups;  // (srs_debug_set_super_scan)

void set_super_scan_min_groups(int64_t g) { g_super_min_groups = g > 0 ? g : kSuperMinGroups; }

int64_t super_rows(int64_t ngroups) { return (ngroups + kSuperGroups - 1) / kSuperGroups; }

__global__ __launch_bounds__(kMaxBins) void super_sum_kernel(const SegPlan* __restrict__ plan,
                                                             const uint32_t* __restrict__ gsum,
                                                             int64_t ngroups,
                                                             uint32_t* __restrict__ ssum) {
  const uint32_t b = threadIdx.x;
  if (b >= (1u << plan[0].bits)) return;
  const int64_t g0 = (int64_t)blockIdx.x * kSuperGroups;
  const int64_t g1 = min(g0 + kSuperGroups, ngroups);
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;  // (<= 64 x 32 tiles x 4096 keys: fits 32 bits)
  int64_t g = g0;
  for (; g + 4 <= g1; g += 4) {
    s0 += gsum[(g + 0) * kMaxBins + b];
    s1 += gsum[(g + 1) * kMaxBins + b];
    s2 += gsum[(g + 2) * kMaxBins + b];
    s3 += gsum[(g + 3) * kMaxBins + b];
  }
  for (; g < g1; g++) s0 += gsum[g * kMaxBins + b];
  ssum[(int64_t)blockIdx.x * kMaxBins + b] = s0 + s1 + s2 + s3;
}

__global__ __launch_bounds__(kMaxBins) void super_apply_kernel(const SegPlan* __restrict__ plan,
                                                               const uint32_t* __restrict__ gsum,
                                                               int64_t ngroups,
                                                               const uint64_t* __restrict__ sofs,
                                                               uint64_t* __restrict__ gofs) {
  const uint32_t b = threadIdx.x;
  if (plan[0].skip || b >= (1u << plan[0].bits)) return;
  const int64_t g0 = (int64_t)blockIdx.x * kSuperGroups;
  const int64_t g1 = min(g0 + kSuperGroups, ngroups);
  uint64_t run = sofs[(int64_t)blockIdx.x * kMaxBins + b];
  for (int64_t g = g0; g < g1; g++) {
    gofs[g * kMaxBins + b] = run;
    run += gsum[g * kMaxBins + b];
  }
}

void launch_offsets(SegPlan* plan, int64_t nbig, const int32_t* group_seg, int64_t ngroups,
                    const uint16_t* hist, uint32_t* gsum, uint64_t* gofs, uint64_t* sbase,
                    uint64_t* offs, uint32_t* offs32, const unsigned long long* var_or,
                    Seg* big_next,
                    Seg* local, Seg* local2, Seg* copy, ListCounters* ctr,
                    const int32_t* lut_rbits, hipStream_t st, int mode, uint32_t* prun) {
  group_sum_kernel<<<(unsigned)ngroups, kMaxBins, 0, st>>>(plan, group_seg, hist, gsum);
  if (nbig == 1 && mode != 1 && ngroups >= g_super_min_groups && super_scan_enabled()) {
    // (the super rows live behind the group rows: the caller sizes gsum and
    // gofs for ngroups + super_rows(ngroups) rows)
    const int64_t ns = super_rows(ngroups);
    uint32_t* ssum = gsum + ngroups * kMaxBins;
    uint64_t* sofs = gofs + ngroups * kMaxBins;
    super_sum_kernel<<<(unsigned)ns, kMaxBins, 0, st>>>(plan, gsum, ngroups, ssum);
    seg_scan_kernel<<<1, kMaxBins, 0, st>>>(plan, ssum, sofs, sbase, var_or, big_next, local,
                                            local2, copy, ctr, lut_rbits, mode, prun, ns);
    super_apply_kernel<<<(unsigned)ns, kMaxBins, 0, st>>>(plan, gsum, ngroups, sofs, gofs);
  } else {
    seg_scan_kernel<<<(unsigned)nbig, kMaxBins, 0, st>>>(plan, gsum, gofs, sbase, var_or,
                                                        big_next, local, local2, copy, ctr,
                                                        lut_rbits, mode, prun, 0);
  }
  tile_offs_kernel<<<(unsigned)ngroups, kMaxBins, 0, st>>>(
      plan, group_seg, hist, gofs, sbase, offs, offs32);
}

void launch_scatter(int key_size, const SortDesc* d, const SegPlan* plan,
                    const int32_t* tile_seg, const uint64_t* offs, const uint32_t* offs32,
                    int64_t ntiles, int lut, int ncols, hipStream_t st, const GTile* gt) {
  const bool pre3 = ncols >= 3;
#define CALL_L(KT, U, CZ, LK)                                                           \
  if (pre3)                                                                             \
    scatter_kernel<KT, U, LK, CZ, true><<<(unsigned)ntiles, kScatterThreads, 0, st>>>(    \
        d, plan, tile_seg, offs, offs32, gt);                                           \
  else                                                                                  \
    scatter_kernel<KT, U, LK, CZ, false><<<(unsigned)ntiles, kScatterThreads, 0, st>>>(   \
        d, plan, tile_seg, offs, offs32, gt)
#define CALL(KT, U, CZ)                                                                 \
  if (lut == 2) {                                                                       \
    CALL_L(KT, U, CZ, 2);                                                               \
  } else if (lut) {                                                                     \
    CALL_L(KT, U, CZ, 1);                                                               \
  } else {                                                                              \
    CALL_L(KT, U, CZ, 0);                                                               \
  }
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
#undef CALL_L
}

void launch_scatter_pairs(int key_size, const SortDesc* d, const SegPlan* plan,
                          const int32_t* tile_seg, const uint64_t* offs, const uint32_t* offs32,
                          int64_t ntiles, int lut, hipStream_t st, const GTile* gt) {
  const unsigned grid = (unsigned)((ntiles + 1) / 2);
#define CALL_P(KT, U, LK)                                                            \
  scatter_pair_kernel<KT, U, LK><<<grid, kPairThreads, 0, st>>>(d, plan, tile_seg, offs, \
                                                               offs32, gt, ntiles)
  if (key_size == 4) {
    if (lut == 2) CALL_P(uint32_t, uint32_t, 2);
    else CALL_P(uint32_t, uint32_t, 0);
  } else {
    if (lut == 2) CALL_P(uint64_t, uint64_t, 2);
    else CALL_P(uint64_t, uint64_t, 0);
  }
#undef CALL_P
}

void launch_stripe_tables(const uint32_t* prun, int64_t nstripes, int nb, uint32_t* ptile,
                          uint64_t* btot, uint32_t* bnt, int rbits, int buf, Seg* big,
                          int32_t* nt_over, uint32_t* btile, ListCounters* ctr,
                          const uint64_t* sbase, const SegPlan* plan, GTile* gt,
                          const int32_t* lut_rbits, hipStream_t st, int32_t* torder,
                          int64_t tiles_cap) {
  stripe_tiles_kernel<<<(unsigned)nb, kStripeThreads, 0, st>>>(prun, nstripes, ptile, btot, bnt);
  stripe_segs_kernel<<<1, kMaxBins, 0, st>>>(btot, bnt, nb, rbits, buf, big, nt_over, btile, ctr,
                                             lut_rbits);
  const int64_t np = nstripes * nb;
  stripe_gtile_kernel<<<(unsigned)((np + 255) / 256), 256, 0, st>>>(prun, ptile, btile, sbase,
                                                                    plan, nstripes, nb, gt);
  if (torder) {
    uint32_t* rowtot = (uint32_t*)(torder + tiles_cap);
    stripe_rows_kernel<<<(unsigned)nstripes, kMaxBins, 0, st>>>(prun, nb, rowtot);
    stripe_order_kernel<<<(unsigned)nstripes, kMaxBins, 0, st>>>(prun, ptile, btile, rowtot, nb,
                                                                 torder);
  }
}

void launch_local(int key_size, const SortDesc* d, const Seg* segs, int64_t nsegs, int big_class,
                  Seg* fallback, unsigned long long* fallback_count, hipStream_t st,
                  bool rec16) {
#define CALL_R(KT, U, CZ, R)                                                                \
  if (big_class)                                                                            \
    local_kernel<KT, U, kLocalThreads, kLocalItems, kLocalWavesPerEU, CZ, R>                \
        <<<(unsigned)nsegs, kLocalThreads, 0, st>>>(d, segs, fallback, fallback_count);     \
  else                                                                                      \
    local_kernel<KT, U, kLocalThreadsSmall, kLocalItemsSmall, kLocalWavesPerEUSmall, CZ, R> \
        <<<(unsigned)nsegs, kLocalThreadsSmall, 0, st>>>(d, segs, fallback, fallback_count)
#define CALL(KT, U, CZ) \
  if (rec16) { CALL_R(KT, U, CZ, true); } else { CALL_R(KT, U, CZ, false); }
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
#undef CALL_R
}

void launch_local_direct(int key_size, int pm, const SortDesc* d, const Seg* segs,
                         int64_t nsegs, Seg* redo, unsigned long long* redo_count, Seg* fallback,
                         unsigned long long* fallback_count, hipStream_t st, bool big) {
#define CALL(KT, PM)                                                                          \
  if (big)                                                                                    \
    local_direct_kernel<KT, KT, kLocalDirectThreads2, kLocalDirectItems2,                     \
                        kLocalDirectWavesPerEU2, PM>                                          \
        <<<(unsigned)nsegs, kLocalDirectThreads2, 0, st>>>(d, segs, redo, redo_count,         \
                                                           fallback, fallback_count, xcd);    \
  else                                                                                        \
    local_direct_kernel<KT, KT, kLocalDirectThreads, kLocalDirectItems,                       \
                        kLocalDirectWavesPerEU, PM>                                           \
        <<<(unsigned)nsegs, kLocalDirectThreads, 0, st>>>(d, segs, redo, redo_count,          \
                                                          fallback, fallback_count, xcd)
  // consecutive list entries on one XCD (SRS_LOCAL_XCD=0: plain order, for
  // A/B runs): C1 local 6.19-6.24 ms vs 5.95-6.56 in list order, same box
  static const int xcd = [] {
    const char* e = getenv("SRS_LOCAL_XCD");
    return (e && *e == '0') ? 0 : 1;
  }();
  if (pm == 1) {
    CALL(uint64_t, 1);
  } else if (pm == 2) {
    CALL(uint32_t, 2);
  } else if (key_size == 4) {
    CALL(uint32_t, 0);
  } else {
    CALL(uint64_t, 0);
  }
#undef CALL
}

void launch_local_list(int key_size, const SortDesc* d, const Seg* segs,
                       const unsigned long long* nsegs, int grid, Seg* fallback,
                       unsigned long long* fallback_count, hipStream_t st, bool big) {
  if (big && key_size == 4)
    local_list_kernel<uint32_t, uint32_t, kLocalThreads, kLocalItems, kLocalWavesPerEU>
        <<<(unsigned)grid, kLocalThreads, 0, st>>>(d, segs, nsegs, fallback, fallback_count);
  else if (big)
    local_list_kernel<uint64_t, uint64_t, kLocalThreads, kLocalItems, kLocalWavesPerEU>
        <<<(unsigned)grid, kLocalThreads, 0, st>>>(d, segs, nsegs, fallback, fallback_count);
  else if (key_size == 4)
    local_list_kernel<uint32_t, uint32_t, kLocalThreadsSmall, kLocalItemsSmall,
                      kLocalWavesPerEUSmall>
        <<<(unsigned)grid, kLocalThreadsSmall, 0, st>>>(d, segs, nsegs, fallback, fallback_count);
  else
    local_list_kernel<uint64_t, uint64_t, kLocalThreadsSmall, kLocalItemsSmall,
                      kLocalWavesPerEUSmall>
        <<<(unsigned)grid, kLocalThreadsSmall, 0, st>>>(d, segs, nsegs, fallback, fallback_count);
}

void launch_local_stable(int key_size, const SortDesc* d, const Seg* segs,
                         const unsigned long long* nsegs, int big_class, Seg* fallback,
                         unsigned long long* fallback_count, int grid, hipStream_t st) {
#define CALL(KT, U, CZ)                                                                \
  if (big_class)                                                                       \
    local_stable_kernel<KT, U, kLocalStableThreads, CZ>                                \
        <<<(unsigned)grid, kLocalStableThreads, 0, st>>>(d, segs, nsegs, fallback,      \
                                                         fallback_count);              \
  else                                                                                 \
    local_stable_kernel<KT, U, kLocalStableThreadsSmall, CZ>                           \
        <<<(unsigned)grid, kLocalStableThreadsSmall, 0, st>>>(d, segs, nsegs, fallback, \
                                                             fallback_count)
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
}

void launch_local_lsd(int key_size, const SortDesc* d, const Seg* segs,
                      const unsigned long long* nsegs, int grid, hipStream_t st) {
#define CALL(KT, U, CZ) \
  local_lsd_kernel<KT, U, CZ><<<(unsigned)grid, kLocalStableThreads, 0, st>>>(d, segs, nsegs)
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
}

int mid_bar_words() { return kMidBarWords; }
int64_t mid_part_bytes(int64_t n) {  // (part: 2 words per tile, >= 1 word per bucket)
  return std::max<int64_t>((n + kTile - 1) / kTile, kMidMaxTiles) * 16;
}

hipError_t launch_mid_sort(int key_size, const SortDesc& d, int64_t n, int src,
                           unsigned long long* part, uint32_t* hist, ListCounters* ctr, Seg* big,
                           unsigned long long* taken, MidFlag* flag, unsigned long long seq,
                           unsigned long long* bar, hipStream_t st) {
  const unsigned T = (unsigned)((n + kTile - 1) / kTile);
  const unsigned nb_max = 1u << std::min(choose_bits(n, 64), kMidMaxBits);
  if (T > (unsigned)kMidMaxTiles) return hipErrorInvalidValue;
  const unsigned G = std::max(T, nb_max);  // (one bucket per workgroup)
  const int wide = T * nb_max > (unsigned)kMidMat ? 1 : 0;  // (phase 2b)
  // every workgroup must be resident at once (the grid barriers): G within
  // the device's CUs x the kernel's resident workgroups per CU, else the
  // caller takes the general path (e.g. a partition of a few CUs). Cached
  // per device and key dispatch (the query costs microseconds per call).
  static std::atomic<int> cap_cache[64][6];  // [device][instantiation]; 0: not queried yet
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidValue;
  const int kb = key_size & 0xff;
  const int slot = (key_size & SRS_KS_CANON) ? (kb == 4 ? 4 : 5) : kb == 1 ? 0 : kb == 2 ? 1 : kb == 4 ? 2 : 3;
  int resident = cap_cache[dev][slot].load(std::memory_order_relaxed);
  if (resident == 0) {
    int cus = 0, per_cu = 0;
    hipError_t oe = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
#define OCC(KT, U, CZ)                                                                            \
  if (oe == hipSuccess)                                                                          \
    oe = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, mid_sort_kernel<KT, U, CZ>,       \
                                                      kLocalThreads, 0)
    SRS_KEY_DISPATCH(key_size, OCC)
#undef OCC
    if (oe != hipSuccess) return oe;
    resident = std::max(1, cus * per_cu);  // (>= 1: "queried")
    if (per_cu < 1) resident = -1;
    cap_cache[dev][slot].store(resident, std::memory_order_relaxed);
  }
  if (resident < 0 || (int64_t)G > (int64_t)resident) return hipErrorCooperativeLaunchTooLarge;
#define CALL(KT, U, CZ)                                                                         \
  mid_sort_kernel<KT, U, CZ><<<G, kLocalThreads, 0, st>>>(d, n, src, part, hist, ctr, big,    \
                                                          taken, flag, seq, bar, wide);       \
  return hipGetLastError()
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
  return hipErrorInvalidValue;
}

int64_t mid_level_part_bytes() { return (int64_t)(kMaxBins + 2 * kMidLevelMaxTiles) * 8; }

hipError_t launch_mid_level(int key_size, const SortDesc& d, int64_t n, int src,
                            unsigned long long* part, uint32_t* hist, ListCounters* ctr, Seg* big,
                            Seg* local, Seg* local2, Seg* copy, SortDesc* d_out, MidFlag* flag,
                            unsigned long long seq, unsigned long long* bar, hipStream_t st) {
  const int64_t T = (n + kTile - 1) / kTile;
  if (n <= 0 || T > kMidLevelMaxTiles) return hipErrorInvalidValue;
  // the grid: as many workgroups as stay resident together (the grid
  // barriers), at most one per tile; cached per device and key dispatch
  static std::atomic<int> cap_cache[64][6];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidValue;
  const int kb = key_size & 0xff;
  const int slot = (key_size & SRS_KS_CANON) ? (kb == 4 ? 4 : 5) : kb == 1 ? 0 : kb == 2 ? 1 : kb == 4 ? 2 : 3;
  int resident = cap_cache[dev][slot].load(std::memory_order_relaxed);
  if (resident == 0) {
    int cus = 0, per_cu = 0;
    hipError_t oe = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
#define OCC(KT, U, CZ)                                                                            \
  if (oe == hipSuccess)                                                                          \
    oe = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, mid_level_kernel<KT, U, CZ>,      \
                                                      kScatterThreads, 0)
    SRS_KEY_DISPATCH(key_size, OCC)
#undef OCC
    if (oe != hipSuccess) return oe;
    resident = std::max(1, cus * per_cu);
    if (per_cu < 1) resident = -1;
    cap_cache[dev][slot].store(resident, std::memory_order_relaxed);
  }
  if (resident < 0) return hipErrorCooperativeLaunchTooLarge;
  const unsigned G = (unsigned)std::min<int64_t>(T, resident);
#define CALL(KT, U, CZ)                                                                          \
  mid_level_kernel<KT, U, CZ><<<G, kScatterThreads, 0, st>>>(d, n, src, part, hist, ctr, big,   \
                                                             local, local2, copy, d_out, flag,  \
                                                             seq, bar);                         \
  return hipGetLastError()
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
  return hipErrorInvalidValue;
}

void launch_small_sort(int key_size, const SortDesc& d, Seg g, int64_t* taken, hipStream_t st) {
  static_assert(kLocalThreads == 1024, "the small sort's shapes");
  const int64_t n = g.len;
#define CALL(KT, U, CZ)                                                       \
  do {                                                                        \
    if (n <= 128 * kLocalItems)                                               \
      small_sort_kernel<KT, U, CZ, 128><<<1, 128, 0, st>>>(d, g, taken);      \
    else if (n <= 256 * kLocalItems)                                          \
      small_sort_kernel<KT, U, CZ, 256><<<1, 256, 0, st>>>(d, g, taken);      \
    else if (n <= 512 * kLocalItems)                                          \
      small_sort_kernel<KT, U, CZ, 512><<<1, 512, 0, st>>>(d, g, taken);      \
    else                                                                      \
      small_sort_kernel<KT, U, CZ, 1024><<<1, 1024, 0, st>>>(d, g, taken);    \
  } while (0)
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
}

// ---------------------------------------------------------------------------
// placement probe: the scatter's write pattern over a whole buffer
// ---------------------------------------------------------------------------
// A tile (256 threads) writes 4096 8-byte elements as 512 runs of 8 into 512
// buckets of a 16 MB window: bucket r of window w starts at a hashed
// 8-byte-aligned offset near r * 32 KB (as a C1 level's children do), tile i
// of the window fills the i-th run of every bucket; windows in order, tiles
// XCD-contiguous (xcd_remap). How fast this runs over a buffer says how fast
// the scatter and local passes will write it.
constexpr int64_t kProbeWindow = int64_t(16) << 20;
__global__ __launch_bounds__(256) void place_probe_kernel(char* __restrict__ buf, int64_t windows) {
  constexpr int kRuns = 512, kRunKeys = 8;
  constexpr int64_t kSpan = kProbeWindow / kRuns;      // 32 KB per bucket
  constexpr int64_t kTiles = kSpan / (kRunKeys * 8) / 2; // tiles per window (half of the span)
  const int64_t t = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t w = t / kTiles, i = t % kTiles;
  if (w >= windows) return;
  const uint64_t v = (uint64_t)t * 0x9E3779B97F4A7C15ull;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int e = k * 256 + (int)threadIdx.x;  // element of the tile
    const int r = e >> 3, o = e & 7;
    // bucket start: r * span + hash(r) * 8 inside the unused half of the span
    const uint32_t hsh = (uint32_t)r * 2654435761u;
    const int64_t start = r * kSpan + (int64_t)((hsh >> 20) % (uint32_t)(kSpan / 16)) * 8;
    uint64_t* dst = (uint64_t*)(buf + w * kProbeWindow + start) + i * kRunKeys + o;
    *dst = v + (uint64_t)e;
  }
}

// Average milliseconds of one probe pass over [buf, buf + bytes) (2 passes
// after one warmup, on stream st; synchronous on st only).
float probe_write_ms(void* buf, size_t bytes, hipStream_t st) {
  const int64_t windows = (int64_t)(bytes / kProbeWindow);
  if (windows < 1) return 0.f;
  constexpr int64_t kTiles = kProbeWindow / 512 / 64 / 2;
  const unsigned grid = (unsigned)(windows * kTiles);
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess) return 0.f;
  if (hipEventCreate(&b) != hipSuccess) {
    (void)hipEventDestroy(a);
    return 0.f;
  }
  place_probe_kernel<<<grid, 256, 0, st>>>((char*)buf, windows);
  (void)hipEventRecord(a, st);
  for (int k = 0; k < 2; k++) place_probe_kernel<<<grid, 256, 0, st>>>((char*)buf, windows);
  (void)hipEventRecord(b, st);
  float ms = 0.f;
  if (hipEventSynchronize(b) != hipSuccess || hipEventElapsedTime(&ms, a, b) != hipSuccess) ms = 0.f;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / 2;
}

void launch_fill(int64_t n, int kind, uint64_t seed, uint64_t first, void* keys,
                 int npay, const Col* pays, hipStream_t st) {
  fill_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, kind, seed, first,
                                                           (char*)keys, npay, pays);
}

}  // namespace srs

namespace srs {

// Histogram of the transformed top `bits` bits (multi-GPU shard split).
template <typename KT, typename U>
__global__ __launch_bounds__(256) void key_hist_kernel(int64_t n, const KT* __restrict__ keys,
                                                       SortDesc d, int bits,
                                                       unsigned long long* __restrict__ hist) {
  __shared__ uint32_t h[1 << kHistMaxBits];
  const int nb = 1 << bits;
  const int shift = d.key_bits - bits;
  Xform<U> xf;
  xf.init(d);
  for (int i = threadIdx.x; i < nb; i += 256) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    atomicAdd(&h[(uint32_t)(xf((U)keys[i]) >> shift)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += 256)
    if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

void launch_key_hist(int key_size, int64_t n, const void* keys, const SortDesc& d, int bits,
                     unsigned long long* hist, hipStream_t st) {
  const int grid = (int)std::min<int64_t>(2048, (n + 255) / 256);
#define CALL(KT, U, CZ) \
  key_hist_kernel<KT, U><<<grid, 256, 0, st>>>(n, (const KT*)keys, d, bits, hist)
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
}

// Kernel arguments are captured at launch, so the descriptor needs no pinned
// staging buffer and is safe to rebuild for the next call immediately.
// The descriptor (~3.5 KB) copied by every thread of the block, a dword
// each: as one lane's struct copy it took a few microseconds of the start
// kernel's 8.5 (a 1M-key call is launch-bound)
static_assert(sizeof(SortDesc) % 4 == 0, "dword copy of the descriptor");
__device__ __forceinline__ void copy_desc(const SortDesc& d, SortDesc* out) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&d);
  uint32_t* dst = reinterpret_cast<uint32_t*>(out);
  for (uint32_t i = threadIdx.x; i < sizeof(SortDesc) / 4; i += blockDim.x) dst[i] = src[i];
}

__global__ void set_desc_kernel(SortDesc d, SortDesc* out) { copy_desc(d, out); }

__device__ __forceinline__ void init_lists_body(Seg seg0, int to_local, Seg* big, Seg* local,
                                                Seg* local2, ListCounters* ctr) {
  if (threadIdx.x == 0) {
    ctr->n_big = to_local ? 0 : 1;
    const bool small = seg0.len <= kLocalCapSmall;
    ctr->n_local = (to_local && small) ? 1 : 0;
    ctr->n_local2 = (to_local && !small) ? 1 : 0;
    ctr->n_copy = 0;
    ctr->n_fallback = 0;
    ctr->n_fallback1 = 0;
    ctr->n_fallback2 = 0;
    ctr->n_redo = 0;
    ctr->n_redo2 = 0;
    ctr->local_elems = to_local ? (unsigned long long)seg0.len : 0;
    if (to_local) (small ? local : local2)[0] = seg0; else big[0] = seg0;
  }
}


// Finished segments home: every segment of the copy list (finished, not in
// OUT) is moved to OUT in one launch, column by column with each buffer's
// stride. (A hipMemcpyAsync per segment and column cost ~5 us each:
// duplicate-heavy inputs finish hundreds of large segments at once.) The
// segments are cut into chunks of kCopyChunk records and a fixed grid walks
// the chunks of all segments (a device prefix sum of chunk counts maps a
// chunk to its segment), so a long segment among many short ones gets the
// whole grid instead of its share of a per-segment split, and the list never
// travels to the host.
constexpr int kCopyChunk = 4096;
constexpr int kCopyGrid = 2048;

__global__ void copy_chunks_kernel(const Seg* __restrict__ segs, int64_t nsegs,
                                   uint64_t* __restrict__ chunks) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nsegs) chunks[i] = (uint64_t)((segs[i].len + kCopyChunk - 1) / kCopyChunk);
}

__global__ __launch_bounds__(256) void copy_list_kernel(const SortDesc* __restrict__ desc,
                                                        const Seg* __restrict__ segs,
                                                        int64_t nsegs,
                                                        const uint64_t* __restrict__ cbase,
                                                        const uint64_t* __restrict__ total) {
  const uint64_t nchunks = *total;
  const int ncols = desc->ncols;
  for (uint64_t w = blockIdx.x; w < nchunks; w += gridDim.x) {
    // the segment holding chunk w: the last s with cbase[s] <= w
    int64_t lo = 0, hi = nsegs - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (cbase[mid] <= w) lo = mid;
      else hi = mid - 1;
    }
    const Seg g = segs[lo];
    const int64_t first = (int64_t)(w - cbase[lo]) * kCopyChunk;
    const int64_t cnt = min((int64_t)kCopyChunk, g.len - first);
    for (int c = 0; c < ncols; c++) {
      const Col& C = desc->cols[c];
      const uint32_t si = C.stride[g.buf], so = C.stride[BUF_OUT];
      const char* src = C.base[g.buf] + (g.start + first) * (int64_t)si;
      char* dst = C.base[BUF_OUT] + (g.start + first) * (int64_t)so;
      with_width(C.width, [&](auto W_) {
        constexpr int W = decltype(W_)::value;
        for (int64_t i = threadIdx.x; i < cnt; i += 256) stw<W>(dst + i * so, ldw<W>(src + i * si));
      });
    }
  }
}

void launch_copy_list(const SortDesc* d, const Seg* segs, int64_t nsegs, uint64_t* chunks,
                      uint64_t* cbase, uint64_t* scan_temp, uint64_t* total, hipStream_t st) {
  if (nsegs <= 0) return;
  copy_chunks_kernel<<<(unsigned)((nsegs + 255) / 256), 256, 0, st>>>(segs, nsegs, chunks);
  launch_excl_scan(chunks, cbase, nsegs, scan_temp, total, st);
  copy_list_kernel<<<kCopyGrid, 256, 0, st>>>(d, segs, nsegs, cbase, total);
}

void set_xcd_rotation(int mode) {
  static int cur = 0;
  if (mode == cur) return;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_xcd_rot), &mode, sizeof(int));
  cur = mode;
}

void launch_set_desc(const SortDesc& d, SortDesc* out, hipStream_t st) {
  set_desc_kernel<<<1, 256, 0, st>>>(d, out);
}

// set_desc + init_lists in one launch (a small sort is launch-bound)
__global__ void start_kernel(SortDesc d, SortDesc* out, Seg seg0, int to_local, Seg* big,
                             Seg* local, Seg* local2, ListCounters* ctr) {
  copy_desc(d, out);
  init_lists_body(seg0, to_local, big, local, local2, ctr);
}

void launch_start(const SortDesc& d, SortDesc* out, Seg seg0, int to_local, Seg* big, Seg* local,
                  Seg* local2, ListCounters* ctr, hipStream_t st) {
  start_kernel<<<1, 256, 0, st>>>(d, out, seg0, to_local, big, local, local2, ctr);
}


}  // namespace srs

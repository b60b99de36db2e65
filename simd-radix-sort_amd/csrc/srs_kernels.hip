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

#include "srs_common.h"
#include "srs_kernels.h"

namespace srs {

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t load_w(const char* p, uint32_t w) {
  switch (w) {
    case 1: return *(const uint8_t*)p;
    case 2: return *(const uint16_t*)p;
    case 4: return *(const uint32_t*)p;
    default: return *(const uint64_t*)p;
  }
}

__device__ __forceinline__ void store_w(char* p, uint32_t w, uint64_t v) {
  switch (w) {
    case 1: *(uint8_t*)p = (uint8_t)v; break;
    case 2: *(uint16_t*)p = (uint16_t)v; break;
    case 4: *(uint32_t*)p = (uint32_t)v; break;
    default: *(uint64_t*)p = v; break;
  }
}

// Key transform (the reference's bitDirUp table, radixSort.hpp:1568-1581,
// folded into one xor): unsigned order of u == the reference's key order.
template <typename U>
struct Xform {
  U mpos, mneg, signbit, negzero;
  bool canon;
  __device__ __forceinline__ void init(const SortDesc& d) {
    mpos = (U)d.mpos;
    mneg = (U)d.mneg;
    signbit = (U)d.signbit;
    negzero = (U)d.negzero;
    canon = d.canon_zero != 0;
  }
  __device__ __forceinline__ U operator()(U bits) const {
    if (canon && bits == negzero) bits = 0;
    return bits ^ ((bits & signbit) ? mneg : mpos);
  }
};

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }

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

// Wave-level multisplit rank (stable): for each item slot k, lanes whose
// digit matches form a peer group found with `nbits` ballots; the rank of a
// key is the wave's running count of its digit (per-wave LDS counter row
// `wc`) plus the number of lower-lane peers. Items are in striped order
// (slot k of lane l = wave-local element k * 64 + l), so ranks follow input
// order within a digit.
template <int ITEMS>
__device__ __forceinline__ void wlms_rank(const uint32_t (&dig)[ITEMS],
                                          const bool (&valid)[ITEMS], int nbits,
                                          uint16_t* wc, uint32_t (&rank)[ITEMS]) {
  const uint64_t lt = (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
#pragma unroll
  for (int k = 0; k < ITEMS; k++) {
    uint64_t peers = __ballot(valid[k]);
    const uint32_t d = dig[k];
#pragma unroll
    for (int b = 0; b < kMaxDigitBits; b++) {
      if (b < nbits) {
        const bool bit = (d >> b) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
    }
    if (valid[k]) {
      const uint32_t below = (uint32_t)__popcll(peers & lt);
      const uint32_t base = wc[d];
      rank[k] = base + below;
      if (below == 0) wc[d] = (uint16_t)(base + (uint32_t)__popcll(peers));
    }
  }
}

// ---------------------------------------------------------------------------
// plan / bookkeeping kernels
// ---------------------------------------------------------------------------

// Digit width for a segment of `len` keys with `rbits` unsorted bits: as many
// bits as needed to bring buckets under kLocalTarget, spread evenly over the
// levels that will take, at most kMaxDigitBits per level.
__device__ __forceinline__ int choose_bits(int64_t len, int rbits) {
  int need = 1;
  while (need < 62 && ((int64_t)kLocalTarget << need) < len) need++;
  const int levels = (need + kMaxDigitBits - 1) / kMaxDigitBits;
  int bits = (need + levels - 1) / levels;
  if (bits > kMaxDigitBits) bits = kMaxDigitBits;
  if (bits > rbits) bits = rbits;
  if (bits < 1) bits = 1;
  return bits;
}

__global__ void plan_kernel(const Seg* __restrict__ big, int64_t nbig,
                            SegPlan* __restrict__ plan, int64_t* __restrict__ tcount,
                            int64_t* __restrict__ hcount,
                            unsigned long long* __restrict__ var_or,
                            uint64_t* __restrict__ elems) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nbig) return;
  const Seg g = big[s];
  atomicAdd((unsigned long long*)elems, (unsigned long long)g.len);
  SegPlan p;
  p.start = g.start;
  p.len = g.len;
  p.bits = choose_bits(g.len, g.rbits);
  p.shift = g.rbits - p.bits;
  p.ntiles = (int32_t)((g.len + kTile - 1) / kTile);
  p.buf = g.buf;
  p.dst = (g.buf == BUF_TMP) ? BUF_OUT : BUF_TMP;
  p.skip = 0;
  p.tile_base = 0;
  p.hist_base = 0;
  plan[s] = p;
  tcount[s] = p.ntiles;
  hcount[s] = (int64_t)p.ntiles << p.bits;
  var_or[s] = 0;
}

__global__ void plan_bases_kernel(SegPlan* __restrict__ plan, int64_t nbig,
                                  const int64_t* __restrict__ tbase,
                                  const int64_t* __restrict__ hbase) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nbig) return;
  plan[s].tile_base = tbase[s];
  plan[s].hist_base = hbase[s];
}

// tile -> segment (binary search over the segments' tile bases).
__global__ void tile_map_kernel(const SegPlan* __restrict__ plan, int64_t nbig,
                                int64_t ntiles, int32_t* __restrict__ tile_seg) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  int64_t lo = 0, hi = nbig - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (plan[mid].tile_base <= t) lo = mid; else hi = mid - 1;
  }
  tile_seg[t] = (int32_t)lo;
}

// ---------------------------------------------------------------------------
// count: per-tile digit histogram (bin-major per segment) + varying bits
// ---------------------------------------------------------------------------
template <typename KT, typename U>
__global__ __launch_bounds__(kScatterThreads) void count_kernel(
    const SortDesc* __restrict__ desc, const SegPlan* __restrict__ plan,
    const int32_t* __restrict__ tile_seg, uint64_t* __restrict__ hist,
    unsigned long long* __restrict__ var_or) {
  __shared__ uint32_t h[kMaxBins];
  __shared__ unsigned long long sh_or;
  const int64_t t = blockIdx.x;
  const int32_t s = tile_seg[t];
  const SegPlan P = plan[s];
  const int64_t tl = t - P.tile_base;
  const uint32_t nb = 1u << P.bits;
  const uint32_t mask = nb - 1;
  Xform<U> xf;
  xf.init(*desc);
  const char* kp = desc->key.base[P.buf];
  const uint32_t ks = desc->key.stride;

  for (uint32_t i = threadIdx.x; i < nb; i += kScatterThreads) h[i] = 0;
  if (threadIdx.x == 0) sh_or = 0;
  __syncthreads();

  const int64_t base = P.start + tl * kTile;
  const int64_t rem = P.len - tl * kTile;
  const int cnt = rem < kTile ? (int)rem : kTile;
  const U uref = xf((U) * (const KT*)(kp + P.start * (int64_t)ks));
  U raw[kScatterItems];
#pragma unroll
  for (int k = 0; k < kScatterItems; k++) {
    const int e = k * kScatterThreads + threadIdx.x;
    raw[k] = e < cnt ? (U) * (const KT*)(kp + (base + e) * (int64_t)ks) : (U)0;
  }
  U vor = 0;
#pragma unroll
  for (int k = 0; k < kScatterItems; k++) {
    const int e = k * kScatterThreads + threadIdx.x;
    if (e < cnt) {
      const U u = xf(raw[k]);
      atomicAdd(&h[(uint32_t)(u >> P.shift) & mask], 1u);
      vor |= u ^ uref;
    }
  }
  if (vor) atomicOr(&sh_or, (unsigned long long)vor);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nb; i += kScatterThreads)
    hist[P.hist_base + (int64_t)i * P.ntiles + tl] = h[i];
  if (threadIdx.x == 0 && sh_or) atomicOr(&var_or[s], sh_or);
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
  Seg* local;
  Seg* copy;
  ListCounters* ctr;
};

__device__ __forceinline__ void emit_child(const Lists& L, Seg c) {
  if (c.len <= 0) return;
  if (c.rbits == 0 || c.len == 1) {
    if (c.buf == BUF_OUT) return;  // finished in place
    if (c.len <= kLocalCap) {
      L.local[atomicAdd(&L.ctr->n_local, 1ull)] = c;
      atomicAdd(&L.ctr->local_elems, (unsigned long long)c.len);
    } else {
      L.copy[atomicAdd(&L.ctr->n_copy, 1ull)] = c;
    }
  } else if (c.len <= kLocalCap) {
    L.local[atomicAdd(&L.ctr->n_local, 1ull)] = c;
    atomicAdd(&L.ctr->local_elems, (unsigned long long)c.len);
  } else {
    L.big[atomicAdd(&L.ctr->n_big, 1ull)] = c;
  }
}

__global__ __launch_bounds__(512) void children_kernel(
    SegPlan* __restrict__ plan, const uint64_t* __restrict__ offs,
    const unsigned long long* __restrict__ var_or, Seg* big_next, Seg* local,
    Seg* copy, ListCounters* ctr) {
  __shared__ int single;
  const int64_t s = blockIdx.x;
  const SegPlan P = plan[s];
  const uint32_t nb = 1u << P.bits;
  const uint64_t seg0 = offs[P.hist_base];
  if (threadIdx.x == 0) single = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
    const int64_t off = (int64_t)(offs[P.hist_base + (int64_t)i * P.ntiles] - seg0);
    const int64_t end = (i + 1 < nb)
        ? (int64_t)(offs[P.hist_base + (int64_t)(i + 1) * P.ntiles] - seg0) : P.len;
    if (end - off == P.len) single = 1;
  }
  __syncthreads();
  Lists L{big_next, local, copy, ctr};
  if (single) {
    if (threadIdx.x == 0) {
      plan[s].skip = 1;
      const unsigned long long v = var_or[s];
      Seg c;
      c.start = P.start;
      c.len = P.len;
      c.rbits = v ? 64 - __clzll((long long)v) : 0;
      if (c.rbits > P.shift) c.rbits = P.shift;  // cannot happen; defensive
      c.buf = P.buf;
      emit_child(L, c);
    }
    return;
  }
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
    const int64_t off = (int64_t)(offs[P.hist_base + (int64_t)i * P.ntiles] - seg0);
    const int64_t end = (i + 1 < nb)
        ? (int64_t)(offs[P.hist_base + (int64_t)(i + 1) * P.ntiles] - seg0) : P.len;
    Seg c;
    c.start = P.start + off;
    c.len = end - off;
    c.rbits = P.shift;
    c.buf = P.dst;
    emit_child(L, c);
  }
}

// ---------------------------------------------------------------------------
// scatter: rank one tile by digit, stage in LDS, write coalesced runs
// ---------------------------------------------------------------------------
template <typename KT, typename U>
__global__ __launch_bounds__(kScatterThreads) void scatter_kernel(
    const SortDesc* __restrict__ desc, const SegPlan* __restrict__ plan,
    const int32_t* __restrict__ tile_seg, const uint64_t* __restrict__ offs) {
  constexpr int NT = kScatterThreads;
  constexpr int IT = kScatterItems;
  constexpr int NW = NT / 64;
  __shared__ uint64_t sval[kTile];
  __shared__ uint16_t sbin[kTile];
  __shared__ uint16_t wc[NW][kMaxBins];
  __shared__ uint32_t bin_start[kMaxBins];
  __shared__ int64_t gdst[kMaxBins];
  __shared__ uint32_t scan_sh[NW + 1];

  const int64_t t = blockIdx.x;
  const int32_t s = tile_seg[t];
  const SegPlan P = plan[s];
  if (P.skip) return;
  const int64_t tl = t - P.tile_base;
  const uint32_t nb = 1u << P.bits;
  const uint32_t mask = nb - 1;
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
  Xform<U> xf;
  xf.init(*desc);
  const char* kp = desc->key.base[P.buf];
  const uint32_t ks = desc->key.stride;

  for (uint32_t i = threadIdx.x; i < (uint32_t)(NW * kMaxBins); i += NT)
    (&wc[0][0])[i] = 0;

  const int64_t base = P.start + tl * kTile;
  const int64_t rem = P.len - tl * kTile;
  const int cnt = rem < kTile ? (int)rem : kTile;

  // striped tile layout: slot k of lane l of wave w = element w*IT*64 + k*64 + l
  U raw[IT];
  bool valid[IT];
  uint32_t dig[IT];
#pragma unroll
  for (int k = 0; k < IT; k++) {
    const int e = (int)wave * IT * 64 + k * 64 + (int)lane;
    valid[k] = e < cnt;
    raw[k] = valid[k] ? (U) * (const KT*)(kp + (base + e) * (int64_t)ks) : (U)0;
  }
#pragma unroll
  for (int k = 0; k < IT; k++) dig[k] = (uint32_t)(xf(raw[k]) >> P.shift) & mask;
  __syncthreads();  // wc zeroed

  uint32_t pos[IT];
  wlms_rank<IT>(dig, valid, P.bits, &wc[wave][0], pos);
  __syncthreads();

  // bin totals over waves -> per-wave exclusive offsets; tile exclusive scan
  {
    const uint32_t b0 = threadIdx.x * 2, b1 = b0 + 1;
    uint32_t t0 = 0, t1 = 0;
    if (b0 < nb) {
#pragma unroll
      for (int w = 0; w < NW; w++) { const uint32_t c = wc[w][b0]; wc[w][b0] = (uint16_t)t0; t0 += c; }
    }
    if (b1 < nb) {
#pragma unroll
      for (int w = 0; w < NW; w++) { const uint32_t c = wc[w][b1]; wc[w][b1] = (uint16_t)t1; t1 += c; }
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan<NT>(t0 + t1, scan_sh, &tot);
    if (b0 < nb) {
      bin_start[b0] = ex;
      const uint64_t o = offs[P.hist_base + (int64_t)b0 * P.ntiles + tl] - offs[P.hist_base];
      gdst[b0] = P.start + (int64_t)o - (int64_t)ex;
    }
    if (b1 < nb) {
      bin_start[b1] = ex + t0;
      const uint64_t o = offs[P.hist_base + (int64_t)b1 * P.ntiles + tl] - offs[P.hist_base];
      gdst[b1] = P.start + (int64_t)o - (int64_t)(ex + t0);
    }
  }
  __syncthreads();

#pragma unroll
  for (int k = 0; k < IT; k++) {
    if (valid[k]) {
      const uint32_t d = dig[k];
      pos[k] = bin_start[d] + wc[wave][d] + pos[k];
      sbin[pos[k]] = (uint16_t)d;
    }
  }
  __syncthreads();

  int64_t dst[IT];
#pragma unroll
  for (int i = 0; i < IT; i++) {
    const int j = i * NT + (int)threadIdx.x;
    dst[i] = j < cnt ? (int64_t)j + gdst[sbin[j]] : 0;
  }

  const int ncols = desc->ncols;
  for (int c = 0; c < ncols; c++) {
    const Col col = desc->cols[c];
    const char* src = col.base[P.buf];
    char* out = col.base[P.dst];
    const uint32_t w = col.width, st = col.stride;
    if (c == 0 && desc->col0_is_key) {
#pragma unroll
      for (int k = 0; k < IT; k++)
        if (valid[k]) sval[pos[k]] = (uint64_t)raw[k];
    } else {
      uint64_t v[IT];
#pragma unroll
      for (int k = 0; k < IT; k++) {
        const int e = (int)wave * IT * 64 + k * 64 + (int)lane;
        v[k] = valid[k] ? load_w(src + (base + e) * (int64_t)st, w) : 0;
      }
#pragma unroll
      for (int k = 0; k < IT; k++)
        if (valid[k]) sval[pos[k]] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IT; i++) {
      const int j = i * NT + (int)threadIdx.x;
      if (j < cnt) store_w(out + dst[i] * (int64_t)st, w, sval[j]);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// local: one workgroup sorts one segment (<= kLocalCap keys) in LDS
// ---------------------------------------------------------------------------
template <typename KT, typename U>
__global__ __launch_bounds__(kLocalThreads) void local_kernel(
    const SortDesc* __restrict__ desc, const Seg* __restrict__ segs) {
  constexpr int NT = kLocalThreads;
  constexpr int IT = kLocalItems;
  constexpr int NW = NT / 64;
  constexpr int RB = 8;  // bits per LDS pass
  __shared__ U su[kLocalCap];
  __shared__ uint16_t sidx[kLocalCap];
  __shared__ uint16_t wc[NW][1 << RB];
  __shared__ uint32_t bin_start[1 << RB];
  __shared__ uint32_t scan_sh[NW + 1];
  __shared__ unsigned long long sh_or;

  const Seg g = segs[blockIdx.x];
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
  Xform<U> xf;
  xf.init(*desc);
  const char* kp = desc->key.base[g.buf];
  const uint32_t ks = desc->key.stride;
  const int cnt = (int)g.len;
  const int64_t base = g.start;

  if (threadIdx.x == 0) sh_or = 0;
  U u[IT];
  uint32_t id[IT];
  bool valid[IT];
#pragma unroll
  for (int k = 0; k < IT; k++) {
    const int e = (int)wave * IT * 64 + k * 64 + (int)lane;
    valid[k] = e < cnt;
    id[k] = (uint32_t)e;
    u[k] = valid[k] ? (U) * (const KT*)(kp + (base + e) * (int64_t)ks) : (U)0;
  }
  const U uref = xf((U) * (const KT*)(kp + base * (int64_t)ks));
  U vor = 0;
#pragma unroll
  for (int k = 0; k < IT; k++) {
    u[k] = xf(u[k]);
    if (valid[k]) vor |= u[k] ^ uref;
  }
  __syncthreads();
  if (vor) atomicOr(&sh_or, (unsigned long long)vor);
  __syncthreads();
  const unsigned long long var = sh_or;

  bool sorted_identity = (var == 0);
  if (!sorted_identity) {
    const int lo = __ffsll((long long)var) - 1;
    const int hi = 63 - __clzll((long long)var);
    for (int sh = lo; sh <= hi; sh += RB) {
      const int nbits = (hi - sh + 1) < RB ? (hi - sh + 1) : RB;
      const uint32_t nb = 1u << nbits, mask = nb - 1;
      for (uint32_t i = threadIdx.x; i < (uint32_t)(NW << RB); i += NT) (&wc[0][0])[i] = 0;
      uint32_t dig[IT];
#pragma unroll
      for (int k = 0; k < IT; k++) dig[k] = (uint32_t)(u[k] >> sh) & mask;
      __syncthreads();
      uint32_t rank[IT];
      wlms_rank<IT>(dig, valid, nbits, &wc[wave][0], rank);
      __syncthreads();
      {
        const uint32_t b = threadIdx.x;  // NT >= 256 bins
        uint32_t tb = 0;
        if (b < nb) {
#pragma unroll
          for (int w = 0; w < NW; w++) { const uint32_t c = wc[w][b]; wc[w][b] = (uint16_t)tb; tb += c; }
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<NT>(tb, scan_sh, &tot);
        if (b < nb) bin_start[b] = ex;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < IT; k++) {
        if (valid[k]) {
          const uint32_t p = bin_start[dig[k]] + wc[wave][dig[k]] + rank[k];
          su[p] = u[k];
          sidx[p] = (uint16_t)id[k];
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < IT; k++) {
        const int e = (int)wave * IT * 64 + k * 64 + (int)lane;
        if (valid[k]) {
          u[k] = su[e];
          id[k] = sidx[e];
        }
      }
      __syncthreads();
    }
  }

  // Move every column: out[start + e] = src[start + id(e)]. Register-staged
  // with a barrier between all loads and all stores, so src == out (segment
  // already in the output buffer) is safe.
  if (sorted_identity && g.buf == BUF_OUT) return;
  const int ncols = desc->ncols;
  for (int c = 0; c < ncols; c++) {
    const Col col = desc->cols[c];
    const char* src = col.base[g.buf];
    char* out = col.base[BUF_OUT];
    const uint32_t w = col.width, st = col.stride;
    uint64_t v[IT];
#pragma unroll
    for (int k = 0; k < IT; k++)
      v[k] = valid[k] ? load_w(src + (base + (int64_t)id[k]) * st, w) : 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; k++) {
      const int e = (int)wave * IT * 64 + k * 64 + (int)lane;
      if (valid[k]) store_w(out + (base + e) * (int64_t)st, w, v[k]);
    }
    __syncthreads();
  }
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
#define SRS_KEY_DISPATCH(KSZ, CALL)                 \
  switch (KSZ) {                                     \
    case 1: CALL(uint8_t, uint32_t); break;          \
    case 2: CALL(uint16_t, uint32_t); break;         \
    case 4: CALL(uint32_t, uint32_t); break;         \
    default: CALL(uint64_t, uint64_t); break;        \
  }

void launch_plan(const Seg* big, int64_t nbig, SegPlan* plan, int64_t* tcount,
                 int64_t* hcount, unsigned long long* var_or, uint64_t* elems,
                 hipStream_t st) {
  plan_kernel<<<(unsigned)((nbig + 255) / 256), 256, 0, st>>>(big, nbig, plan, tcount,
                                                              hcount, var_or, elems);
}

void launch_plan_bases(SegPlan* plan, int64_t nbig, const int64_t* tbase,
                       const int64_t* hbase, hipStream_t st) {
  plan_bases_kernel<<<(unsigned)((nbig + 255) / 256), 256, 0, st>>>(plan, nbig, tbase,
                                                                    hbase);
}

void launch_tile_map(const SegPlan* plan, int64_t nbig, int64_t ntiles, int32_t* tile_seg,
                     hipStream_t st) {
  tile_map_kernel<<<(unsigned)((ntiles + 255) / 256), 256, 0, st>>>(plan, nbig, ntiles,
                                                                    tile_seg);
}

void launch_count(int key_size, const SortDesc* d, const SegPlan* plan,
                  const int32_t* tile_seg, int64_t ntiles, uint64_t* hist,
                  unsigned long long* var_or, hipStream_t st) {
#define CALL(KT, U)                                                                  \
  count_kernel<KT, U><<<(unsigned)ntiles, kScatterThreads, 0, st>>>(d, plan, tile_seg, \
                                                                    hist, var_or)
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

void launch_children(SegPlan* plan, int64_t nbig, const uint64_t* offs,
                     const unsigned long long* var_or, Seg* big_next, Seg* local,
                     Seg* copy, ListCounters* ctr, hipStream_t st) {
  children_kernel<<<(unsigned)nbig, 512, 0, st>>>(plan, offs, var_or, big_next, local,
                                                  copy, ctr);
}

void launch_scatter(int key_size, const SortDesc* d, const SegPlan* plan,
                    const int32_t* tile_seg, const uint64_t* offs, int64_t ntiles,
                    hipStream_t st) {
#define CALL(KT, U) \
  scatter_kernel<KT, U><<<(unsigned)ntiles, kScatterThreads, 0, st>>>(d, plan, tile_seg, offs)
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
}

void launch_local(int key_size, const SortDesc* d, const Seg* segs, int64_t nsegs,
                  hipStream_t st) {
#define CALL(KT, U) local_kernel<KT, U><<<(unsigned)nsegs, kLocalThreads, 0, st>>>(d, segs)
  SRS_KEY_DISPATCH(key_size, CALL)
#undef CALL
}

void launch_fill(int64_t n, int kind, uint64_t seed, uint64_t first, void* keys,
                 int npay, const Col* pays, hipStream_t st) {
  fill_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, kind, seed, first,
                                                           (char*)keys, npay, pays);
}

}  // namespace srs

namespace srs {

// Kernel arguments are captured at launch, so the descriptor needs no pinned
// staging buffer and is safe to rebuild for the next call immediately.
__global__ void set_desc_kernel(SortDesc d, SortDesc* out) {
  if (threadIdx.x == 0) *out = d;
}

__global__ void init_lists_kernel(Seg seg0, int to_local, Seg* big, Seg* local,
                                  ListCounters* ctr) {
  if (threadIdx.x == 0) {
    ctr->n_big = to_local ? 0 : 1;
    ctr->n_local = to_local ? 1 : 0;
    ctr->n_copy = 0;
    ctr->local_elems = to_local ? (unsigned long long)seg0.len : 0;
    if (to_local) local[0] = seg0; else big[0] = seg0;
  }
}

void launch_set_desc(const SortDesc& d, SortDesc* out, hipStream_t st) {
  set_desc_kernel<<<1, 64, 0, st>>>(d, out);
}

void launch_init_lists(Seg seg0, int to_local, Seg* big, Seg* local, ListCounters* ctr,
                       hipStream_t st) {
  init_lists_kernel<<<1, 64, 0, st>>>(seg0, to_local, big, local, ctr);
}

}  // namespace srs

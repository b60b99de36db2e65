// srs_common.h — data layout shared by the HIP kernels and the host driver.
//
// The sort is an MSB radix sort organised breadth-first over "segments"
// (contiguous index ranges whose keys agree on all bits above `rbits`):
//
//   * global digit pass (count -> scan -> scatter) for segments larger than
//     the LDS capacity; one launch handles every large segment of a level;
//   * local LDS sort (one workgroup per segment) for segments that fit.
//
// This replaces the reference's depth-first 1-bit recursion
// (radixRecursion, radixSort.hpp:1734-1759) and its AVX-512 compress-store
// partition (BitSorterSIMD::sortBit, radixSort.hpp:1587-1686).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srs {

// Buffer slots a segment can live in. IN may alias OUT (in-place call).
// TMP2: second workspace buffer, used only when AoS records travel as SoA
// slice columns between the first and the last pass (SortDesc::tmp2).
enum BufId : int32_t { BUF_IN = 0, BUF_OUT = 1, BUF_TMP = 2, BUF_TMP2 = 3 };
constexpr int kNumBufs = 4;

// A column of fixed-width elements (the key column, a payload column, or an
// 8-byte slice of an AoS record). Element i of buffer b lives at
// base[b] + i * stride[b], `width` bytes (1, 2, 4 or 8). The stride depends
// on the buffer: an AoS slice has the record size in IN / OUT and its own
// width in the workspace when the workspace holds it as a SoA column.
struct Col {
  char* base[kNumBufs];
  uint32_t width;  // 32-bit fields: scalar loads (a 16-bit field is read with a
  uint32_t stride[kNumBufs];  // vector load and a vmcnt wait behind the tile's)
};

// the key + 64 payload columns (srs_c_api.h SRS_MAX_PAYLOADS), or <= 8 AoS
// slices; SortDesc stays under the 4 KB kernel-argument limit
#define SRS_MAX_COLS 65

// Everything a kernel needs to read keys and move records.
struct SortDesc {
  Col key;                 // key view (width = key size)
  Col cols[SRS_MAX_COLS];  // columns moved with every key; cols[0] holds the
                           // key in its low bytes (SoA key column / AoS slice 0)
  int32_t ncols;
  int32_t key_bits;        // 8 * key size
  int32_t canon_zero;      // float keys, n <= cmpSortThreshold: -0.0 == +0.0
  int32_t tmp2;            // AoS records as SoA slice columns in TMP / TMP2
                           // (scatters go IN -> TMP, TMP <-> TMP2; the local
                           // pass writes the records back to OUT)
  int32_t pair;            // SoA key + two 4-byte payloads (C2): cols 1 and 2
                           // are one interleaved 8-byte word per record in
                           // TMP / TMP2 (stride 8, col 2 at +4; tmp2 is set),
                           // separate arrays in IN / OUT
  int32_t leaf_skip;       // CmpSorterNoSort (src/cmp_sorters.hpp:66-78): the local
                           // pass leaves buckets of <= leaf_skip keys in bucket-pass
                           // order instead of ranking them (0: leaves sorted)
  // transformed key u = bits ^ (bits & signbit ? mneg : mpos)
  uint64_t mpos, mneg, signbit, negzero;
  // partition passes only: digit = digit_lut[u >> lut_shift]
  const int32_t* digit_lut;
  int32_t lut_shift;
  int32_t lut_bits;   // mode 0: table size 2^lut_bits; staged in LDS when <= kLdsLutBits
  int32_t lut_mode;   // 0 flat int32 table, 1 two-level u16 table, 2 key ranges (see DigitLut)
  int32_t lut_entries;  // mode 1: u16 entries (4096 + 16 per split bin)
  // lut_mode 2 (range level): up to kMaxRanges clusters of
  // keys; key u belongs to range c = #{k : u > rng_hi[k]} and goes to bucket
  // (uint32)(u >> lut_shift) + rng_adj[c] (wrapping): the range's buckets are
  // consecutive aligned blocks of 2^lut_shift key values
  uint64_t rng_hi[4];
  uint32_t rng_adj[4];
  unsigned long long* stamp_acc;  // diagnostic builds only (SRS_STAMPS)
  // diagnostic builds only (SRS_DIAG_LOOKBACK): per (tile, digit) look-back
  // status words of the scatter and error counters [mismatch, timeout, hops]
  uint32_t* lb_status;
  unsigned long long* lb_err;
};

struct Seg {
  int64_t start;
  int64_t len;
  int32_t rbits;  // keys agree on transformed bits >= rbits
  int32_t buf;    // BufId where the segment's data currently lives
};

// Per large segment, for one global digit pass.
struct SegPlan {
  int64_t start;
  int64_t len;
  int64_t tile_base;  // first tile of this segment in the level's tile space
  int64_t group_base; // first scan group (kScanGroup tiles) of this segment
  int32_t ntiles;
  int32_t ngroups;
  int32_t shift;      // digit = (u >> shift) & ((1 << bits) - 1)
  int32_t bits;
  int32_t buf;        // source buffer
  int32_t dst;        // destination buffer of the scatter
  int32_t skip;       // set by the children kernel: one bucket holds everything
};

// Stripe first level: the first digit partitions each stripe
// of kStripeKeysPerBucket << bits keys on its own, so a tile's scattered runs
// land in the stripe's window instead of across the whole array; bucket b's
// pieces (one per stripe, in stripe order) are then read by the second level
// through a table of gathered tiles: tile t of that level holds the cnt
// records at element src of its source buffer (never straddling a piece).
struct GTile {
  int64_t src;
  int32_t cnt;
  int32_t pad;
};
// average piece (one stripe's share of one bucket) for uniform keys: 95 % of
// a tile, so a piece almost never spills a second, nearly empty tile
#ifndef SRS_STRIPE_KPB
#define SRS_STRIPE_KPB 3904
#endif
constexpr int kStripeKeysPerBucket = SRS_STRIPE_KPB;

// The mid-size launch's answer to the host (coherent pinned host memory):
// written by workgroup 0 once the first level's bucket sizes are known, so
// the host need not wait for the whole kernel (seq last, release).
struct MidFlag {
  unsigned long long n_big;  // buckets handed back to the general levels (bit 63: error)
  unsigned long long seq;    // the call's sequence number
  unsigned long long err;    // the seq of a call whose grid barrier timed out (0: none)
  // (mid_level_kernel) the other lists' lengths and the local lists' records
  unsigned long long n_local, n_local2, n_copy, local_elems;
};

// Work-list counters (device), read back by the host once per level.
struct ListCounters {
  unsigned long long n_big;    // segments for the next global level
  unsigned long long n_local;  // segments for the LDS sort
  unsigned long long n_copy;   // finished segments that must be copied to OUT
  unsigned long long local_elems;  // keys in the local lists (timing stats)
  unsigned long long n_local2; // segments for the large-class LDS sort
  unsigned long long n_fallback;  // large-class segments handed to the stable kernel
  unsigned long long n_fallback1; // small-class segments handed to the stable kernel
  unsigned long long n_fallback2; // segments handed on to the LSD local kernel
  unsigned long long n_redo;      // small-class segments the direct kernel handed to the fast one
  unsigned long long n_redo2;     // large-class segments the direct kernel handed to the fast one
};

// Tuning constants (see DESIGN.md §4 for how they were chosen).
// (overridable at build time for tuning sweeps: tools/build_variants.sh)
#ifndef SRS_SCATTER_THREADS
#define SRS_SCATTER_THREADS 1024
#endif
#ifndef SRS_SCATTER_ITEMS
#define SRS_SCATTER_ITEMS 4
#endif
#ifndef SRS_SCATTER_WAVES_PER_EU
#define SRS_SCATTER_WAVES_PER_EU 8
#endif
#ifndef SRS_SCATTER_SDIG
#define SRS_SCATTER_SDIG 1   // stage each slot's digit (0: recompute it from the key)
#endif
#ifndef SRS_LOCAL_RANK_SPLIT
#define SRS_LOCAL_RANK_SPLIT 2
#endif
constexpr int kScatterThreads = SRS_SCATTER_THREADS;
constexpr int kScatterItems = SRS_SCATTER_ITEMS;
constexpr int kTile = kScatterThreads * kScatterItems;   // keys per tile
#ifndef SRS_COUNT_THREADS
#define SRS_COUNT_THREADS 256
#endif
constexpr int kCountThreads = SRS_COUNT_THREADS;         // count kernel: one tile per block
constexpr int kCountItems = kTile / kCountThreads;
static_assert(kCountItems * kCountThreads == kTile, "count block shape");
#ifndef SRS_MAX_DIGIT_BITS
#define SRS_MAX_DIGIT_BITS 9
#endif
constexpr int kMaxDigitBits = SRS_MAX_DIGIT_BITS;
// launch_* key_size flag: the canon-zero float case (SortDesc::canon_zero),
// selects the kernel instantiations that map -0.0 to +0.0
#define SRS_KS_CANON 0x100
constexpr int kMaxBins = 1 << kMaxDigitBits;   // histogram row stride (tile-major)
static_assert(kScatterThreads >= kMaxBins, "the scatter tile scan gives one bin per thread");
#ifndef SRS_SCAN_GROUP
#define SRS_SCAN_GROUP 32
#endif
constexpr int kScanGroup = SRS_SCAN_GROUP;      // tiles per column-scan group
constexpr int kHistMaxBits = 12;                // srs_key_histogram_device
constexpr int kMaxRanges = 4;                   // key clusters of a range level (lut_mode 2)
constexpr int kLdsLutBits = 12;                 // flat digit tables up to 4096 entries live in LDS
constexpr int kLdsLutEntries = 4096 + 16 * 512; // two-level table worst case (24 KB of u16)
// sampled 16-bit skew histogram (balanced first level): workgroups, and the
// sample's shape; a workgroup's packed u16 LDS bins hold < 65536 keys
constexpr int kSampleWGs = 256;
constexpr int kSampleChunk = 1024;      // contiguous keys per sampled chunk
constexpr int kSampleMaxChunks = 4096;
static_assert((kSampleMaxChunks + kSampleWGs - 1) / kSampleWGs * kSampleChunk < 65536,
              "sample histogram: u16 bins per workgroup");

// local sort classes: fast kernel (atomic bucket pass + rank) in two sizes,
// then the stable kernel and the LSD kernel as fallbacks (same capacity as
// the large class)
#ifndef SRS_LOCAL_THREADS
#define SRS_LOCAL_THREADS 1024
#endif
#ifndef SRS_LOCAL_ITEMS
#define SRS_LOCAL_ITEMS 8
#endif
constexpr int kLocalItems = SRS_LOCAL_ITEMS;
constexpr int kLocalThreads = SRS_LOCAL_THREADS;
constexpr int kLocalCap = kLocalThreads * kLocalItems;    // 8192 keys per segment
#ifndef SRS_LOCAL_SMALL_THREADS
#define SRS_LOCAL_SMALL_THREADS 512
#endif
#ifndef SRS_LOCAL_SMALL_WGS_PER_CU
#define SRS_LOCAL_SMALL_WGS_PER_CU 3
#endif
constexpr int kLocalThreadsSmall = SRS_LOCAL_SMALL_THREADS;
constexpr int kLocalItemsSmall = 4096 / kLocalThreadsSmall;
constexpr int kLocalCapSmall = kLocalThreadsSmall * kLocalItemsSmall;  // 4096
// occupancy the LDS footprint allows (90 KB -> 1 block/CU; 49 KB -> 3 blocks/CU)
constexpr int kLocalWavesPerEU = kLocalThreads / 64 / 4;
constexpr int kLocalWavesPerEUSmall = SRS_LOCAL_SMALL_WGS_PER_CU * kLocalThreadsSmall / 64 / 4;
// direct local kernel (small class, common SoA shape): 4 workgroups of
// 256 x 16 per CU
constexpr int kLocalDirectThreads = 256;
constexpr int kLocalDirectItems = 4096 / kLocalDirectThreads;
#ifndef SRS_LOCAL_DIRECT_WGS_PER_CU
#define SRS_LOCAL_DIRECT_WGS_PER_CU 4
#endif
constexpr int kLocalDirectWavesPerEU = SRS_LOCAL_DIRECT_WGS_PER_CU * kLocalDirectThreads / 64 / 4;
// and its large class (up to kLocalCap records): 2 workgroups of 512 x 16 per CU
constexpr int kLocalDirectThreads2 = 512;
constexpr int kLocalDirectItems2 = 8192 / kLocalDirectThreads2;
constexpr int kLocalDirectWavesPerEU2 = 2 * kLocalDirectThreads2 / 64 / 4;
// cache-policy bits of the scatter's / the direct local kernel's column
// loads (buffer-load aux operand; 0 = default)
#ifndef SRS_SCATTER_LOAD_AUX
#define SRS_SCATTER_LOAD_AUX 0
#endif
#ifndef SRS_LOCAL_LOAD_AUX
#define SRS_LOCAL_LOAD_AUX 0
#endif
// direct local kernel: bucket digit = the sort word's top bits (1; measured
// slower for C2: local 4.62-4.65 -> 6.02-6.07 ms), or the
// key's top varying bits with a ballot-ranked exact pass in the pair mode (0)
#ifndef SRS_DIRECT_WORD_DIGIT
#define SRS_DIRECT_WORD_DIGIT 0
#endif
#ifndef SRS_DIRECT_RANK_SPLIT
#define SRS_DIRECT_RANK_SPLIT 2
#endif
#ifndef SRS_DIRECT_EARLY_PAYLOAD
#define SRS_DIRECT_EARLY_PAYLOAD 0
#endif
#ifndef SRS_LOCAL_STABLE_ITEMS
#define SRS_LOCAL_STABLE_ITEMS 8
#endif
constexpr int kLocalStableItems = SRS_LOCAL_STABLE_ITEMS;
constexpr int kLocalStableThreads = kLocalCap / kLocalStableItems;
constexpr int kLocalStableThreadsSmall = kLocalCapSmall / kLocalStableItems;
static_assert(kLocalStableThreads * kLocalStableItems == kLocalCap, "fallback capacity");
static_assert(kLocalStableThreadsSmall * kLocalStableItems == kLocalCapSmall, "fallback capacity");
constexpr int kLocalTarget = 6144;                        // digit sizing target
// average bucket that still lands in the small class: ~94 % full for uniform
// keys (the small class is 2.5x cheaper per key than the large one, and a
// half-empty small segment costs ~1.5x per key of a full one)
#ifndef SRS_LOCAL_SMALL_TARGET
#define SRS_LOCAL_SMALL_TARGET 3840
#endif
constexpr int kLocalSmallTarget = SRS_LOCAL_SMALL_TARGET;

// Digit width for a segment of `len` keys with `rbits` unsorted bits: as many
// bits as needed to bring buckets under kLocalTarget, spread evenly over the
// levels that will take, at most kMaxDigitBits per level. (Host and device:
// the host sizes the stripe level with it.)
__host__ __device__ inline int levels_for(int64_t len, int64_t target, int* need_out) {
  int need = 1;
  while (need < 62 && (target << need) < len) need++;
  *need_out = need;
  return (need + kMaxDigitBits - 1) / kMaxDigitBits;
}

// average bucket up to which a segment still takes one level fewer: its
// buckets then land in the large LDS class (<= kLocalCap records; its own
// direct kernel since round 4) instead of paying a count + scatter level and
// its launches and host sync. 512 x 7808 = 4.0 M: C2's densest first-level
// groups hold 3.9 M keys
constexpr int kLocalCapTarget = 7808;

__host__ __device__ inline int choose_bits(int64_t len, int rbits) {
  // bits needed to bring buckets under kLocalTarget, spread evenly over the
  // levels that takes (<= kMaxDigitBits each); one more bit when that lands
  // the buckets in the smaller (faster) LDS class without an extra level
  int need, need_small, need_cap;
  int levels = levels_for(len, kLocalTarget, &need);
  const int levels_cap = levels_for(len, kLocalCapTarget, &need_cap);
  if (levels_cap < levels) {
    levels = levels_cap;
    need = need_cap;
  }
  const int levels_small = levels_for(len, kLocalSmallTarget, &need_small);
  if (levels_small == levels) need = need_small;
  int bits = (need + levels - 1) / levels;
  if (bits > kMaxDigitBits) bits = kMaxDigitBits;
  if (bits > rbits) bits = rbits;
  if (bits < 1) bits = 1;
  return bits;
}

}  // namespace srs

// srs_kernels.h — host-side launch wrappers for the kernels in srs_kernels.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srs_common.h"

namespace srs {

void launch_plan(const Seg* big, int64_t nbig, SegPlan* plan, int64_t* tcount,
                 int64_t* gcount, unsigned long long* var_or, uint64_t* elems, int force_bits,
                 int tmp2, hipStream_t st, const int32_t* nt_over = nullptr);
void launch_plan_small(const Seg* big, int64_t nbig, SegPlan* plan, int64_t* tbase,
                       int64_t* gbase, unsigned long long* var_or, uint64_t* totals,
                       unsigned long long* n_big_next, int force_bits, int tmp2,
                       hipStream_t st, const int32_t* nt_over = nullptr);
constexpr int64_t kPlanSmallMax = 16384;  // plan_small_kernel: one workgroup loops over these
void launch_seg_map2(const int64_t* tbase, int64_t ntiles, int32_t* tile_seg,
                     const int64_t* gbase, int64_t ngroups, int32_t* group_seg, int64_t nbig,
                     hipStream_t st);
void launch_start(const SortDesc& d, SortDesc* out, Seg seg0, int to_local, Seg* big, Seg* local,
                  Seg* local2, ListCounters* ctr, hipStream_t st);
void launch_plan_bases(SegPlan* plan, int64_t nbig, const int64_t* tbase,
                       const int64_t* gbase, hipStream_t st);
void launch_count(int key_size, const SortDesc* d, const SegPlan* plan,
                  const int32_t* tile_seg, int64_t ntiles, uint16_t* hist,
                  unsigned long long* var_or, unsigned long long* var_and, int lut,
                  hipStream_t st, const GTile* gt = nullptr, const int32_t* torder = nullptr);
int64_t scan_temp_elems(int64_t n);
void launch_excl_scan(const uint64_t* x, uint64_t* y, int64_t n, uint64_t* temp,
                      uint64_t* total, hipStream_t st);
// rows launch_offsets' super-group scan adds behind gsum's and gofs' group rows
int64_t super_rows(int64_t ngroups);
// the scan groups from which a one-segment level takes it (<= 0: the default, 256)
void set_super_scan_min_groups(int64_t g);
void launch_offsets(SegPlan* plan, int64_t nbig, const int32_t* group_seg, int64_t ngroups,
                    const uint16_t* hist, uint32_t* gsum, uint64_t* gofs, uint64_t* sbase,
                    uint64_t* offs, uint32_t* offs32, const unsigned long long* var_or,
                    Seg* big_next, Seg* local, Seg* local2, Seg* copy, ListCounters* ctr,
                    const int32_t* lut_rbits, hipStream_t st, int mode = 0,
                    uint32_t* prun = nullptr);
void launch_scatter(int key_size, const SortDesc* d, const SegPlan* plan,
                    const int32_t* tile_seg, const uint64_t* offs, const uint32_t* offs32,
                    int64_t ntiles, int lut, int ncols, hipStream_t st,
                    const GTile* gt = nullptr);
// the same level's scatter with two count tiles per workgroup (lut 0 or 2;
// 4- or 8-byte keys; the key plus one column or C2's pair word; no canon zero)
void launch_scatter_pairs(int key_size, const SortDesc* d, const SegPlan* plan,
                          const int32_t* tile_seg, const uint64_t* offs, const uint32_t* offs32,
                          int64_t ntiles, int lut, hipStream_t st, const GTile* gt = nullptr);
// stripe first level -> the second level's segment list (W->big, n_big),
// tile counts (nt_over) and gathered tile table (gt); see GTile
void launch_stripe_tables(const uint32_t* prun, int64_t nstripes, int nb, uint32_t* ptile,
                          uint64_t* btot, uint32_t* bnt, int rbits, int buf, Seg* big,
                          int32_t* nt_over, uint32_t* btile, ListCounters* ctr,
                          const uint64_t* sbase, const SegPlan* plan, GTile* gt,
                          const int32_t* lut_rbits, hipStream_t st, int32_t* torder = nullptr,
                          int64_t tiles_cap = 0);  // torder: tiles_cap entries + nstripes of scratch
void launch_key_hist(int key_size, int64_t n, const void* keys, const SortDesc& d, int bits,
                     unsigned long long* hist, hipStream_t st);
// rec16: AoS records of 16 bytes held as two slice columns in TMP / TMP2
// (the local pass then writes whole records, one 16-byte store each)
void launch_local(int key_size, const SortDesc* d, const Seg* segs, int64_t nsegs, int big_class,
                  Seg* fallback, unsigned long long* fallback_count, hipStream_t st,
                  bool rec16 = false);
// the direct kernel (no canon-zero, 4/8-byte keys; pm 0: one 8-byte SoA
// payload, 1: 16-byte AoS records as slices, 2: desc->pair; big: the large
// class, up to kLocalCap records): segments it does not take go to `redo`,
// large buckets to `fallback`; launch_local_list then runs the fast kernel
// of the same class over `redo`
void launch_local_direct(int key_size, int pm, const SortDesc* d, const Seg* segs, int64_t nsegs,
                         Seg* redo, unsigned long long* redo_count, Seg* fallback,
                         unsigned long long* fallback_count, hipStream_t st, bool big = false);
void launch_local_list(int key_size, const SortDesc* d, const Seg* segs,
                       const unsigned long long* nsegs, int grid, Seg* fallback,
                       unsigned long long* fallback_count, hipStream_t st, bool big = false);
void launch_local_stable(int key_size, const SortDesc* d, const Seg* segs,
                         const unsigned long long* nsegs, int big_class, Seg* fallback,
                         unsigned long long* fallback_count, int grid, hipStream_t st);
// n <= kLocalCap: the whole sort in one single-workgroup launch
void launch_small_sort(int key_size, const SortDesc& d, Seg g, int64_t* taken, hipStream_t st);
// kLocalCap < n <= 64 tiles: one launch with grid barriers (mid_sort_kernel;
// every workgroup resident, else an error and the caller takes the general
// path); big buckets (> kLocalCap) are appended to `big` with ctr->n_big, and
// their count reaches the host early through `flag` (MidFlag, host memory).
// bar: mid_bar_words() u64 of device memory, zeroed once when allocated and
// left ready by every launch (a call whose barrier timed out posts its seq
// to flag->err). part: mid_part_bytes(n); hist: T x kMaxBins u32
constexpr int kMidMaxKeys = 256 * kTile;
int mid_bar_words();
int64_t mid_part_bytes(int64_t n);
hipError_t launch_mid_sort(int key_size, const SortDesc& d, int64_t n, int src,
                           unsigned long long* part, uint32_t* hist, ListCounters* ctr, Seg* big,
                           unsigned long long* taken, MidFlag* flag, unsigned long long seq,
                           unsigned long long* bar, hipStream_t st);
// kMidMaxKeys < n <= kMidLevelMaxKeys: the FIRST level in one launch
// (mid_level_kernel: count, column scans and scatter into TMP with grid
// barriers, the workgroups looping over tiles). The buckets go to the work
// lists as a level's would; their lengths reach the host through `flag`
// before the scatter ends (MidFlag n_big / n_local / n_local2 / n_copy), so
// the caller enqueues the LDS pass without a read-back. Writes the
// descriptor to d_out and resets ctr. part: mid_level_part_bytes(); hist: T x
// kMaxBins u32. Every workgroup resident, else an error (the general path).
constexpr int kMidLevelMaxKeys = 1024 * kTile;
int64_t mid_level_part_bytes();
hipError_t launch_mid_level(int key_size, const SortDesc& d, int64_t n, int src,
                            unsigned long long* part, uint32_t* hist, ListCounters* ctr, Seg* big,
                            Seg* local, Seg* local2, Seg* copy, SortDesc* d_out, MidFlag* flag,
                            unsigned long long seq, unsigned long long* bar, hipStream_t st);
void launch_local_lsd(int key_size, const SortDesc* d, const Seg* segs,
                      const unsigned long long* nsegs, int grid, hipStream_t st);
int64_t sample_partial_bytes();
void launch_key_minmax(const void* keys, int key_bytes, int elem_bytes, int64_t n, uint64_t mpos,
                       uint64_t mneg, const uint64_t* hi, unsigned long long* mm, hipStream_t st);
bool launch_sample_hist16(const void* keys, int key_bytes, int elem_bytes, int64_t n,
                          int64_t stride, int chunk, int64_t blocks, uint64_t mpos, uint64_t mneg,
                          uint32_t* partial, uint32_t* hist, hipStream_t st);
void launch_fill(int64_t n, int kind, uint64_t seed, uint64_t first, void* keys,
                 int npay, const Col* pays, hipStream_t st);
void launch_set_desc(const SortDesc& d, SortDesc* out, hipStream_t st);
// placement probe: ms of the scatter's write pattern over a buffer (sync)
float probe_write_ms(void* buf, size_t bytes, hipStream_t st);
// diagnostics: phase of each XCD's walk over its block range (xcd_remap)
void set_xcd_rotation(int mode);
// the copy list (finished segments not in OUT) home in one launch, column by
// column with each buffer's stride (AoS slice columns back into records)
// (chunks / cbase: nsegs u64 each; scan_temp: scan_temp_elems(nsegs) u64;
// total: one u64)
void launch_copy_list(const SortDesc* d, const Seg* segs, int64_t nsegs, uint64_t* chunks,
                      uint64_t* cbase, uint64_t* scan_temp, uint64_t* total, hipStream_t st);

}  // namespace srs

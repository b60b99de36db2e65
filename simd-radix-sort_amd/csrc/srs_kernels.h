// srs_kernels.h — host-side launch wrappers for the kernels in srs_kernels.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srs_common.h"

namespace srs {

void launch_plan(const Seg* big, int64_t nbig, SegPlan* plan, int64_t* tcount,
                 int64_t* hcount, unsigned long long* var_or, uint64_t* elems,
                 hipStream_t st);
void launch_plan_bases(SegPlan* plan, int64_t nbig, const int64_t* tbase,
                       const int64_t* hbase, hipStream_t st);
void launch_tile_map(const SegPlan* plan, int64_t nbig, int64_t ntiles, int32_t* tile_seg,
                     hipStream_t st);
void launch_count(int key_size, const SortDesc* d, const SegPlan* plan,
                  const int32_t* tile_seg, int64_t ntiles, uint64_t* hist,
                  unsigned long long* var_or, hipStream_t st);
int64_t scan_temp_elems(int64_t n);
void launch_excl_scan(const uint64_t* x, uint64_t* y, int64_t n, uint64_t* temp,
                      uint64_t* total, hipStream_t st);
void launch_children(SegPlan* plan, int64_t nbig, const uint64_t* offs,
                     const unsigned long long* var_or, Seg* big_next, Seg* local,
                     Seg* copy, ListCounters* ctr, hipStream_t st);
void launch_scatter(int key_size, const SortDesc* d, const SegPlan* plan,
                    const int32_t* tile_seg, const uint64_t* offs, int64_t ntiles,
                    hipStream_t st);
void launch_local(int key_size, const SortDesc* d, const Seg* segs, int64_t nsegs,
                  hipStream_t st);
void launch_fill(int64_t n, int kind, uint64_t seed, uint64_t first, void* keys,
                 int npay, const Col* pays, hipStream_t st);
void launch_set_desc(const SortDesc& d, SortDesc* out, hipStream_t st);
void launch_init_lists(Seg seg0, int to_local, Seg* big, Seg* local, ListCounters* ctr,
                       hipStream_t st);

}  // namespace srs

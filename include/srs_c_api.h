/*
 * srs_c_api.h — C ABI of the MI355X-native MSB radix sort (libsrs_amd.so).
 *
 * This is the drop-in boundary for the reference's hot path. Every entry point
 * takes plain pointers and sizes; there are no C++ or torch types in the
 * signatures, so cgo / ctypes / JNI / N-API can bind it directly.
 *
 * Reference interfaces replaced (jonicho/simd-radix-sort, /root/reference):
 *   srs_sort_soa     <- simd_sort::radix_sort::sort(num, keys, payloads...)
 *                       radixSort.hpp:1780-1783, and the thresholded form
 *                       sort<Up,BitSorter,CmpSorter>(cmpSortThreshold, num,
 *                       keys, payloads...) radixSort.hpp:1761-1768
 *                       (src/radix_sort.hpp:297-312, :334-337)
 *   srs_sort_aos     <- sort<Up,BitSorter,CmpSorter>(cmpSortThreshold, num,
 *                       DataElement<K,Ps...>* elements) radixSort.hpp:1770-1778
 *                       (src/radix_sort.hpp:314-332)
 *   *_device         <- same semantics on arrays already resident in HBM,
 *                       enqueued on a caller-provided hipStream_t.
 *
 * Semantics (identical to the reference):
 *   - In place: on return the caller's arrays hold the sorted data.
 *   - Key order is the reference's per-bit direction order
 *     (bitDirUp, radixSort.hpp:1568-1581): unsigned ascending, two's
 *     complement signed, IEEE floats by value with -0.0 before +0.0 (n >
 *     cmp_sort_threshold) or -0.0 == +0.0 kept in input order (n <=
 *     cmp_sort_threshold, the reference's insertion-sort leaf,
 *     radixSort.hpp:159-178 / :1743). up == 0 reverses the order.
 *   - num <= 1 is a no-op (radixSort.hpp:1740). num < 0 is a no-op.
 *   - Payload order inside a run of equal keys: the GPU sort is STABLE
 *     (input order). The reference is unstable there; see DESIGN.md §5 for
 *     what parity means for equal keys.
 *   - NaN keys are outside the contract (the reference's leaf never moves
 *     them; its output depends on leaf boundaries).
 *
 * Error convention: every function returns SRS_OK (0) or a negative
 * srs_status; srs_last_error() returns a thread-local message. The reference
 * API is void (no error channel); the C++ drop-in header
 * (include/simd_sort/radix_sort.hpp) turns a non-zero status into
 * std::abort() with the message, i.e. it fails loudly. There is NO CPU
 * fallback inside the library.
 */
#ifndef SRS_C_API_H_
#define SRS_C_API_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Key kinds: the ten key types the reference supports and tests
 * (src/test.cpp:156-169). Values are part of the ABI. */
typedef enum srs_key_kind {
  SRS_KEY_U8 = 0,
  SRS_KEY_I8 = 1,
  SRS_KEY_U16 = 2,
  SRS_KEY_I16 = 3,
  SRS_KEY_U32 = 4,
  SRS_KEY_I32 = 5,
  SRS_KEY_U64 = 6,
  SRS_KEY_I64 = 7,
  SRS_KEY_F32 = 8,
  SRS_KEY_F64 = 9
} srs_key_kind;

typedef enum srs_status {
  SRS_OK = 0,
  SRS_ERR_INVALID_ARG = -1,
  SRS_ERR_UNSUPPORTED = -2,
  SRS_ERR_HIP = -3,
  SRS_ERR_OUT_OF_MEMORY = -4,
  SRS_ERR_NO_DEVICE = -5,
  SRS_ERR_INTERNAL = -6
} srs_status;

/* Maximum number of payload columns per call (the reference's test uses up
 * to 63 one-byte payloads, src/test.cpp:125-134). */
#define SRS_MAX_PAYLOADS 64

/* ---- host-pointer drop-in entry points (synchronous) -------------------- */

/* Sort `num` keys (kind `key_kind`) and `num_payloads` payload columns in
 * place. payload_sizes[i] is the element size in bytes of column i
 * (1, 2, 4 or 8). cmp_sort_threshold is the reference's cmpSortThreshold
 * (16 in the two-argument sort()). Host memory; copies through HBM. */
int srs_sort_soa(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                 void* keys, int32_t num_payloads, void* const* payloads,
                 const uint32_t* payload_sizes);

/* Sort `num` combined elements of `elem_size` bytes (a power of two, 1..64,
 * >= the key size) whose key of kind `key_kind` sits at byte offset 0
 * (simd_sort::DataElement<K, Ps...>). The payload bytes are opaque and move
 * with their key. */
int srs_sort_aos(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                 void* elements, uint32_t elem_size);

/* Leaf handling: the reference's CmpSorter template argument
 * (src/cmp_sorters.hpp). SRS_LEAF_SORTED = CmpSorterInsertionSort (and
 * CmpSorterBramasSmallSort): leaves of <= cmp_sort_threshold keys are sorted,
 * so the output is fully sorted. SRS_LEAF_UNSORTED = CmpSorterNoSort
 * (src/cmp_sorters.hpp:66-78, thesis:3113-3124): the recursion stops at
 * leaves of <= cmp_sort_threshold keys and leaves them in partition order.
 * Every leaf then holds exactly the keys (and their payloads) a full sort
 * puts there, so each element ends within cmp_sort_threshold - 1 places of
 * its sorted slot; num <= cmp_sort_threshold leaves the input untouched.
 * The order inside a leaf is unspecified and may differ from run to run (the
 * GPU's bucket pass places a leaf's elements with LDS atomics); only the
 * leaf's contents are guaranteed, as for the reference's no-op leaf. */
#define SRS_LEAF_SORTED 0
#define SRS_LEAF_UNSORTED 1

/* srs_sort_soa / srs_sort_aos with the leaf handling chosen by leaf_mode:
 * sort<Up, BitSorter, CmpSorter>(cmpSortThreshold, num, ...) for every
 * CmpSorter of src/cmp_sorters.hpp (radixSort.hpp:1761-1778). */
int srs_sort_soa_leaf(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                      int leaf_mode, void* keys, int32_t num_payloads, void* const* payloads,
                      const uint32_t* payload_sizes);
int srs_sort_aos_leaf(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                      int leaf_mode, void* elements, uint32_t elem_size);

/* ---- device-pointer entry points (asynchronous on `stream`) ------------- */

/* Same as srs_sort_soa on device pointers. `stream` is a hipStream_t (NULL =
 * the default stream). If keys_out/payloads_out are NULL the sort is in place;
 * otherwise the inputs are left untouched and the result is written to the
 * *_out arrays (which must not alias the inputs). The call enqueues work and
 * may block briefly on small control read-backs; results are ready when the
 * stream completes. By size: num <= 8192 is one launch and no host wait;
 * 8192 < num <= 2^20 (no segment list) is one launch with its own grid
 * barriers, and the call waits until that kernel has posted its first
 * level's bucket sizes to host memory (a skewed input then continues on the
 * general levels); larger sorts read back a small counter block once per
 * global level. */
int srs_sort_soa_device(int64_t num, int key_kind, int up,
                        int64_t cmp_sort_threshold, void* keys,
                        int32_t num_payloads, void* const* payloads,
                        const uint32_t* payload_sizes, void* keys_out,
                        void* const* payloads_out, void* stream);

int srs_sort_aos_device(int64_t num, int key_kind, int up,
                        int64_t cmp_sort_threshold, void* elements,
                        uint32_t elem_size, void* elements_out, void* stream);

/* The device forms with the leaf handling chosen by leaf_mode (see above). */
int srs_sort_soa_device_leaf(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                             int leaf_mode, void* keys, int32_t num_payloads,
                             void* const* payloads, const uint32_t* payload_sizes,
                             void* keys_out, void* const* payloads_out, void* stream);
int srs_sort_aos_device_leaf(int64_t num, int key_kind, int up, int64_t cmp_sort_threshold,
                             int leaf_mode, void* elements, uint32_t elem_size,
                             void* elements_out, void* stream);

/* Sorts each segment [segment_bounds[i], segment_bounds[i+1]) of a device
 * key column and its payload columns independently, in place, as sub-ranges
 * of one sort (no n <= threshold rule per segment). segment_bounds is a HOST
 * array of num_segments + 1 non-decreasing offsets within [0, num]; elements
 * outside every segment are untouched. known_top_bits: the caller guarantees
 * that inside each segment all keys agree on their top known_top_bits
 * transformed bits (0 = no knowledge); those bits are not examined again.
 * Asynchronous on `stream` (returns once the work is queued). Replaces
 * calling radix_sort::sort (radixSort.hpp:1780) once per sub-range; the
 * multi-GPU shard sorts its receive groups with it. */
int srs_sort_segments_device(int64_t num, int key_kind, int up, void* keys,
                             int32_t num_payloads, void* const* payloads,
                             const uint32_t* payload_sizes, int64_t num_segments,
                             const int64_t* segment_bounds, int32_t known_top_bits,
                             void* stream);

/* ---- multi-GPU shard primitives (top-radix-bits partition) --
 * A node-wide sort of one array spread over N GPUs: every rank histograms
 * its keys' top bits (srs_key_histogram_device), the histograms are summed
 * (RCCL all-reduce), contiguous bucket ranges are assigned to ranks, every
 * rank partitions its keys by destination (srs_partition_device), the groups
 * are exchanged (RCCL all-to-all) and each rank sorts what it received
 * (srs_sort_soa_device). Concatenating the ranks in order gives the sorted
 * array. The reference has no multi-device path; these have no counterpart. */

/* Adds the histogram of the transformed top `bits` (1..12) bits of `num`
 * device keys into the device array hist[2^bits] (uint64). Asynchronous. */
int srs_key_histogram_device(int64_t num, int key_kind, int up, const void* keys,
                             int bits, uint64_t* hist, void* stream);

/* Stable partition of a key column and its payload columns into num_parts
 * (<= 512) groups: a key whose transformed top `bits` (1..16) bits equal b
 * goes to group part_of_bucket[b] (DEVICE int32 array of 2^bits entries;
 * non-decreasing makes every group a contiguous key range). Groups are
 * written back to back, group 0 first, to keys_out / payloads_out (device,
 * not aliasing the inputs); part_counts (HOST array of num_parts int64)
 * receives the group sizes. Returns after the counts are known; the data
 * movement completes on `stream`. */
int srs_partition_device(int64_t num, int key_kind, int up, const void* keys,
                         int32_t num_payloads, const void* const* payloads,
                         const uint32_t* payload_sizes, int bits,
                         const int32_t* part_of_bucket, int32_t num_parts,
                         void* keys_out, void* const* payloads_out,
                         int64_t* part_counts, void* stream);

/* ---- the multi-GPU shard sort (C ABI) ----------------------
 * One array spread over N GPUs is sorted across them: rank r ends with the
 * r-th key range, so concatenating the ranks' outputs gives the sorted array
 * (stable). The protocol is the one above: histogram all-reduce, 512
 * key-range groups, chunked partition, rounds of grouped send/recv over
 * xGMI, each round's range sorted on a side stream while the later rounds
 * are in flight. RCCL is loaded at first use (librccl.so.1); without it the
 * RCCL communicators return SRS_ERR_NO_DEVICE. The reference has no
 * multi-device path. This is the only implementation of the protocol (the
 * Python bench drives it through ctypes).
 *
 * Communicators: one process per GPU (srs_shard_unique_id on one rank, the
 * 128 bytes passed to every rank, srs_shard_comm_init on each with its GPU
 * current), or one process driving several GPUs (srs_shard_comm_init_all,
 * then srs_shard_sort_multi).
 *
 * Failures: every rank returns an error if any rank fails (invalid or
 * disagreeing arguments, an allocation, a partition or a round sort), with
 * the communicator still usable afterwards; a rank never returns early while
 * its peers wait for its messages. A transport failure (RCCL error, timeout)
 * aborts the communicator (ncclCommAbort): later sorts on it fail and it
 * must be destroyed. Host waits on peers are bounded by SRS_SHARD_TIMEOUT_S
 * seconds (default 600). */
#define SRS_SHARD_ID_BYTES 128
typedef struct srs_shard_comm_s* srs_shard_comm;
int srs_shard_unique_id(void* id);
int srs_shard_comm_init(int32_t world, int32_t rank, const void* id, srs_shard_comm* comm);
int srs_shard_comm_init_all(int32_t num_devices, const int32_t* devices, srs_shard_comm* comms);
int srs_shard_comm_destroy(srs_shard_comm comm);

/* `world` communicators over the CURRENT device whose collectives and peer
 * messages travel through host memory (threads of one process; drive them
 * with srs_shard_sort_multi). Every kernel of the protocol runs as with
 * RCCL; only the transport differs. For tests and for machines with fewer
 * GPUs than ranks (RCCL puts no two ranks on one device). */
int srs_shard_comm_init_staged(int32_t world, srs_shard_comm* comms);

/* Exchange rounds (1..64) and partition chunks (1..16) of later sorts on
 * this communicator; 0 = the default (from 2 ranks up 8 rounds and 4
 * chunks; at one rank 8 rounds and 1 chunk). Every rank must use the same values (checked: a mismatch
 * fails every rank with SRS_ERR_INVALID_ARG). */
int srs_shard_set_options(srs_shard_comm comm, int32_t rounds, int32_t chunks);

/* Message options of later sorts on this communicator. self_messages = 1:
 * this rank's own pieces travel as transport messages to itself (a send and
 * a receive inside the round's group, as a peer's do) instead of device
 * copies, so that one rank exercises every transport call of the exchange
 * (the receive buffer then never aliases the partition buffer).
 * max_message_bytes: the largest single message, a multiple of 64 in
 * [64, 2^30]; 0 = the default 256 MiB (RCCL corrupts messages above 1 GiB,
 * DESIGN.md §7). Every rank must use the same cap (checked like the options
 * above); self messages are a rank's own choice. */
int srs_shard_set_message_options(srs_shard_comm comm, int32_t self_messages,
                                  int64_t max_message_bytes);

/* This rank's part of the shard sort of device columns (inputs untouched):
 * *keys_out / payloads_out[k] receive device pointers to this rank's sorted
 * key range and *num_out its length; the memory belongs to the communicator
 * and stays valid until its next sort or its destruction. Work runs on
 * `stream` (and the communicator's own streams); the call returns when the
 * sort is complete. Every rank of the communicator must call it. */
int srs_shard_sort_device(srs_shard_comm comm, int64_t num, int key_kind, int up,
                          const void* keys, int32_t num_payloads, const void* const* payloads,
                          const uint32_t* payload_sizes, void** keys_out, void** payloads_out,
                          int64_t* num_out, void* stream);

/* All ranks of a single-process communicator set at once (one host thread
 * per rank; synchronous): rank i sorts nums[i] records at keys[i] and
 * payloads[i * num_payloads + k]; outputs as above, per rank. */
int srs_shard_sort_multi(int32_t num_devices, const srs_shard_comm* comms, const int64_t* nums,
                         int key_kind, int up, const void* const* keys, int32_t num_payloads,
                         const void* const* payloads, const uint32_t* payload_sizes,
                         void** keys_out, void** payloads_out, int64_t* nums_out);

/* The last successful sort on this communicator as JSON: transport, world,
 * rank, chunks, rounds, groups, records in / out, record bytes, "stamps_ms"
 * (HIP-event times since its start of: hist, plan, partition<c>,
 * round<r>_recv, round<r>_sort_start, round<r>_sort_end, end) and
 * "bytes_to_peer_per_round" ([round][peer] bytes this rank sent; itself too
 * with self messages), self_messages, max_message_bytes, sends / recvs (the
 * transport calls posted) and deferred_frees (workspace buffers that grew
 * during the exchange; their old memory is freed after it). */
int srs_shard_last_report(srs_shard_comm comm, char* buf, int64_t cap);

/* Test hook: the next sort on this communicator fails at `point` (0 = none,
 * 1 = argument error, 2 = allocation before the exchange, 3 = partition
 * after the first messages, 4 = the last round's sort, 5 = transport
 * failure after the first messages: aborts). */
int srs_shard_debug_inject(srs_shard_comm comm, int32_t point);

/* The shard plan of one rank, host only (no GPU): from every rank's chunk
 * histograms (chunk_hists[src][chunk][2^min(12, key_bits)] of the
 * transformed top key bits), this rank's record count and whether its own
 * pieces travel as self messages (srs_shard_set_message_options), the JSON of
 * group_of_bin, rank_of_group, chunk_bounds, total (records received),
 * "posts" (every message group in posting order: its (round, chunk) pieces
 * and msgs = [op (0 send, 1 receive, 2 own-piece copy), peer, partitioned
 * offset, receive offset, records]) and "rounds" (each round's receive
 * range, its sort segments and known top bits). The same code plans the
 * device sort; tests drive the protocol with it on CPU (gloo). */
int srs_debug_shard_plan(int32_t world, int32_t rank, int32_t chunks, int32_t rounds,
                         int32_t key_bits, int32_t self_messages, const uint64_t* chunk_hists,
                         int64_t num, char* json, int64_t cap);

/* ---- host arrays over several GPUs --------------------------------------- */

/* Devices the host-pointer entry points (srs_sort_soa, srs_sort_soa_leaf)
 * may use. 0 devices (the default) = the calling thread's current device.
 * With G > 1 devices a large SoA sort (>= 2^22 keys) splits the host array
 * G ways: chunk g goes over device g's own PCIe link, the chunks are
 * partitioned into G key ranges (a stable top-bits radix level), range h is
 * gathered on device h over xGMI, sorted there and copied back to its place.
 * The result is the same array a one-device sort gives. A device may be
 * listed more than once (its shards then share it). The environment
 * variable SRS_HOST_DEVICES ("all" or "0,1,2") sets the initial list. The
 * reference sorts on one host thread and has no counterpart. */
int srs_set_host_devices(int32_t num_devices, const int32_t* devices);

/* ---- device memory for sort buffers --------------------------------------- */

/* Allocates `bytes` of device memory on the current device for arrays the
 * sort will write (out-of-place outputs, in-place arrays). The scatter's
 * write rate depends on where a buffer sits in HBM (the same
 * kernel writes some allocations ~13 % slower); buffers of 256 MB and more
 * are probed with the sort's write pattern and re-placed (up to 6 tries,
 * while free memory allows) when slower than the fastest placement seen.
 * The sort's own workspace is placed the same way. SRS_PLACE=0 turns the
 * probing off. srs_free_device releases it. No counterpart in the
 * reference (host arrays only). */
int srs_alloc_device(uint64_t bytes, void** ptr);
int srs_free_device(void* ptr);

/* ---- synthetic data (bench / tests) ------------------------------------- */

/* keys[i] = splitmix64(seed + first_index + i) truncated/reinterpreted to the
 * key kind (floats: uniform in [-1,1) on a 2^-23 / 2^-52 grid); payload column
 * c gets the low bytes of splitmix64(bits(key[i]) ^ c * 0xD1B54A32D192ED03)
 * (a function of the key). */
int srs_fill_synthetic_device(int64_t num, int key_kind, uint64_t seed,
                              uint64_t first_index, void* keys,
                              int32_t num_payloads, void* const* payloads,
                              const uint32_t* payload_sizes, void* stream);

/* ---- diagnostics ---------------------------------------------------------- */

/* Thread-local description of the last error (never NULL). */
const char* srs_last_error(void);

/* Library version string ("srs_amd <semver> gfx950"). */
const char* srs_version(void);

/* Per-kernel timing with HIP events recorded on the launch stream around
 * every kernel launch (enable 1; off by default; 2: around the scatter
 * launches only, as bench.py's timed region). srs_kernel_stats fills, for kernel
 * name `name` ("count", "scatter", "local", "scan", ...), the number of
 * launches and the summed device milliseconds since the last reset; the
 * stream must have completed. Returns SRS_ERR_INVALID_ARG for unknown names. */
int srs_set_kernel_timing(int enable);
int srs_reset_kernel_stats(void);
int srs_kernel_stats(const char* name, int64_t* launches, double* total_ms,
                     double* elements);

/* Diagnostic builds only (-DSRS_STAMPS=1): device buffer of 64 uint64 that
 * accumulates per-phase s_memtime cycles of the scatter (slots 0..15) and
 * local (16..31) kernels; NULL disables. No effect in the product build. */
int srs_debug_set_stamp_buffer(void* device_acc);

/* Diagnostic builds only (-DSRS_DIAG_LOOKBACK): the scatter also runs a
 * decoupled look-back over its tiles and checks it against the count pass's
 * offsets. status: >= ntiles * 512 uint32 of device memory; err: 4 uint64
 * (mismatches, spin timeouts, look-back hops of digit 0). NULL disables. */
int srs_debug_set_lookback(void* status, void* err);

/* The super-group column scan: a level over one large segment
 * scans sums of 64 scan groups once it has at least min_groups groups of 32
 * tiles (default 256, i.e. 33.5 M keys; <= 0 restores it). Process-wide;
 * tests lower it so that the path runs at small sizes. */
int srs_debug_set_super_scan(int64_t min_groups);

/* Segments the local-level fallback kernels took in the last sort on the
 * current device: counts[0] = handed to the stable kernel, counts[1] = handed
 * on to the LSD kernel. Synchronizes the device. Tests use it to prove that
 * an input exercised a given path. */
int srs_debug_last_fallbacks(int64_t* counts);

/* Local-level segment counts of the last (non-small) sort on the current
 * device: counts[0] = segments of the local level, counts[1] = of those, the
 * ones the direct local kernel handed to the fast kernel.
 * Synchronizes the device. Tests use it to prove the direct kernel ran. */
int srs_debug_last_local_counts(int64_t* counts);

/* The same by LDS class: counts[0] / counts[1] = small (<= 4096 records) /
 * large (<= 8192) segments of the local level, counts[2] / counts[3] = of
 * those, the ones the direct kernel of the class handed to the fast kernel.
 * Synchronizes the device. */
int srs_debug_last_local_classes(int64_t* counts);

/* Placement diagnostics. srs_debug_alloc allocates `bytes` of
 * device memory on the current device the way mode says (0 = hipMalloc,
 * 1 = physically contiguous, 2 = one hipMemCreate handle mapped at 1 GiB
 * alignment, 3 / 4 = 2 MB handles mapped in a shuffled order / in order; the
 * workspace's own big buffers follow SRS_WS_ALLOC = malloc|contig|vmm|
 * vmmshuf|vmm2m);
 * srs_debug_free releases it. srs_debug_workspace reports the current
 * device's TMP and TMP2 buffers (NULL / 0 when not allocated). */
int srs_debug_alloc(uint64_t bytes, int mode, void** ptr);
int srs_debug_free(void* ptr);
int srs_debug_workspace(void** tmp, uint64_t* tmp_bytes, void** tmp2, uint64_t* tmp2_bytes);
/* Milliseconds of one pass of the scatter's write pattern (512 runs of 8
 * elements per 4096-element tile into 16 MB windows) over [ptr, ptr + bytes)
 * of device memory: the rate the sort's scatter and local passes can write
 * that memory at. Synchronizes the device. */
int srs_debug_probe_write(void* ptr, uint64_t bytes, float* ms);

/* The balanced first level's digit table, planned on the host from a
 * 65536-bin histogram of the top 16 transformed key bits (the sample the
 * sort takes of large inputs) for `num` input keys of key_bits (32 / 64):
 * *mode 0 (no table), 1 (table = 65536 group ids, one per 16-bit bin) or 3
 * (table = 512 split entries: first group | lg << 16 per top-9-bit bin);
 * rbits = 512 per-group unsorted bit counts; *overflow = keys the next
 * level is predicted to leave above the LDS capacity (overflow_other: for
 * the other table). Host only (no GPU); tests check the plan with it. */
int srs_debug_plan_table(const uint32_t* hist, int64_t num, int key_bits, int32_t* mode,
                         int32_t* groups, double* overflow, double* overflow_other,
                         int32_t* table, int32_t* rbits);

/* Release cached device workspaces (for leak checks / shutdown). */
int srs_release_workspace(void);

#ifdef __cplusplus
}
#endif

#endif /* SRS_C_API_H_ */

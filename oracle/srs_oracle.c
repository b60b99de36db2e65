/*
 * srs_oracle.c — plain-C restatement of jonicho/simd-radix-sort's hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see srs_oracle.h). Not part of the product.
 *
 * What is restated, with the reference location each piece follows
 * (paths relative to /root/reference):
 *   key_bits / is_bit_set   radixSort.hpp:1543-1552 (isBitSet: bit_cast to
 *                           UInt<sizeof K>, DataElement -> .key)
 *   bit_dir_up              radixSort.hpp:1568-1581 (bitDirUp)
 *   sort_bit_simd           radixSort.hpp:1587-1686 (BitSorterSIMD::sortBit)
 *                           with getSortMasks :1689-1704 and
 *                           compress_store_left_right :1706-1731; a "vector"
 *                           is V = 64 / sizeof(K) consecutive elements
 *                           (numElemsPerVec :1585), emulated lane by lane
 *                           (loadu / maskz_loadu / mask_compressstoreu /
 *                           kpopcnt, src/simd.hpp:195-389, :1292-1299)
 *   sort_bit_seq            src/radix_sort.hpp:66-92 (BitSorterSequential)
 *   insertion_sort          radixSort.hpp:159-178 (CmpSorterInsertionSort:
 *                           stable, uses the key type's operator< / >)
 *   radix_recursion         radixSort.hpp:1734-1759 (radixRecursion)
 *   entry points            radixSort.hpp:1761-1783
 *
 * Data model: a sort call is a set of parallel "streams" (the key column and
 * each payload column for SoA; one stream of whole DataElement records for
 * AoS). Every element move is applied to all streams, like the reference's
 * mirrored key/payload loads and stores.
 */
#include "srs_oracle.h"

#include <stdlib.h>
#include <string.h>

enum {
  K_U8 = 0, K_I8, K_U16, K_I16, K_U32, K_I32, K_U64, K_I64, K_F32, K_F64
};

#define MAX_STREAMS 65

typedef struct {
  int nstreams;
  uint8_t* ptr[MAX_STREAMS];
  uint32_t size[MAX_STREAMS];
  int key_kind;
  int key_size;
  int64_t V;               /* elements per emulated 64-byte vector */
  int64_t thresh;          /* cmpSortThreshold */
  int up;
  /* scratch: three vectors (store, current, rest) + one element */
  uint8_t* vec[3][MAX_STREAMS];
  uint8_t* tmp[MAX_STREAMS];
} ctx_t;

static int key_size_of(int kind) {
  switch (kind) {
    case K_U8: case K_I8: return 1;
    case K_U16: case K_I16: return 2;
    case K_U32: case K_I32: case K_F32: return 4;
    case K_U64: case K_I64: case K_F64: return 8;
    default: return 0;
  }
}

static inline void copy_elem(uint8_t* dst, const uint8_t* src, uint32_t sz) {
  switch (sz) {
    case 1: *dst = *src; break;
    case 2: memcpy(dst, src, 2); break;
    case 4: memcpy(dst, src, 4); break;
    case 8: memcpy(dst, src, 8); break;
    default: memcpy(dst, src, sz); break;
  }
}

/* Raw key bits of a stored key (little endian, key at byte 0 of stream 0). */
static inline uint64_t key_bits_at(const ctx_t* c, const uint8_t* p) {
  uint64_t v = 0;
  memcpy(&v, p, (size_t)c->key_size);
  return v;
}

/* isBitSet, radixSort.hpp:1543-1552 */
static inline int is_bit_set(const ctx_t* c, const uint8_t* p, int bit_no) {
  return (int)((key_bits_at(c, p) >> bit_no) & 1u);
}

/* bitDirUp<T,Up,IsHighestBit,IsRightSide>, radixSort.hpp:1568-1581 */
static inline int bit_dir_up(int kind, int up, int is_highest, int is_right) {
  switch (kind) {
    case K_U8: case K_U16: case K_U32: case K_U64:
      return up;
    case K_I8: case K_I16: case K_I32: case K_I64:
      return is_highest ? !up : up;
    case K_F32: case K_F64:
      return is_highest ? !up : is_right;
    default:
      return up;
  }
}

/* operator< of the key type (DataElement::operator< compares .key,
 * src/data.hpp:29-30). Floats compare by value: -0.0 == +0.0. */
static inline int key_less(int kind, const uint8_t* a, const uint8_t* b) {
  switch (kind) {
    case K_U8: return *(const uint8_t*)a < *(const uint8_t*)b;
    case K_I8: return *(const int8_t*)a < *(const int8_t*)b;
    case K_U16: { uint16_t x, y; memcpy(&x, a, 2); memcpy(&y, b, 2); return x < y; }
    case K_I16: { int16_t x, y; memcpy(&x, a, 2); memcpy(&y, b, 2); return x < y; }
    case K_U32: { uint32_t x, y; memcpy(&x, a, 4); memcpy(&y, b, 4); return x < y; }
    case K_I32: { int32_t x, y; memcpy(&x, a, 4); memcpy(&y, b, 4); return x < y; }
    case K_U64: { uint64_t x, y; memcpy(&x, a, 8); memcpy(&y, b, 8); return x < y; }
    case K_I64: { int64_t x, y; memcpy(&x, a, 8); memcpy(&y, b, 8); return x < y; }
    case K_F32: { float x, y; memcpy(&x, a, 4); memcpy(&y, b, 4); return x < y; }
    case K_F64: { double x, y; memcpy(&x, a, 8); memcpy(&y, b, 8); return x < y; }
    default: return 0;
  }
}

static inline uint8_t* elem(const ctx_t* c, int s, int64_t i) {
  return c->ptr[s] + (size_t)i * c->size[s];
}

/* CmpSorterInsertionSort::sort, radixSort.hpp:159-178 */
static void insertion_sort(ctx_t* c, int64_t left, int64_t right) {
  for (int64_t i = left + 1; i <= right; i++) {
    for (int s = 0; s < c->nstreams; s++) copy_elem(c->tmp[s], elem(c, s, i), c->size[s]);
    int64_t j = i;
    while (j > left && (c->up ? key_less(c->key_kind, c->tmp[0], elem(c, 0, j - 1))
                              : key_less(c->key_kind, elem(c, 0, j - 1), c->tmp[0]))) {
      for (int s = 0; s < c->nstreams; s++) copy_elem(elem(c, s, j), elem(c, s, j - 1), c->size[s]);
      j--;
    }
    for (int s = 0; s < c->nstreams; s++) copy_elem(elem(c, s, j), c->tmp[s], c->size[s]);
  }
}

/* --- vector emulation (src/simd.hpp loadu / maskz_loadu / compressstoreu) --- */

/* loadu: V consecutive elements of every stream into vector slot `slot`. */
static inline void vec_load(ctx_t* c, int slot, int64_t pos, int64_t count) {
  for (int s = 0; s < c->nstreams; s++) {
    memcpy(c->vec[slot][s], elem(c, s, pos), (size_t)count * c->size[s]);
    if (count < c->V)  /* maskz_loadu: masked lanes are zero */
      memset(c->vec[slot][s] + (size_t)count * c->size[s], 0,
             (size_t)(c->V - count) * c->size[s]);
  }
}

/* getSortMasks (radixSort.hpp:1689-1704): lane mask of elements whose
 * tested bit equals `dir_up` goes RIGHT; the complement goes LEFT. */
static inline void sort_masks(const ctx_t* c, int slot, int bit_no, int dir_up,
                              uint64_t* left, uint64_t* right) {
  uint64_t set = 0;
  for (int64_t l = 0; l < c->V; l++)
    if (is_bit_set(c, c->vec[slot][0] + (size_t)l * c->size[0], bit_no)) set |= 1ull << l;
  const uint64_t all = (c->V == 64) ? ~0ull : ((1ull << c->V) - 1);
  if (dir_up) { *right = set; *left = all & ~set; }
  else { *left = set; *right = all & ~set; }
}

/* mask_compressstoreu on every stream: selected lanes, in lane order,
 * stored contiguously from element position `pos`. */
static inline void compress_store(ctx_t* c, int slot, int64_t pos, uint64_t mask) {
  int64_t w = pos;
  for (int64_t l = 0; l < c->V; l++) {
    if (!((mask >> l) & 1)) continue;
    for (int s = 0; s < c->nstreams; s++)
      copy_elem(elem(c, s, w), c->vec[slot][s] + (size_t)l * c->size[s], c->size[s]);
    w++;
  }
}

static inline int64_t popc(uint64_t m) { return (int64_t)__builtin_popcountll(m); }

/* BitSorterSIMD::sortBit, radixSort.hpp:1587-1686 (line-by-line order of
 * loads and stores preserved: the next vector is loaded before the current
 * one is compress-stored). */
static int64_t sort_bit_simd(ctx_t* c, int bit_no, int64_t left, int64_t right,
                             int dir_up) {
  const int64_t V = c->V;
  const int64_t num_elems = right - left + 1;
  int64_t read_left = left;
  int64_t read_right = right - V + 1;
  int64_t write_left = left;
  int64_t write_right = right;
  enum { STORE = 0, CUR = 1, REST = 2 };

  if (num_elems >= V) {                                   /* :1603-1609 */
    vec_load(c, STORE, read_left, V);
    read_left += V;
  }
  while (read_left <= read_right) {                        /* :1611-1640 */
    /* keyVec = keyVecStore */
    for (int s = 0; s < c->nstreams; s++)
      memcpy(c->vec[CUR][s], c->vec[STORE][s], (size_t)V * c->size[s]);
    uint64_t ml, mr;
    sort_masks(c, CUR, bit_no, dir_up, &ml, &mr);
    const int64_t n_left = popc(ml);
    const int64_t n_right = V - n_left;
    if ((read_left - write_left) >= n_left) {
      vec_load(c, STORE, read_right, V);
      read_right -= V;
    } else {
      vec_load(c, STORE, read_left, V);
      read_left += V;
    }
    compress_store(c, CUR, write_left, ml);
    compress_store(c, CUR, write_right - n_right + 1, mr);
    write_left += n_left;
    write_right -= n_right;
  }

  const int64_t num_rest = read_right + V - read_left;    /* :1642 */
  uint64_t rest_mask = 0;
  if (num_rest != 0) {                                     /* :1644-1654 */
    rest_mask = (num_rest == 64) ? ~0ull : ((1ull << num_rest) - 1);
    vec_load(c, REST, read_left, num_rest);
    read_left += num_rest;
  }
  if (num_elems >= V) {                                    /* :1656-1666 */
    uint64_t ml, mr;
    sort_masks(c, STORE, bit_no, dir_up, &ml, &mr);
    const int64_t n_left = popc(ml);
    const int64_t n_right = V - n_left;
    compress_store(c, STORE, write_left, ml);
    compress_store(c, STORE, write_right - n_right + 1, mr);
    write_left += n_left;
    write_right -= n_right;
  }
  if (num_rest != 0) {                                     /* :1668-1684 */
    uint64_t ml, mr;
    sort_masks(c, REST, bit_no, dir_up, &ml, &mr);
    ml &= rest_mask;
    mr &= rest_mask;
    const int64_t n_left = popc(ml);
    const int64_t n_right = num_rest - n_left;
    compress_store(c, REST, write_left, ml);
    compress_store(c, REST, write_left + n_left, mr);
    write_left += n_left;
    write_right -= n_right;
  }
  return write_left;
}

/* BitSorterSequential::sortBit, src/radix_sort.hpp:66-92 */
static int64_t sort_bit_seq(ctx_t* c, int bit_no, int64_t left, int64_t right,
                            int dir_up) {
  int64_t l = left, r = right;
  while (l <= r) {
    while (l <= r && (dir_up != is_bit_set(c, elem(c, 0, l), bit_no))) l++;
    while (l <= r && ((!dir_up) != is_bit_set(c, elem(c, 0, r), bit_no))) r--;
    if (l < r) {
      for (int s = 0; s < c->nstreams; s++) {
        copy_elem(c->tmp[s], elem(c, s, l), c->size[s]);
        copy_elem(elem(c, s, l), elem(c, s, r), c->size[s]);
        copy_elem(elem(c, s, r), c->tmp[s], c->size[s]);
      }
    }
  }
  return l;
}

/* radixRecursion, radixSort.hpp:1734-1759 */
static void radix_recursion(ctx_t* c, int bit_sorter, int is_right, int is_highest,
                            int bit_no, int64_t left, int64_t right) {
  if (right - left <= 0) return;
  if (right - left < c->thresh) {
    insertion_sort(c, left, right);
    return;
  }
  const int dir = bit_dir_up(c->key_kind, c->up, is_highest, is_right);
  const int64_t split = bit_sorter == 0 ? sort_bit_simd(c, bit_no, left, right, dir)
                                        : sort_bit_seq(c, bit_no, left, right, dir);
  if (bit_no > 0) {
    radix_recursion(c, bit_sorter, is_highest ? 0 : is_right, 0, bit_no - 1, left, split - 1);
    radix_recursion(c, bit_sorter, is_highest ? 1 : is_right, 0, bit_no - 1, split, right);
  }
}

static int run(ctx_t* c, int64_t num, int bit_sorter) {
  int rc = 0;
  for (int s = 0; s < c->nstreams; s++) {
    for (int v = 0; v < 3; v++) {
      c->vec[v][s] = (uint8_t*)malloc((size_t)c->V * c->size[s]);
      if (!c->vec[v][s]) rc = -1;
    }
    c->tmp[s] = (uint8_t*)malloc(c->size[s]);
    if (!c->tmp[s]) rc = -1;
  }
  if (rc == 0)  /* sort(): radixRecursion(sizeof(K)*8-1, thresh, 0, num-1, ...) */
    radix_recursion(c, bit_sorter, 0, 1, 8 * c->key_size - 1, 0, num - 1);
  for (int s = 0; s < c->nstreams; s++) {
    for (int v = 0; v < 3; v++) free(c->vec[v][s]);
    free(c->tmp[s]);
  }
  return rc;
}

int srs_oracle_sort_soa(int64_t num, int key_kind, int up,
                        int64_t cmp_sort_threshold, void* keys,
                        int32_t num_payloads, void* const* payloads,
                        const uint32_t* payload_sizes, int bit_sorter) {
  ctx_t c;
  memset(&c, 0, sizeof c);
  c.key_size = key_size_of(key_kind);
  if (c.key_size == 0 || num_payloads < 0 || num_payloads >= MAX_STREAMS) return -1;
  if (num <= 1) return 0;
  c.key_kind = key_kind;
  c.up = up ? 1 : 0;
  c.thresh = cmp_sort_threshold;
  c.V = 64 / c.key_size;
  c.nstreams = 1 + num_payloads;
  c.ptr[0] = (uint8_t*)keys;
  c.size[0] = (uint32_t)c.key_size;
  for (int i = 0; i < num_payloads; i++) {
    c.ptr[1 + i] = (uint8_t*)payloads[i];
    c.size[1 + i] = payload_sizes[i];
    if (payload_sizes[i] == 0) return -1;
  }
  return run(&c, num, bit_sorter);
}

int srs_oracle_sort_aos(int64_t num, int key_kind, int up,
                        int64_t cmp_sort_threshold, void* elements,
                        uint32_t elem_size, int bit_sorter) {
  ctx_t c;
  memset(&c, 0, sizeof c);
  c.key_size = key_size_of(key_kind);
  /* static_assert(is_power_of_two<sizeof(DataElement<K, Ps...>)>),
   * radixSort.hpp:1774; at most one element per 64-byte vector. */
  if (c.key_size == 0 || elem_size < (uint32_t)c.key_size || elem_size > 64 ||
      (elem_size & (elem_size - 1)) != 0)
    return -1;
  if (num <= 1) return 0;
  c.key_kind = key_kind;
  c.up = up ? 1 : 0;
  c.thresh = cmp_sort_threshold;
  c.V = 64 / elem_size;   /* numElemsPerVec with K = DataElement */
  c.nstreams = 1;
  c.ptr[0] = (uint8_t*)elements;
  c.size[0] = elem_size;
  return run(&c, num, bit_sorter);
}

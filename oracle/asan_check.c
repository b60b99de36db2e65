/*
 * asan_check.c — sanitizer run of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * Built with -fsanitize=address,undefined (oracle/Makefile target `asan`)
 * and run by tests/test_oracle.py. Sorts seeded random inputs of every key
 * kind, both directions, SoA with 0-3 payload columns of mixed widths and
 * AoS records of 2..64 bytes, at sizes around the leaf threshold and the
 * vector widths of the emulated BitSorterSIMD (radixSort.hpp:1587-1686),
 * and checks the reference's own invariants (src/data.hpp:272-310): keys in
 * order, payload = f(key) for every record, and the key multiset unchanged
 * (an order-independent sum). The sanitizers catch any out-of-bounds access
 * in the lane-by-lane compress-store emulation.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srs_oracle.h"

static uint64_t sm(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

static const int ksz[10] = {1, 1, 2, 2, 4, 4, 8, 8, 4, 8};

/* transformed key: unsigned order == the reference's order (Up) */
static uint64_t ukey(int kind, const unsigned char* p) {
  uint64_t b = 0;
  memcpy(&b, p, ksz[kind]);
  const int kb = 8 * ksz[kind];
  const uint64_t sb = 1ull << (kb - 1), all = kb == 64 ? ~0ull : ((1ull << kb) - 1);
  if (kind == 8 || kind == 9) return (b & sb) ? (~b & all) : (b ^ sb);
  if (kind == 1 || kind == 3 || kind == 5 || kind == 7) return b ^ sb;
  return b;
}

/* keys: random bits, low-entropy values, or a few distinct ones; floats are
 * kept finite and non-zero (NaN and -0.0/+0.0 ties are outside parity) */
static void gen_key(int kind, uint64_t r, int mode, unsigned char* out) {
  uint64_t v = mode == 0 ? r : mode == 1 ? (r & 7) : (r % 3) * 0x0101010101010101ull;
  if (kind == 8) {
    float f = (float)((double)(int64_t)(r >> 11) / 9007199254740992.0 * 2e3 + 1e-3);
    memcpy(out, &f, 4);
    return;
  }
  if (kind == 9) {
    double d = (double)(int64_t)(r >> 11) / 9007199254740992.0 * 2e9 + 1e-9;
    memcpy(out, &d, 8);
    return;
  }
  memcpy(out, &v, ksz[kind]);
}

static int failures = 0;
#define CHECK(c, ...)                 \
  do {                                \
    if (!(c)) {                       \
      fprintf(stderr, __VA_ARGS__);   \
      fprintf(stderr, "\n");          \
      failures++;                     \
      return;                         \
    }                                 \
  } while (0)

static void run_soa(int kind, int up, int64_t n, int mode, int npay, uint64_t seed) {
  const uint32_t psz[3] = {8, 1, 4};
  const int ks = ksz[kind];
  unsigned char* keys = malloc(n * ks + 1);
  void* pays[3];
  uint64_t sum = 0;
  for (int64_t i = 0; i < n; i++) {
    gen_key(kind, sm(seed + i), mode, keys + i * ks);
    sum += ukey(kind, keys + i * ks);
  }
  for (int c = 0; c < npay; c++) {
    pays[c] = malloc(n * psz[c] + 1);
    for (int64_t i = 0; i < n; i++) {
      uint64_t f = sm(ukey(kind, keys + i * ks) ^ (uint64_t)(c + 1));
      memcpy((char*)pays[c] + i * psz[c], &f, psz[c]);
    }
  }
  CHECK(srs_oracle_sort_soa(n, kind, up, 16, keys, npay, pays, psz, 0) == 0, "soa call");
  uint64_t sum2 = 0;
  for (int64_t i = 0; i < n; i++) {
    const uint64_t u = ukey(kind, keys + i * ks);
    sum2 += u;
    if (i) {
      const uint64_t p = ukey(kind, keys + (i - 1) * ks);
      CHECK(up ? p <= u : p >= u, "soa order kind %d up %d n %lld at %lld", kind, up,
            (long long)n, (long long)i);
    }
    for (int c = 0; c < npay; c++) {
      uint64_t f = sm(u ^ (uint64_t)(c + 1)), g = 0;
      memcpy(&g, (char*)pays[c] + i * psz[c], psz[c]);
      CHECK(!memcmp(&f, &g, psz[c]), "soa payload kind %d col %d at %lld", kind, c, (long long)i);
    }
  }
  CHECK(sum == sum2, "soa key multiset kind %d n %lld", kind, (long long)n);
  for (int c = 0; c < npay; c++) free(pays[c]);
  free(keys);
}

static void run_aos(int kind, int up, int64_t n, uint32_t esz, uint64_t seed) {
  const int ks = ksz[kind];
  if ((uint32_t)ks > esz) return;
  unsigned char* rec = malloc(n * esz + 1);
  uint64_t sum = 0;
  for (int64_t i = 0; i < n; i++) {
    unsigned char* r = rec + i * esz;
    memset(r, 0, esz);
    gen_key(kind, sm(seed + i), 0, r);
    const uint64_t u = ukey(kind, r);
    sum += u;
    for (uint32_t b = ks; b < esz; b++) r[b] = (unsigned char)(sm(u + b) & 0xFF);
  }
  CHECK(srs_oracle_sort_aos(n, kind, up, 16, rec, esz, 0) == 0, "aos call");
  uint64_t sum2 = 0;
  for (int64_t i = 0; i < n; i++) {
    const unsigned char* r = rec + i * esz;
    const uint64_t u = ukey(kind, r);
    sum2 += u;
    if (i) {
      const uint64_t p = ukey(kind, rec + (i - 1) * esz);
      CHECK(up ? p <= u : p >= u, "aos order kind %d esz %u at %lld", kind, esz, (long long)i);
    }
    for (uint32_t b = ks; b < esz; b++)
      CHECK(r[b] == (unsigned char)(sm(u + b) & 0xFF), "aos payload kind %d esz %u", kind, esz);
  }
  CHECK(sum == sum2, "aos key multiset kind %d esz %u", kind, esz);
  free(rec);
}

int main(void) {
  const int64_t sizes[] = {0, 1, 2, 15, 16, 17, 63, 64, 65, 257, 1000, 4099};
  int cases = 0;
  for (int kind = 0; kind < 10; kind++)
    for (int up = 0; up < 2; up++)
      for (size_t s = 0; s < sizeof sizes / sizeof sizes[0]; s++) {
        for (int mode = 0; mode < 3; mode++)
          for (int np = 0; np <= 3; np += 3 - (mode != 0) * 2) {
            run_soa(kind, up, sizes[s], mode, np, 1000u * kind + 7u * s + mode);
            cases++;
          }
        for (uint32_t esz = 2; esz <= 64; esz *= 2) {
          run_aos(kind, up, sizes[s], esz, 77u * kind + s + esz);
          cases++;
        }
      }
  printf("asan_check: %d cases, %d failures\n", cases, failures);
  return failures ? 1 : 0;
}

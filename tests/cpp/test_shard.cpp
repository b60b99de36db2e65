// test_shard.cpp — the multi-GPU shard sort through the C ABI (RCCL and the
// host-staged transport)
// (srs_shard_*), driven from C++ with no torch: the
// single-process communicator (srs_shard_comm_init_all + srs_shard_sort_multi)
// and the one-process-per-GPU one (srs_shard_unique_id + srs_shard_comm_init
// + srs_shard_sort_device) at world 1 on one GPU, each checked against the
// plain one-GPU sort (srs_sort_soa_device) bit for bit. The input and the
// shard output are written to <prefix>_{in,out}_{k,p}.bin, so that
// tests/test_cpp_dropin.py can compare them with the reference's own sort.
// usage: test_shard <n> <prefix>
#include <hip/hip_runtime.h>
#include <srs_c_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    int rc_ = (int)(x);                                                           \
    if (rc_ != 0) {                                                               \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,       \
              srs_last_error());                                                  \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

static int save(const std::string& path, const void* p, size_t bytes) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return 1;
  const size_t w = fwrite(p, 1, bytes, f);
  fclose(f);
  return w == bytes ? 0 : 1;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (int64_t(1) << 22);
  const std::string prefix = argc > 2 ? argv[2] : "/tmp/srs_shard";
  const size_t bytes = (size_t)n * 8;
  int dev = 0;
  CK(hipGetDevice(&dev));
  void *keys, *pays;
  CK(hipMalloc(&keys, bytes));
  CK(hipMalloc(&pays, bytes));
  const uint32_t psz[1] = {8};
  void* pl[1] = {pays};
  CK(srs_fill_synthetic_device(n, SRS_KEY_U64, 9ull << 32, 0, keys, 1, pl, psz, nullptr));
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> hk(n), hp(n), rk(n), rp(n), sk(n), sp(n);
  CK(hipMemcpy(hk.data(), keys, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hp.data(), pays, bytes, hipMemcpyDeviceToHost));
  CK(save(prefix + "_in_k.bin", hk.data(), bytes));
  CK(save(prefix + "_in_p.bin", hp.data(), bytes));

  // the plain one-GPU sort (out of place) as the yardstick
  void *ko, *po;
  CK(hipMalloc(&ko, bytes));
  CK(hipMalloc(&po, bytes));
  void* pol[1] = {po};
  CK(srs_sort_soa_device(n, SRS_KEY_U64, 1, 16, keys, 1, pl, psz, ko, pol, nullptr));
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(rk.data(), ko, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(rp.data(), po, bytes, hipMemcpyDeviceToHost));

  // 1. single-process communicator over this GPU (world 1)
  srs_shard_comm comm = nullptr;
  const int32_t devs[1] = {dev};
  CK(srs_shard_comm_init_all(1, devs, &comm));
  const int64_t nums[1] = {n};
  const void* kin[1] = {keys};
  const void* pin[1] = {pays};
  void* kout[1] = {nullptr};
  void* pout[1] = {nullptr};
  int64_t nout[1] = {0};
  CK(srs_shard_sort_multi(1, &comm, nums, SRS_KEY_U64, 1, kin, 1, pin, psz, kout, pout, nout));
  if (nout[0] != n) {
    fprintf(stderr, "shard (multi): %lld records out, %lld in\n", (long long)nout[0], (long long)n);
    return 1;
  }
  CK(hipMemcpy(sk.data(), kout[0], bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(sp.data(), pout[0], bytes, hipMemcpyDeviceToHost));
  if (memcmp(sk.data(), rk.data(), bytes) || memcmp(sp.data(), rp.data(), bytes)) {
    fprintf(stderr, "shard (multi) differs from the one-GPU sort\n");
    return 1;
  }
  CK(save(prefix + "_out_k.bin", sk.data(), bytes));
  CK(save(prefix + "_out_p.bin", sp.data(), bytes));
  // the input is untouched
  std::vector<uint64_t> again(n);
  CK(hipMemcpy(again.data(), keys, bytes, hipMemcpyDeviceToHost));
  if (memcmp(again.data(), hk.data(), bytes)) {
    fprintf(stderr, "shard changed its input\n");
    return 1;
  }
  CK(srs_shard_comm_destroy(comm));

  // 2. one-process-per-GPU communicator (rank 0 of world 1), on a stream
  char id[SRS_SHARD_ID_BYTES];
  CK(srs_shard_unique_id(id));
  srs_shard_comm c2 = nullptr;
  CK(srs_shard_comm_init(1, 0, id, &c2));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  void* k2 = nullptr;
  void* p2[1] = {nullptr};
  int64_t n2 = 0;
  CK(srs_shard_sort_device(c2, n, SRS_KEY_U64, 1, keys, 1, pin, psz, &k2, p2, &n2, st));
  CK(hipStreamSynchronize(st));
  if (n2 != n) return 1;
  CK(hipMemcpy(sk.data(), k2, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(sp.data(), p2[0], bytes, hipMemcpyDeviceToHost));
  if (memcmp(sk.data(), rk.data(), bytes) || memcmp(sp.data(), rp.data(), bytes)) {
    fprintf(stderr, "shard (per-rank) differs from the one-GPU sort\n");
    return 1;
  }
  CK(srs_shard_comm_destroy(c2));
  CK(hipStreamDestroy(st));

  // 3. three ranks on this GPU over the host-staged transport: the input cut
  // into three ragged shards; the concatenated outputs equal the sort
  {
    const int W = 3;
    srs_shard_comm cs[W];
    CK(srs_shard_comm_init_staged(W, cs));
    const int64_t cut[W + 1] = {0, n / 7, n / 7 + n / 2, n};
    int64_t nm[W];
    const void* km[W];
    const void* pm[W];
    void* ko3[W];
    void* po3[W];
    int64_t no3[W];
    for (int r = 0; r < W; r++) {
      nm[r] = cut[r + 1] - cut[r];
      km[r] = (const char*)keys + cut[r] * 8;
      pm[r] = (const char*)pays + cut[r] * 8;
    }
    CK(srs_shard_sort_multi(W, cs, nm, SRS_KEY_U64, 1, km, 1, pm, psz, ko3, po3, no3));
    int64_t at = 0;
    for (int r = 0; r < W; r++) {
      if (at + no3[r] > n) return 1;
      CK(hipMemcpy(sk.data() + at, ko3[r], (size_t)no3[r] * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(sp.data() + at, po3[r], (size_t)no3[r] * 8, hipMemcpyDeviceToHost));
      at += no3[r];
    }
    if (at != n || memcmp(sk.data(), rk.data(), bytes) || memcmp(sp.data(), rp.data(), bytes)) {
      fprintf(stderr, "shard (staged, 3 ranks) differs from the one-GPU sort\n");
      return 1;
    }
    for (int r = 0; r < W; r++) CK(srs_shard_comm_destroy(cs[r]));
  }
  printf("shard ok: n=%lld, every communicator kind equals the one-GPU sort\n", (long long)n);
  return 0;
}

"""Diagnostic: which step of the shard path changes the record multiset?
Compares in-place sort, out-of-place sort and ShardSorter (RCCL, world 1)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "simd-radix-sort_amd", "python"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
import srs_amd  # noqa: E402
from srs_amd.dist import HipShardOps, ShardSorter  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**8
K = srs_amd.KEY_U64
keys = torch.empty(n, dtype=torch.int64, device="cuda")
pay = torch.empty(n, dtype=torch.int64, device="cuda")
srs_amd.fill_synthetic_device(keys, pay, seed=42 << 32, first_index=0, key_kind=K)
h0 = bench._hash_pairs(keys, [pay], torch)
print("input hash", h0, flush=True)
ko, po = torch.empty_like(keys), torch.empty_like(pay)
srs_amd.sort_device(keys, pay, key_kind=K, out=(ko, po))
print("out-of-place", bench._hash_pairs(ko, [po], torch) == h0,
      "input intact", bench._hash_pairs(keys, [pay], torch) == h0, flush=True)
ki, pi = keys.clone(), pay.clone()
srs_amd.sort_device(ki, pi, key_kind=K)
print("in-place", bench._hash_pairs(ki, [pi], torch) == h0, "equal to out-of-place",
      bool(torch.equal(ki, ko) and torch.equal(pi, po)), flush=True)
del ki, pi
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29544", RANK="0", WORLD_SIZE="1")
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
s = ShardSorter(HipShardOps(K), n, [torch.int64], torch.int64, "cuda")
hist = s.ops.histogram(keys, s.bits)
print("hist total", int(hist.sum().item()) == n, flush=True)
rk, (rp,) = s.sort(keys, [pay])
print("shard counts", s.last_counts, flush=True)
print("part copy", bench._hash_pairs(s.part_keys[:n], [s.part_pays[0][:n]], torch) == h0, flush=True)
print("shard", bench._hash_pairs(rk, [rp], torch) == h0, "input intact",
      bench._hash_pairs(keys, [pay], torch) == h0, "equal to out-of-place",
      bool(torch.equal(rk, ko) and torch.equal(rp, po)), flush=True)
dist.destroy_process_group()

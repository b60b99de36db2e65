"""Multi-GPU shard sort: one array spread over N GPUs (one process per GPU,
torch.distributed over RCCL/xGMI), sorted by its top radix bits.

Protocol, per rank r holding n_r keys (+ payload columns):
  1. histogram of the transformed top `bits` key bits   (srs_key_histogram_device)
  2. all-reduce of the 2^bits histogram                  (RCCL, 32 KB at 12 bits)
  3. bucket -> rank map: contiguous bucket ranges with ~equal key counts
  4. stable partition of the local columns by destination rank
                                                         (srs_partition_device)
  5. all-gather of the group sizes, then every column moves peer to peer
     (batched isend/irecv = RCCL's grouped send/recv over xGMI), in rounds
     of at most 256 MB per message: RCCL corrupted a single 8 GB message
     (measured: all_to_all_single of 1e9 int64 at world 1; 1e8 was exact)
  6. local sort of what was received                     (srs_sort_soa_device)
Rank r then holds the r-th contiguous slice of the globally sorted array:
every key on rank r orders before every key on rank r+1.

The device work goes through an `ops` backend (ShardOps) so that the same
protocol code runs on CPU under gloo in the tests (NumpyShardOps in
tests/test_dist.py) and on MI355X under RCCL (HipShardOps, the product path).
The reference (jonicho/simd-radix-sort) has no multi-device path.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def balanced_split(hist: torch.Tensor, world: int) -> torch.Tensor:
    """Bucket -> rank map (int32, non-decreasing) giving each rank a contiguous
    range of buckets holding ~total/world keys: bucket b goes to rank
    floor(world * (keys before b + half of b) / total)."""
    h = hist.to(torch.float64)
    total = float(h.sum().item())
    if total <= 0:
        return torch.zeros(hist.numel(), dtype=torch.int32, device=hist.device)
    before = torch.cumsum(h, 0) - h
    mid = before + 0.5 * h
    part = torch.floor(mid * world / total).clamp_(0, world - 1)
    part = torch.cummax(part, 0).values  # non-decreasing by construction; guard rounding
    return part.to(torch.int32)


_COMM_DT = {1: torch.int8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


def _comm(t):
    """Same bytes as a signed-integer tensor (collectives do not take every
    dtype, e.g. gloo rejects uint64; the exchange moves bits only)."""
    return t.view(_COMM_DT[t.element_size()])


class HipShardOps:
    """Device backend: the HIP kernels of libsrs_amd.so via the C ABI."""

    def __init__(self, kind: int):
        import srs_amd
        self.srs = srs_amd
        self.kind = kind

    def histogram(self, keys, bits):
        h = torch.zeros(1 << bits, dtype=torch.int64, device=keys.device)
        self.srs.key_histogram_device(keys, h, bits, key_kind=self.kind)
        return h

    def partition(self, keys, pays, bits, part_of_bucket, nparts, out):
        return self.srs.partition_device(keys, pays, bits, part_of_bucket, nparts, out,
                                         key_kind=self.kind)

    def sort(self, keys, pays):
        self.srs.sort_device(keys, *pays, key_kind=self.kind)


class ShardSorter:
    """Sorts the union of every rank's (keys, payloads) across the process
    group. Buffers are allocated once (capacity = slack * n per rank)."""

    def __init__(self, ops, n_local: int, payload_dtypes, key_dtype, device, bits: int = 12,
                 slack: float = 1.25, group=None, chunk_bytes: int = 256 << 20):
        self.ops = ops
        self.bits = bits
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device
        self.n = n_local
        cap = int(n_local * slack) + 1024
        self.part_keys = torch.empty(n_local, dtype=key_dtype, device=device)
        self.part_pays = [torch.empty(n_local, dtype=dt, device=device) for dt in payload_dtypes]
        self.recv_keys = torch.empty(cap, dtype=key_dtype, device=device)
        self.recv_pays = [torch.empty(cap, dtype=dt, device=device) for dt in payload_dtypes]
        self.last_counts = None
        self.chunk_bytes = chunk_bytes

    def _ensure_capacity(self, total):
        if total <= self.recv_keys.numel():
            return
        cap = int(total * 1.1) + 1024
        self.recv_keys = torch.empty(cap, dtype=self.recv_keys.dtype, device=self.device)
        self.recv_pays = [torch.empty(cap, dtype=p.dtype, device=self.device)
                          for p in self.recv_pays]

    def _exchange(self, send, recv, in_splits, out_splits, biggest):
        """send: groups by destination rank; recv: groups by source rank.
        The own group is a local copy; the others move in rounds of at most
        `chunk_bytes` per message, every rank running the same rounds."""
        w, me = self.world, self.rank
        soff = [0] * w
        roff = [0] * w
        for i in range(1, w):
            soff[i] = soff[i - 1] + in_splits[i - 1]
            roff[i] = roff[i - 1] + out_splits[i - 1]
        if in_splits[me]:
            recv[roff[me]:roff[me] + in_splits[me]].copy_(send[soff[me]:soff[me] + in_splits[me]])
        if w == 1:
            return
        C = max(1, self.chunk_bytes // send.element_size())
        rounds = (biggest + C - 1) // C
        s_c, r_c = _comm(send), _comm(recv)
        for r in range(rounds):
            a = r * C
            ops = []
            for peer in range(w):
                if peer == me:
                    continue
                ls = min(C, in_splits[peer] - a)
                if ls > 0:
                    ops.append(dist.P2POp(dist.isend, s_c[soff[peer] + a:soff[peer] + a + ls], peer,
                                          group=self.group))
                lr = min(C, out_splits[peer] - a)
                if lr > 0:
                    ops.append(dist.P2POp(dist.irecv, r_c[roff[peer] + a:roff[peer] + a + lr], peer,
                                          group=self.group))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()

    def sort(self, keys, pays):
        """Returns (keys, payloads) views: this rank's slice of the sorted union."""
        w = self.world
        if keys.numel() > self.part_keys.numel():
            self.part_keys = torch.empty(keys.numel(), dtype=keys.dtype, device=self.device)
            self.part_pays = [torch.empty(keys.numel(), dtype=p.dtype, device=self.device)
                              for p in self.part_pays]
        # 1-3: global histogram -> contiguous bucket ranges per rank
        hist = self.ops.histogram(keys, self.bits)
        dist.all_reduce(hist, group=self.group)
        part_of_bucket = balanced_split(hist, w)
        # 4: stable partition by destination rank
        counts = self.ops.partition(keys, pays, self.bits, part_of_bucket, w,
                                    (self.part_keys, *self.part_pays))
        # 5: exchange sizes (full matrix, so every rank agrees on the rounds)
        send = torch.tensor(counts, dtype=torch.int64, device=hist.device)
        mat = [torch.empty_like(send) for _ in range(w)]
        dist.all_gather(mat, send, group=self.group)
        mat = [m.tolist() for m in mat]           # mat[src][dst]
        in_splits = [int(c) for c in counts]
        out_splits = [int(mat[src][self.rank]) for src in range(w)]
        total = sum(out_splits)
        self._ensure_capacity(total)
        biggest = max(max(row) for row in mat)
        rk = self.recv_keys[:total]
        self._exchange(self.part_keys[:keys.numel()], rk, in_splits, out_splits, biggest)
        rps = []
        for src, dstbuf in zip(self.part_pays, self.recv_pays):
            rp = dstbuf[:total]
            self._exchange(src[:keys.numel()], rp, in_splits, out_splits, biggest)
            rps.append(rp)
        # 6: local sort of the received slice
        self.ops.sort(rk, rps)
        self.last_counts = (in_splits, out_splits)
        return rk, rps

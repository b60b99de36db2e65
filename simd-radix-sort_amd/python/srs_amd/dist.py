"""Multi-GPU shard sort: one array spread over N GPUs (one process per GPU,
torch.distributed over RCCL/xGMI), sorted across the GPUs.

Protocol, per rank r holding n_r records (key + payload columns):
  1. histogram of the transformed top `bits` key bits    (srs_key_histogram_device)
  2. all-reduce of the 2^bits histogram                   (RCCL, 32 KB at 12 bits)
  3. bins -> G (<= 512) key-range groups of ~equal size; contiguous runs of
     groups -> ranks, again balanced by size
  4. all-gather of every rank's group sizes per input chunk (exact from
     per-chunk histograms: a group is a union of bins) -> receive layout
  5. stable partition of the local records into the G groups, chunk by
     chunk (srs_partition_device). This IS the first MSB level of the sort:
     nothing is partitioned twice. Each chunk's first-round messages go out
     as soon as it is partitioned, while the next chunk is partitioned.
  6. the groups move peer to peer (batched isend/irecv = RCCL grouped
     send/recv over xGMI) in `rounds`: round i moves a contiguous run of
     each receiver's groups, one message per (round, peer, column), each
     <= 256 MB (RCCL corrupted a single 8 GB all_to_all message: measured at
     world 1, 1e9 int64; 1e8 was exact). A round lands source-major in its
     own key range of the receive buffer (source-major, then chunk: input
     order of equal keys is kept); while round i+1 is in flight,
     round i's range is sorted on a second stream (srs_sort_segments_device)
Rank r then holds the r-th slice of the globally sorted array: every key on
rank r orders before every key on rank r+1.

The device work goes through an `ops` backend so that the same protocol code
runs on CPU under gloo in the tests (NumpyShardOps in tests/test_dist.py) and
on MI355X under RCCL (HipShardOps, the product path). The reference
(jonicho/simd-radix-sort) has no multi-device path.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist


def balanced_split(hist: torch.Tensor, world: int) -> torch.Tensor:
    """Bucket -> part map (int32, non-decreasing) giving each of `world`
    parts a contiguous range of buckets holding ~total/world keys: bucket b
    goes to part floor(world * (keys before b + half of b) / total)."""
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


class PhaseClock:
    """Stamps of one shard sort's phases: HIP events recorded on the stream
    the phase runs on (read once the caller has synchronized), or host wall
    time when the device is the CPU (the gloo tests)."""

    def __init__(self, device):
        self.cuda = torch.device(device).type == "cuda"
        self.marks = []

    def reset(self):
        self.marks = []

    def stamp(self, name, stream=None):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            self.marks.append((name, e))
        else:
            self.marks.append((name, time.perf_counter()))

    def read(self):
        """{name: ms since the first stamp}."""
        if not self.marks:
            return {}
        t0 = self.marks[0][1]
        if self.cuda:
            return {n: round(t0.elapsed_time(e), 4) for n, e in self.marks}
        return {n: round((t - t0) * 1e3, 4) for n, t in self.marks}


class HipShardOps:
    """Device backend: the HIP kernels of libsrs_amd.so via the C ABI."""

    def __init__(self, kind: int):
        import srs_amd
        self.srs = srs_amd
        self.kind = kind
        self.stream = None

    def histogram(self, keys, bits):
        h = torch.zeros(1 << bits, dtype=torch.int64, device=keys.device)
        self.srs.key_histogram_device(keys, h, bits, key_kind=self.kind)
        return h

    def partition(self, keys, pays, bits, part_of_bucket, nparts, out):
        return self.srs.partition_device(keys, pays, bits, part_of_bucket, nparts, out,
                                         key_kind=self.kind)

    def sort(self, keys, pays):
        self.srs.sort_device(keys, *pays, key_kind=self.kind)

    def sort_segments(self, keys, pays, bounds, known_top_bits=0, stamp=None):
        """Queue the sort of the given segments on a side stream, after the
        work already queued on the current stream (the receives). stamp(name,
        stream) marks the start and end of the sort on that stream."""
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=keys.device)
        self.stream.wait_stream(torch.cuda.current_stream(keys.device))
        if stamp:
            stamp("sort_start", self.stream)
        self.srs.sort_segments_device(keys, *pays, bounds=bounds, key_kind=self.kind,
                                      known_top_bits=known_top_bits, stream=self.stream)
        if stamp:
            stamp("sort_end", self.stream)

    def finish(self, device):
        if self.stream is not None:
            torch.cuda.current_stream(device).wait_stream(self.stream)


class ShardSorter:
    """Sorts the union of every rank's (keys, payloads) across the process
    group. Buffers are allocated once (receive capacity = slack * n per rank)
    and grown if a rank receives more."""

    def __init__(self, ops, n_local: int, payload_dtypes, key_dtype, device, bits: int = 12,
                 groups: int = 512, rounds: int = 4, slack: float = 1.25, group=None,
                 chunk_bytes: int = 256 << 20, stage_host: bool = False, chunks: int = 4):
        # stage_host: the messages travel through host memory (test mode:
        # several gloo ranks sharing one GPU run the real kernels; RCCL
        # cannot put two ranks on one device)
        self.stage_host = stage_host
        self.ops = ops
        self.key_bits = 8 * torch.empty(0, dtype=key_dtype).element_size()
        self.bits = min(bits, self.key_bits)
        self.groups = min(groups, 512, 1 << self.bits)
        self.rounds = max(1, rounds)
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device
        self.n = n_local
        self.chunk_bytes = chunk_bytes
        # input chunks partitioned one after another, each one's first-round
        # messages overlapping the next one's partition (one at world 1: no
        # messages, and each group stays one contiguous segment)
        self.chunks = max(1, chunks) if self.world > 1 else 1
        cap = int(n_local * slack) + 1024
        self.part_keys = torch.empty(n_local, dtype=key_dtype, device=device)
        self.part_pays = [torch.empty(n_local, dtype=dt, device=device) for dt in payload_dtypes]
        self.recv_keys = torch.empty(cap, dtype=key_dtype, device=device)
        self.recv_pays = [torch.empty(cap, dtype=dt, device=device) for dt in payload_dtypes]
        self.last_counts = None
        self.rec_bytes = (torch.empty(0, dtype=key_dtype).element_size() +
                          sum(torch.empty(0, dtype=dt).element_size() for dt in payload_dtypes))
        self.clock = PhaseClock(device)
        self.last_bytes = None  # bytes this rank sent to each peer, per round

    def _ensure_capacity(self, total):
        if total <= self.recv_keys.numel():
            return
        cap = int(total * 1.1) + 1024
        self.recv_keys = torch.empty(cap, dtype=self.recv_keys.dtype, device=self.device)
        self.recv_pays = [torch.empty(cap, dtype=p.dtype, device=self.device)
                          for p in self.recv_pays]

    def plan(self, hist):
        """bins -> groups (device int32, for the partition), groups -> ranks
        (host list, non-decreasing) and each group's (first, last) bin."""
        G, w = self.groups, self.world
        group_of_bin = balanced_split(hist, G)
        gtot = torch.zeros(G, dtype=torch.int64, device=hist.device)
        gtot.index_add_(0, group_of_bin.to(torch.int64), hist.to(torch.int64))
        rank_of_group = balanced_split(gtot, w).tolist()
        gb = group_of_bin.tolist()
        first, last = [None] * G, [None] * G
        for b, g in enumerate(gb):
            if first[g] is None:
                first[g] = b
            last[g] = b
        return group_of_bin, rank_of_group, first, last

    def sort(self, keys, pays):
        """Returns (keys, payloads) views: this rank's slice of the sorted union."""
        w, me, G, R = self.world, self.rank, self.groups, self.rounds
        n = keys.numel()
        if n > self.part_keys.numel():
            self.part_keys = torch.empty(n, dtype=keys.dtype, device=self.device)
            self.part_pays = [torch.empty(n, dtype=p.dtype, device=self.device)
                              for p in self.part_pays]
        C = max(1, min(self.chunks, n))
        cb = [n * c // C for c in range(C + 1)]          # chunk c = input [cb[c], cb[c+1])
        clk = self.clock
        clk.reset()
        clk.stamp("start")
        # 1-3: per-chunk histograms -> global histogram -> groups -> ranks
        hists = [self.ops.histogram(keys[cb[c]:cb[c + 1]], self.bits) for c in range(C)]
        hist = hists[0].clone()
        for h in hists[1:]:
            hist += h
        clk.stamp("hist")
        dist.all_reduce(hist, group=self.group)
        group_of_bin, rank_of_group, first, last = self.plan(hist)
        # 4: every rank's group sizes per chunk (a group is a union of bins,
        # so the chunk histograms give them exactly) -> receive layout; known
        # before any partition, so no collective waits behind the messages
        gob = group_of_bin.to(torch.int64)
        cc = torch.zeros(C, G, dtype=torch.int64, device=hist.device)
        for c in range(C):
            cc[c].index_add_(0, gob, hists[c].to(torch.int64))
        allcc = [torch.empty_like(cc) for _ in range(w)]
        dist.all_gather(allcc, cc, group=self.group)
        mat = [m.tolist() for m in allcc]                 # mat[src][chunk][g]
        clk.stamp("plan")  # (after the host read of the all-gather: collectives done)
        counts = [sum(mat[me][c][g] for c in range(C)) for g in range(G)]
        owned = [[g for g in range(G) if rank_of_group[g] == r] for r in range(w)]
        # exchange round r of rank d moves d's groups owned[d][rg[d][r]]: a
        # contiguous run of groups, hence one contiguous piece of every
        # sender's partitioned chunk
        rg = [[range(i * len(owned[d]) // R, (i + 1) * len(owned[d]) // R) for i in range(R)]
              for d in range(w)]
        soff = []                                         # soff[c][g]: group g of chunk c
        for c in range(C):
            o = [cb[c]] * (G + 1)
            for g in range(G):
                o[g + 1] = o[g] + mat[me][c][g]
            soff.append(o)

        def piece(src_counts, d, r):
            """(first group, #records) of the round-r piece for rank d"""
            gs = [owned[d][i] for i in rg[d][r]]
            return (gs[0] if gs else 0), sum(src_counts[g] for g in gs)

        # receive layout: round-major, then source (rank order), then chunk:
        # one message per (round, peer, chunk, column). Equal keys share a
        # group, so inside a round they arrive in (source rank, input index)
        # order, and the round's key range lies above the previous round's.
        roff, rbound, pos = {}, [], 0
        for r in range(R):
            start = pos
            for src in range(w):
                for c in range(C):
                    roff[(r, src, c)] = pos
                    pos += piece(mat[src][c], me, r)[1]
            rbound.append((start, pos))
        total = pos
        # one rank, one chunk: the receive layout (round, then group order)
        # IS the partitioned buffer's layout, so the rounds sort it in place
        # and the exchange copies nothing (world-1 self copies were ~10 ms
        # of the 1e9 C1 shard step)
        alias = w == 1 and C == 1 and not self.stage_host
        if alias:
            rk = self.part_keys[:total]
            rps = [b[:total] for b in self.part_pays]
        else:
            self._ensure_capacity(total)
            rk = self.recv_keys[:total]
            rps = [b[:total] for b in self.recv_pays]
        cols = [(self.part_keys, rk)] + list(zip(self.part_pays, rps))
        mcols = cols                                      # what the messages move
        if self.stage_host:
            # (host buffers, filled chunk by chunk as they are partitioned)
            mcols = [(torch.empty(n, dtype=sb.dtype), torch.empty(total, dtype=rb.dtype))
                     for sb, rb in cols]

        # 6: rounds of peer-to-peer moves for the given chunks; round r+1 is in
        # flight before the (host-synchronising) sort of round r is queued
        def issue(r, chunks):
            p2p = []
            for d in range(w):
                for c in chunks:
                    g0, cnt = piece(mat[me][c], d, r)
                    if d == me:
                        for src in range(w):
                            rcnt = piece(mat[src][c], me, r)[1]
                            if rcnt == 0:
                                continue
                            a = roff[(r, src, c)]
                            for (sbuf, rbuf), (_, mrbuf) in zip(cols, mcols):
                                if src == me:
                                    if not alias:  # (aliased: already in place)
                                        rbuf[a:a + rcnt].copy_(sbuf[soff[c][g0]:soff[c][g0] + rcnt])
                                else:
                                    self._msgs(p2p, dist.irecv, mrbuf, a, rcnt, src)
                    elif cnt:
                        for msbuf, _ in mcols:
                            self._msgs(p2p, dist.isend, msbuf, soff[c][g0], cnt, d)
            return dist.batch_isend_irecv(p2p) if p2p else []

        def land(r):
            """host-staged mode: the round's received pieces to the device"""
            for src in range(w):
                if src == me:
                    continue
                for c in range(C):
                    a, rcnt = roff[(r, src, c)], piece(mat[src][c], me, r)[1]
                    if rcnt:
                        for (_, rbuf), (_, mrbuf) in zip(cols, mcols):
                            rbuf[a:a + rcnt].copy_(mrbuf[a:a + rcnt])

        # 5: partition chunk by chunk; each chunk's round-0 messages go out
        # while the next chunk is partitioned
        pending = []
        bad = False
        for c in range(C):
            a, b = cb[c], cb[c + 1]
            got = self.ops.partition(keys[a:b], [p[a:b] for p in pays], self.bits, group_of_bin,
                                     G, (self.part_keys[a:b], *[p[a:b] for p in self.part_pays]))
            if list(got) != mat[me][c]:
                # earlier chunks' messages are already posted and the peers
                # expect this chunk's: keep to the agreed message plan (the
                # buffers are sized by it) and fail on every rank at the end
                bad = True
            clk.stamp(f"partition{c}")
            if self.stage_host:  # the staged send buffers take the partitioned chunk
                for (sb, _), (msb, _) in zip(cols, mcols):
                    msb[a:b].copy_(sb[a:b])
            pending += issue(0, [c])
        # bytes this rank sends to each peer in each round (the link load)
        self.last_bytes = [[0 if d == me else
                            sum(piece(mat[me][c], d, r)[1] for c in range(C)) * self.rec_bytes
                            for d in range(w)] for r in range(R)]
        for r in range(R):
            for req in pending:
                req.wait()
            clk.stamp(f"round{r}_recv")
            pending = issue(r + 1, range(C)) if r + 1 < R else []
            if self.stage_host:
                land(r)
            a, b = rbound[r]
            gs = [owned[me][i] for i in rg[me][r]]
            if b > a:
                # top key bits shared by every segment's key range
                def shared(grps):
                    bins = [(first[g], last[g]) for g in grps if first[g] is not None]
                    if not bins:
                        return 0
                    lo, hi = bins[0][0], bins[-1][1]
                    return min(self.bits - (lo ^ hi).bit_length(), self.key_bits - 1)
                if w == 1 and C == 1:
                    # one source: the round's groups lie contiguous, each its
                    # own segment (the partition was their first level)
                    bounds = [a]
                    for g in gs:
                        bounds.append(bounds[-1] + counts[g])
                    self.ops.sort_segments(rk, rps, bounds, min(shared([g]) for g in gs),
                                           stamp=lambda nm, st, r=r: clk.stamp(f"round{r}_{nm}", st))
                else:
                    # several sources (or chunks) interleave the groups: the
                    # round's key range is one segment (at w >= 2 its size
                    # needs no more levels than a group's would)
                    self.ops.sort_segments(rk, rps, [a, b], shared(gs),
                                           stamp=lambda nm, st, r=r: clk.stamp(f"round{r}_{nm}", st))
        self.ops.finish(self.device)
        clk.stamp("end")
        # every rank learns whether any partition disagreed with the plan
        flag = torch.tensor([1 if bad else 0], dtype=torch.int64, device=hist.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        if int(flag.item()):
            raise RuntimeError("partition sizes differ from the chunk histogram"
                               + ("" if bad else " (on another rank)"))
        self.last_counts = (counts, [sum(mat[s][c][g] for c in range(C) for g in owned[me])
                                     for s in range(w)])
        return rk, rps

    def phases(self, link_gbs_model=(50.0, 77.0)):
        """The last sort's phase stamps (ms since its start; call after the
        device is synchronized) and the link figures: bytes sent to each peer
        per round, the busiest link's bytes over the exchange window (first
        partition chunk done -> last round received) as the implied GB/s, and
        what the DESIGN.md §7 model predicts for these bytes: the histogram
        and plan, the first partition chunk, then the exchange at the given
        per-link one-way rates, then the last round's sort."""
        ph = self.clock.read()
        out = {"stamps_ms": ph}
        if self.last_bytes is None:
            return out
        R, w = len(self.last_bytes), self.world
        per_peer = [sum(self.last_bytes[r][d] for r in range(R)) for d in range(w)]
        busiest = max(per_peer) if per_peer else 0
        out["bytes_to_peer_per_round"] = self.last_bytes
        out["busiest_link_bytes"] = busiest
        t_ex0 = ph.get("partition0")
        t_ex1 = ph.get(f"round{R - 1}_recv")
        if busiest and t_ex0 is not None and t_ex1 is not None and t_ex1 > t_ex0:
            out["link_gbs"] = round(busiest / ((t_ex1 - t_ex0) * 1e-3) / 1e9, 2)
        last_sort = None
        if f"round{R - 1}_sort_end" in ph and f"round{R - 1}_sort_start" in ph:
            last_sort = ph[f"round{R - 1}_sort_end"] - ph[f"round{R - 1}_sort_start"]
        if t_ex0 is not None:
            model = {}
            for gbs in link_gbs_model:
                ex = busiest / (gbs * 1e9) * 1e3
                model[f"T_ms_at_{int(gbs)}GBs"] = round(t_ex0 + ex + (last_sort or 0.0), 3)
            out["model"] = model
            out["measured_T_ms"] = ph.get("end")
        return out

    def _msgs(self, p2p, op, buf, off, cnt, peer):
        """One message per <= chunk_bytes piece (sender and receiver split a
        group the same way, so the pieces pair up in order)."""
        C = max(1, self.chunk_bytes // buf.element_size())
        v = _comm(buf)
        for a in range(0, cnt, C):
            b = min(cnt, a + C)
            p2p.append(dist.P2POp(op, v[off + a:off + b], peer, group=self.group))

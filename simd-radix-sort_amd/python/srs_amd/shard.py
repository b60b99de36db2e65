"""Multi-GPU shard sort from Python: the srs_shard_* C ABI of libsrs_amd.so
(csrc/srs_shard.hip) through ctypes. There is one
implementation of the protocol, in the library; this module only binds it.

One array spread over N GPUs is sorted across them: rank r ends with the
r-th key range. Per rank (one process per GPU, RCCL over xGMI):

    uid = shard.unique_id() on rank 0, broadcast to every rank
    comm = shard.ShardComm.rccl(world, rank, uid)
    keys_out, pays_out = comm.sort(keys, *payloads, key_kind=...)

or all ranks from one process (threads inside the library):
`shard.staged(world)` (host-staged transport: several ranks on one GPU, the
tests' mode) or `shard.init_all(devices)` (RCCL), then `shard.sort_multi`.

The reference (jonicho/simd-radix-sort) has no multi-device path; its
single-array entry point is radix_sort::sort (radixSort.hpp:1780).
"""
from __future__ import annotations

import ctypes
import json

from . import SrsError, _check, _ptr_array, _size_array, _torch_kind, lib

ID_BYTES = 128
# srs_shard_debug_inject points
INJECT_ARG, INJECT_ALLOC, INJECT_PARTITION, INJECT_ROUND_SORT, INJECT_TRANSPORT = range(1, 6)

_bound = False


def _lib():
    global _bound
    L = lib()
    if not _bound:
        i64, i32, vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
        L.srs_shard_unique_id.argtypes = [vp]
        L.srs_shard_comm_init.argtypes = [i32, i32, vp, ctypes.POINTER(vp)]
        L.srs_shard_comm_init_all.argtypes = [i32, vp, vp]
        L.srs_shard_comm_init_staged.argtypes = [i32, vp]
        L.srs_shard_comm_destroy.argtypes = [vp]
        L.srs_shard_set_options.argtypes = [vp, i32, i32]
        L.srs_shard_set_message_options.argtypes = [vp, i32, i64]
        L.srs_shard_debug_inject.argtypes = [vp, i32]
        L.srs_shard_sort_device.argtypes = [vp, i64, ctypes.c_int, ctypes.c_int, vp, i32, vp, vp,
                                            ctypes.POINTER(vp), vp, ctypes.POINTER(i64), vp]
        L.srs_shard_sort_multi.argtypes = [i32, vp, vp, ctypes.c_int, ctypes.c_int, vp, i32, vp,
                                           vp, vp, vp, vp]
        L.srs_shard_last_report.argtypes = [vp, ctypes.c_char_p, i64]
        L.srs_debug_shard_plan.argtypes = [i32, i32, i32, i32, i32, i32, vp, i64, ctypes.c_char_p,
                                           i64]
        _bound = True
    return L


def unique_id() -> bytes:
    """An RCCL unique id (128 bytes) for srs_shard_comm_init; made on one
    rank and passed to every rank."""
    buf = ctypes.create_string_buffer(ID_BYTES)
    _check(_lib().srs_shard_unique_id(buf))
    return buf.raw


_TYPESTR = None


def _view(ptr, n, dtype, device, owner):
    """A torch tensor over n elements of communicator-owned device memory
    (no copy; keeps `owner` alive)."""
    import torch
    global _TYPESTR
    if _TYPESTR is None:
        _TYPESTR = {torch.int64: "<i8", torch.int32: "<i4", torch.float32: "<f4",
                    torch.float64: "<f8", torch.int16: "<i2", torch.uint8: "|u1",
                    torch.int8: "|i1"}
        for name, ts in (("uint16", "<u2"), ("uint32", "<u4"), ("uint64", "<u8")):
            if hasattr(torch, name):
                _TYPESTR[getattr(torch, name)] = ts

    class _Arr:
        pass
    a = _Arr()
    a.__cuda_array_interface__ = {"shape": (int(n),), "typestr": _TYPESTR[dtype],
                                  "data": (int(ptr or 0), False), "version": 2, "strides": None}
    if n == 0:
        return torch.empty(0, dtype=dtype, device=device)
    t = torch.as_tensor(a, device=device)
    if t.data_ptr() != int(ptr):
        raise SrsError("shard: torch copied the output instead of viewing it")
    t._srs_owner = owner
    return t


class ShardComm:
    """One rank's communicator (srs_shard_comm)."""

    def __init__(self, handle: int, device, world: int, rank: int):
        self.handle = ctypes.c_void_p(handle)
        self.device = device
        self.world = world
        self.rank = rank

    @classmethod
    def rccl(cls, world: int, rank: int, uid: bytes, device=None) -> "ShardComm":
        """srs_shard_comm_init on `device` (default: torch's current GPU)."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else \
            torch.device(device)
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            _check(_lib().srs_shard_comm_init(world, rank, ctypes.c_char_p(uid), ctypes.byref(h)))
        return cls(h.value, dev, world, rank)

    def set_options(self, rounds: int = 0, chunks: int = 0) -> None:
        """Exchange rounds and partition chunks (0 = the library default);
        every rank must pass the same."""
        _check(_lib().srs_shard_set_options(self.handle, int(rounds), int(chunks)))

    def set_message_options(self, self_messages: bool = False, max_message_bytes: int = 0) -> None:
        """Own pieces as messages to this rank instead of device copies, and
        the largest message (0 = 256 MiB); every rank must pass the same cap
        (srs_shard_set_message_options)."""
        _check(_lib().srs_shard_set_message_options(self.handle, int(bool(self_messages)),
                                                    int(max_message_bytes)))

    def inject(self, point: int) -> None:
        """Test hook: the next sort fails at `point` (srs_shard_debug_inject)."""
        _check(_lib().srs_shard_debug_inject(self.handle, int(point)))

    def sort(self, keys, *payloads, key_kind: int | None = None, up: bool = True, stream=None):
        """This rank's part of the shard sort: returns (keys, [payloads]) as
        tensor views of the communicator's output (valid until its next sort).
        Synchronous (the call returns when the sort is complete)."""
        import torch
        kind = _torch_kind(keys) if key_kind is None else int(key_kind)
        np_ = len(payloads)
        kout = ctypes.c_void_p()
        pout = (ctypes.c_void_p * max(1, np_))()
        nout = ctypes.c_int64()
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        with torch.cuda.device(self.device):
            _check(_lib().srs_shard_sort_device(
                self.handle, keys.numel(), kind, int(bool(up)), keys.data_ptr(), np_,
                _ptr_array([p.data_ptr() for p in payloads]),
                _size_array([p.element_size() for p in payloads]), ctypes.byref(kout), pout,
                ctypes.byref(nout), s.cuda_stream))
        n = nout.value
        return (_view(kout.value, n, keys.dtype, self.device, self),
                [_view(pout[k], n, p.dtype, self.device, self) for k, p in enumerate(payloads)])

    def report(self) -> dict:
        """srs_shard_last_report as a dict."""
        buf = ctypes.create_string_buffer(1 << 20)
        _check(_lib().srs_shard_last_report(self.handle, buf, len(buf)))
        return json.loads(buf.value.decode())

    def close(self) -> None:
        if self.handle and self.handle.value:
            _lib().srs_shard_comm_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def staged(world: int, device=None) -> list:
    """`world` communicators on one GPU whose messages travel through host
    memory (srs_shard_comm_init_staged); drive them with sort_multi."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else \
        torch.device(device)
    arr = (ctypes.c_void_p * world)()
    with torch.cuda.device(dev):
        _check(_lib().srs_shard_comm_init_staged(world, arr))
    return [ShardComm(arr[i], dev, world, i) for i in range(world)]


def init_all(devices) -> list:
    """One RCCL communicator per listed GPU, in this process
    (srs_shard_comm_init_all); drive them with sort_multi."""
    import torch
    d = [int(x) for x in devices]
    arr = (ctypes.c_void_p * len(d))()
    devs = (ctypes.c_int32 * len(d))(*d)
    _check(_lib().srs_shard_comm_init_all(len(d), devs, arr))
    return [ShardComm(arr[i], torch.device("cuda", d[i]), len(d), i) for i in range(len(d))]


def sort_multi(comms, inputs, key_kind: int | None = None, up: bool = True):
    """srs_shard_sort_multi: inputs[i] = (keys, [payloads]) of rank i (on
    comms[i]'s GPU). Returns [(keys, [payloads])] per rank (views)."""
    w = len(comms)
    keys0, pays0 = inputs[0]
    kind = _torch_kind(keys0) if key_kind is None else int(key_kind)
    np_ = len(pays0)
    nums = (ctypes.c_int64 * w)(*[k.numel() for k, _ in inputs])
    kin = _ptr_array([k.data_ptr() for k, _ in inputs])
    pin = _ptr_array([p.data_ptr() for _, ps in inputs for p in ps])
    sizes = _size_array([p.element_size() for p in pays0])
    kout = (ctypes.c_void_p * w)()
    pout = (ctypes.c_void_p * max(1, w * np_))()
    nout = (ctypes.c_int64 * w)()
    handles = (ctypes.c_void_p * w)(*[c.handle.value for c in comms])
    _check(_lib().srs_shard_sort_multi(w, handles, nums, kind, int(bool(up)), kin, np_, pin, sizes,
                                       kout, pout, nout))
    out = []
    for i, c in enumerate(comms):
        n = nout[i]
        out.append((_view(kout[i], n, keys0.dtype, c.device, c),
                    [_view(pout[i * np_ + k], n, pays0[k].dtype, c.device, c)
                     for k in range(np_)]))
    return out


def debug_plan(world: int, rank: int, chunks: int, rounds: int, key_bits: int, chunk_hists,
               num: int, self_messages: bool = False) -> dict:
    """srs_debug_shard_plan (host only): the plan rank `rank` follows, from
    every rank's chunk histograms (uint64 numpy array [world][chunks][bins])."""
    import numpy as np
    h = np.ascontiguousarray(chunk_hists, dtype=np.uint64)
    cap = 1 << 26
    buf = ctypes.create_string_buffer(cap)
    _check(_lib().srs_debug_shard_plan(world, rank, chunks, rounds, key_bits,
                                       int(bool(self_messages)), h.ctypes.data, int(num), buf,
                                       cap))
    return json.loads(buf.value.decode())


def link_figures(rep: dict, link_gbs_model=(50.0, 64.0, 77.0)) -> dict:
    """From one rank's report: the busiest link's bytes (the most this rank
    sent one peer), the rate they imply over the exchange window (first
    partition chunk done -> last round received), the non-overlapped head
    (start -> first partition chunk) and tail (the last round's sort), and
    the DESIGN.md §7 model T = head + busiest / rate + tail at the given
    per-link one-way rates."""
    st = rep["stamps_ms"]
    b = rep["bytes_to_peer_per_round"]
    R = len(b)
    w = len(b[0]) if b else 1
    per_peer = [sum(b[r][d] for r in range(R)) for d in range(w)]
    busiest = max(per_peer) if per_peer else 0
    out = {"busiest_link_bytes": busiest}
    t0 = st.get("partition0")
    t1 = st.get(f"round{R - 1}_recv")
    if busiest and t0 is not None and t1 is not None and t1 > t0:
        out["link_gbs"] = round(busiest / ((t1 - t0) * 1e-3) / 1e9, 2)
    s0, s1 = st.get(f"round{R - 1}_sort_start"), st.get(f"round{R - 1}_sort_end")
    tail = (s1 - s0) if s0 is not None and s1 is not None else 0.0
    out["head_ms"] = t0
    out["tail_ms"] = round(tail, 4)
    if t0 is not None:
        out["model"] = {f"T_ms_at_{int(g)}GBs": round(t0 + busiest / (g * 1e9) * 1e3 + tail, 3)
                        for g in link_gbs_model}
        out["measured_T_ms"] = st.get("end")
    return out


def t8_model(head_ms: float, tail_ms: float, t1_ms: float, n: int = 10**9,
             rec_bytes: int = 16, world: int = 8, link_gbs=(50.0, 64.0, 77.0)) -> dict:
    """DESIGN.md §7's weak-scaling model from measured pieces: at `world`
    ranks of n records each, every link carries n * rec_bytes / world bytes
    each way; T(world) = head + those bytes / link rate + tail (the HBM work
    of the rounds hides under the transfers). Also the per-link rate at which
    `world` GPUs reach 6/8 of perfect scaling (6x at 8) against a one-GPU
    step of t1_ms, given this head and tail."""
    link_bytes = n * rec_bytes / world
    out = {f"T{world}_ms_at_{int(g)}GBs": round(head_ms + link_bytes / (g * 1e9) * 1e3 + tail_ms, 3)
           for g in link_gbs}
    budget = t1_ms / 0.75  # world * n / T >= 0.75 * world * n / T1
    room = budget - head_ms - tail_ms
    out["budget_ms_for_6x"] = round(budget, 3)
    out["link_gbs_needed_for_6x"] = round(link_bytes / (room * 1e-3) / 1e9, 1) if room > 0 else None
    out["link_bytes_each_way"] = link_bytes
    return out

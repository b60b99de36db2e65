"""srs_amd — Python mirror of simd_sort::radix_sort over the C ABI of
libsrs_amd.so (include/srs_c_api.h).

Reference interface mirrored (jonicho/simd-radix-sort, radixSort.hpp):
  sort(keys, *payloads, up=True)                     radix_sort::sort<Up>(num, keys, payloads...)   :1780
  sort_thresh(thresh, keys, *payloads, up=True)      sort<Up,BitSorter,CmpSorter>(thresh, num, ...)  :1761
  sort_combined(elements, key_kind, up=True)         sort(thresh, num, DataElement<K,Ps...>*)         :1770

Host numpy arrays are sorted in place (the reference's contract). The
*_device functions take torch tensors already resident in HBM and enqueue on
torch's current stream.

There is no CPU fallback: if the HIP library is missing or the call fails,
an exception is raised.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

try:  # load torch first so one HIP runtime (torch's) serves both libraries
    import torch  # noqa: F401
    _HAVE_TORCH = True
except Exception:  # pragma: no cover - torch is present in this image
    _HAVE_TORCH = False

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB_PATH = os.environ.get("SRS_AMD_LIB") or os.path.join(_PKG_ROOT, "lib", "libsrs_amd.so")

# srs_key_kind (include/srs_c_api.h)
KEY_U8, KEY_I8, KEY_U16, KEY_I16, KEY_U32, KEY_I32, KEY_U64, KEY_I64, KEY_F32, KEY_F64 = range(10)
_NP_KIND = {np.dtype(np.uint8): KEY_U8, np.dtype(np.int8): KEY_I8,
            np.dtype(np.uint16): KEY_U16, np.dtype(np.int16): KEY_I16,
            np.dtype(np.uint32): KEY_U32, np.dtype(np.int32): KEY_I32,
            np.dtype(np.uint64): KEY_U64, np.dtype(np.int64): KEY_I64,
            np.dtype(np.float32): KEY_F32, np.dtype(np.float64): KEY_F64}

SRS_OK = 0
# leaf handling (srs_c_api.h): the reference's CmpSorter (src/cmp_sorters.hpp)
LEAF_SORTED, LEAF_UNSORTED = 0, 1
_LEAF = {"insertion": LEAF_SORTED, "bramas": LEAF_SORTED, "nosort": LEAF_UNSORTED}


class SrsError(RuntimeError):
    pass


_lib = None


def lib() -> ctypes.CDLL:
    """The HIP library; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libsrs_amd.so not built: {LIB_PATH} (run `make -C simd-radix-sort_amd`)")
    L = ctypes.CDLL(LIB_PATH)
    i64, i32, u32, vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32, ctypes.c_void_p
    L.srs_sort_soa.argtypes = [i64, ctypes.c_int, ctypes.c_int, i64, vp, i32, vp, vp]
    L.srs_sort_aos.argtypes = [i64, ctypes.c_int, ctypes.c_int, i64, vp, u32]
    L.srs_sort_soa_leaf.argtypes = [i64, ctypes.c_int, ctypes.c_int, i64, ctypes.c_int, vp, i32,
                                    vp, vp]
    L.srs_sort_aos_leaf.argtypes = [i64, ctypes.c_int, ctypes.c_int, i64, ctypes.c_int, vp, u32]
    L.srs_sort_soa_device_leaf.argtypes = [i64, ctypes.c_int, ctypes.c_int, i64, ctypes.c_int, vp,
                                           i32, vp, vp, vp, vp, vp]
    L.srs_sort_aos_device_leaf.argtypes = [i64, ctypes.c_int, ctypes.c_int, i64, ctypes.c_int, vp,
                                           u32, vp, vp]
    L.srs_sort_soa_device.argtypes = [i64, ctypes.c_int, ctypes.c_int, i64, vp, i32, vp, vp,
                                      vp, vp, vp]
    L.srs_sort_aos_device.argtypes = [i64, ctypes.c_int, ctypes.c_int, i64, vp, u32, vp, vp]
    L.srs_sort_segments_device.argtypes = [i64, ctypes.c_int, ctypes.c_int, vp, i32, vp, vp, i64,
                                           vp, i32, vp]
    L.srs_fill_synthetic_device.argtypes = [i64, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                            vp, i32, vp, vp, vp]
    L.srs_key_histogram_device.argtypes = [i64, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, vp,
                                           vp]
    L.srs_partition_device.argtypes = [i64, ctypes.c_int, ctypes.c_int, vp, i32, vp, vp,
                                       ctypes.c_int, vp, i32, vp, vp, vp, vp]
    L.srs_debug_last_fallbacks.argtypes = [ctypes.POINTER(i64)]
    L.srs_debug_set_super_scan.argtypes = [i64]
    L.srs_debug_last_local_counts.argtypes = [ctypes.POINTER(i64)]
    L.srs_debug_last_local_classes.argtypes = [ctypes.POINTER(i64)]
    L.srs_set_host_devices.argtypes = [i32, vp]
    L.srs_last_error.restype = ctypes.c_char_p
    L.srs_version.restype = ctypes.c_char_p
    L.srs_set_kernel_timing.argtypes = [ctypes.c_int]
    L.srs_kernel_stats.argtypes = [ctypes.c_char_p, ctypes.POINTER(i64),
                                   ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double)]
    L.srs_debug_alloc.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(vp)]
    L.srs_debug_free.argtypes = [vp]
    L.srs_alloc_device.argtypes = [ctypes.c_uint64, ctypes.POINTER(vp)]
    L.srs_free_device.argtypes = [vp]
    L.srs_debug_probe_write.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_float)]
    L.srs_debug_workspace.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_uint64)]
    _lib = L
    return L


def _check(rc: int):
    if rc != SRS_OK:
        raise SrsError(f"srs error {rc}: {lib().srs_last_error().decode()}")


def version() -> str:
    return lib().srs_version().decode()


def key_kind_of(dtype) -> int:
    dt = np.dtype(dtype)
    if dt not in _NP_KIND:
        raise TypeError(f"unsupported key dtype {dt}")
    return _NP_KIND[dt]


def _ptr_array(ptrs):
    return (ctypes.c_void_p * max(1, len(ptrs)))(*ptrs)


def _size_array(sizes):
    return (ctypes.c_uint32 * max(1, len(sizes)))(*sizes)


# --------------------------------------------------------------------------
# host arrays (drop-in semantics: in place, synchronous)
# --------------------------------------------------------------------------
def _leaf(cmp_sorter: str) -> int:
    if cmp_sorter not in _LEAF:
        raise ValueError(f"cmp_sorter must be one of {sorted(_LEAF)}")
    return _LEAF[cmp_sorter]


def sort_thresh(cmp_sort_threshold: int, keys: np.ndarray, *payloads: np.ndarray,
                up: bool = True, cmp_sorter: str = "insertion") -> None:
    """radix_sort::sort<Up, BitSorterSIMD, CmpSorter>(thresh, num, keys,
    payloads...) on host numpy arrays, in place. cmp_sorter: "insertion"
    (CmpSorterInsertionSort), "bramas" (sorted leaves as well) or "nosort"
    (CmpSorterNoSort: leaves of <= thresh keys stay in partition order)."""
    n = len(keys)
    for a in (keys,) + payloads:
        if not (isinstance(a, np.ndarray) and a.flags.c_contiguous and a.ndim == 1):
            raise ValueError("arrays must be 1-D C-contiguous numpy arrays")
        if len(a) != n:
            raise ValueError("all arrays must have the same length")
    _check(lib().srs_sort_soa_leaf(n, key_kind_of(keys.dtype), int(bool(up)),
                                   int(cmp_sort_threshold), _leaf(cmp_sorter), keys.ctypes.data,
                                   len(payloads), _ptr_array([p.ctypes.data for p in payloads]),
                                   _size_array([p.dtype.itemsize for p in payloads])))


def set_host_devices(devices=()) -> None:
    """GPUs the host-array sorts may use (srs_set_host_devices): () = the
    current device; [0, 1, ...] splits large host arrays over them (a device
    may repeat)."""
    d = [int(x) for x in devices]
    arr = (ctypes.c_int32 * max(1, len(d)))(*d)
    _check(lib().srs_set_host_devices(len(d), arr))


def sort(keys: np.ndarray, *payloads: np.ndarray, up: bool = True) -> None:
    """radix_sort::sort<Up>(num, keys, payloads...) (radixSort.hpp:1780): threshold 16."""
    sort_thresh(16, keys, *payloads, up=up)


def sort_combined(elements: np.ndarray, key_kind: int, up: bool = True,
                  cmp_sort_threshold: int = 16, cmp_sorter: str = "insertion") -> None:
    """radix_sort::sort(num, (DataElement<K, Ps...>*) combined): `elements` is a
    C-contiguous array whose rows are records (2-D uint8 (n, elem_size), or a
    structured / plain 1-D array); the key of kind `key_kind` is at byte 0."""
    if not elements.flags.c_contiguous:
        raise ValueError("elements must be C-contiguous")
    n = elements.shape[0]
    esz = elements.nbytes // n if n else elements.dtype.itemsize
    _check(lib().srs_sort_aos_leaf(n, int(key_kind), int(bool(up)), int(cmp_sort_threshold),
                                   _leaf(cmp_sorter), elements.ctypes.data, esz))


# --------------------------------------------------------------------------
# device tensors (torch, already in HBM; asynchronous on the current stream)
# --------------------------------------------------------------------------
_TORCH_KIND = None


def _torch_kind(t) -> int:
    global _TORCH_KIND
    import torch
    if _TORCH_KIND is None:
        _TORCH_KIND = {torch.uint8: KEY_U8, torch.int8: KEY_I8, torch.int16: KEY_I16,
                       torch.int32: KEY_I32, torch.int64: KEY_I64, torch.float32: KEY_F32,
                       torch.float64: KEY_F64}
        for name, k in (("uint16", KEY_U16), ("uint32", KEY_U32), ("uint64", KEY_U64)):
            if hasattr(torch, name):
                _TORCH_KIND[getattr(torch, name)] = k
    if t.dtype not in _TORCH_KIND:
        raise TypeError(f"unsupported key dtype {t.dtype}")
    return _TORCH_KIND[t.dtype]


def _stream_ptr(stream=None, device=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return s.cuda_stream


def _on_device(t):
    """Context that makes t's GPU the current HIP device: the library picks
    its workspace (and torch its current stream) from the current device."""
    import torch
    return torch.cuda.device(t.device)


def _check_columns(keys, cols, what="tensors"):
    """Every column is a 1-D contiguous tensor on keys' GPU with keys' length."""
    for t in cols:
        if not (t.is_cuda and t.is_contiguous() and t.dim() == 1 and t.numel() == keys.numel()):
            raise ValueError(f"{what} must be 1-D contiguous device tensors of equal length")
        if t.device != keys.device:
            raise ValueError(f"{what} must all be on {keys.device} (got {t.device})")


def sort_device(keys, *payloads, up: bool = True, cmp_sort_threshold: int = 16,
                key_kind: int | None = None, out=None, stream=None,
                cmp_sorter: str = "insertion") -> None:
    """Sort device tensors. In place unless `out` = (keys_out, *payloads_out).
    `key_kind` overrides the kind derived from keys.dtype (e.g. torch.int64
    storage holding uint64 keys). Runs on keys' GPU, on `stream` or that
    GPU's current stream."""
    _check_columns(keys, (keys,) + payloads)
    kind = _torch_kind(keys) if key_kind is None else int(key_kind)
    np_ = len(payloads)
    pays = _ptr_array([p.data_ptr() for p in payloads])
    sizes = _size_array([p.element_size() for p in payloads])
    if out is not None:
        if len(out) != 1 + np_:
            raise ValueError("out must hold keys_out followed by every payload_out")
        _check_columns(keys, tuple(out), "out tensors")
        for o, i in zip(out, (keys,) + payloads):
            if o.element_size() != i.element_size():
                raise ValueError("every out tensor must have its input's element size")
        kout = out[0].data_ptr()
        pout = _ptr_array([o.data_ptr() for o in out[1:]])
    else:
        kout, pout = None, None
    with _on_device(keys):
        _check(lib().srs_sort_soa_device_leaf(keys.numel(), kind, int(bool(up)),
                                              int(cmp_sort_threshold), _leaf(cmp_sorter),
                                              keys.data_ptr(), np_, pays, sizes, kout, pout,
                                              _stream_ptr(stream, keys.device)))


def sort_segments_device(keys, *payloads, bounds, up: bool = True, key_kind: int | None = None,
                         known_top_bits: int = 0, stream=None) -> None:
    """Sort every segment [bounds[i], bounds[i+1]) of the device columns
    independently, in place (srs_sort_segments_device). `bounds`: host
    sequence of non-decreasing offsets; `known_top_bits`: top transformed
    key bits every segment's keys are known to share."""
    _check_columns(keys, (keys,) + payloads)
    kind = _torch_kind(keys) if key_kind is None else int(key_kind)
    b = (ctypes.c_int64 * len(bounds))(*[int(x) for x in bounds])
    with _on_device(keys):
        _check(lib().srs_sort_segments_device(
            keys.numel(), kind, int(bool(up)), keys.data_ptr(), len(payloads),
            _ptr_array([p.data_ptr() for p in payloads]),
            _size_array([p.element_size() for p in payloads]),
            max(0, len(bounds) - 1), b, int(known_top_bits), _stream_ptr(stream, keys.device)))


def sort_combined_device(elements, key_kind: int, up: bool = True,
                         cmp_sort_threshold: int = 16, out=None, stream=None,
                         cmp_sorter: str = "insertion") -> None:
    """DataElement array on the device: `elements` is a contiguous (n, elem_size)
    uint8 tensor (or any contiguous tensor whose first dim is the record)."""
    if not (elements.is_cuda and elements.is_contiguous()):
        raise ValueError("elements must be a contiguous device tensor")
    n = elements.shape[0]
    esz = elements.numel() * elements.element_size() // max(1, n)
    if out is not None:
        if not (out.is_cuda and out.is_contiguous() and out.device == elements.device and
                out.numel() * out.element_size() == elements.numel() * elements.element_size()):
            raise ValueError("out must be a contiguous tensor of the same bytes on the same GPU")
    with _on_device(elements):
        _check(lib().srs_sort_aos_device_leaf(n, int(key_kind), int(bool(up)),
                                              int(cmp_sort_threshold), _leaf(cmp_sorter),
                                              elements.data_ptr(), esz,
                                              None if out is None else out.data_ptr(),
                                              _stream_ptr(stream, elements.device)))


def fill_synthetic_device(keys, *payloads, seed: int = 42 << 32, first_index: int = 0,
                          key_kind: int | None = None, stream=None) -> None:
    """keys[i] = splitmix64(seed + first_index + i) (see srs_c_api.h);
    payloads are functions of the key."""
    kind = _torch_kind(keys) if key_kind is None else int(key_kind)
    _check_columns(keys, (keys,) + payloads)
    with _on_device(keys):
        _check(lib().srs_fill_synthetic_device(keys.numel(), kind, seed, first_index,
                                               keys.data_ptr(), len(payloads),
                                               _ptr_array([p.data_ptr() for p in payloads]),
                                               _size_array([p.element_size() for p in payloads]),
                                               _stream_ptr(stream, keys.device)))


# --------------------------------------------------------------------------
# multi-GPU shard primitives (the shard sort itself: srs_amd.shard)
# --------------------------------------------------------------------------
def key_histogram_device(keys, hist, bits: int, up: bool = True, key_kind: int | None = None,
                         stream=None) -> None:
    """Adds the histogram of the transformed top `bits` key bits into `hist`
    (int64 device tensor of 2^bits entries)."""
    kind = _torch_kind(keys) if key_kind is None else int(key_kind)
    if hist.numel() != (1 << bits) or hist.element_size() != 8 or not hist.is_cuda:
        raise ValueError("hist must be a device tensor of 2^bits 64-bit counters")
    _check_columns(keys, (keys,))
    if hist.device != keys.device or not hist.is_contiguous():
        raise ValueError("hist must be contiguous and on the keys' GPU")
    with _on_device(keys):
        _check(lib().srs_key_histogram_device(keys.numel(), kind, int(bool(up)), keys.data_ptr(),
                                              int(bits), hist.data_ptr(),
                                              _stream_ptr(stream, keys.device)))


def partition_device(keys, payloads, bits: int, part_of_bucket, num_parts: int, out,
                     up: bool = True, key_kind: int | None = None, stream=None):
    """Stable partition by destination group (srs_partition_device).
    `part_of_bucket`: int32 device tensor of 2^bits entries. `out` =
    (keys_out, *payloads_out). Returns the host list of group sizes."""
    kind = _torch_kind(keys) if key_kind is None else int(key_kind)
    if part_of_bucket.dtype.itemsize != 4 or part_of_bucket.numel() != (1 << bits):
        raise ValueError("part_of_bucket must hold 2^bits int32 entries")
    pays = list(payloads)
    _check_columns(keys, [keys] + pays)
    if not (part_of_bucket.is_cuda and part_of_bucket.device == keys.device and
            part_of_bucket.is_contiguous()):
        raise ValueError("part_of_bucket must be a contiguous tensor on the keys' GPU")
    if len(out) != 1 + len(pays):
        raise ValueError("out must hold keys_out followed by every payload_out")
    for o, i in zip(out, [keys] + pays):
        if not (o.is_cuda and o.device == keys.device and o.is_contiguous() and o.dim() == 1 and
                o.numel() >= keys.numel() and o.element_size() == i.element_size()):
            raise ValueError("out tensors must be contiguous, on the keys' GPU, at least as long "
                             "as the input and of its element size")
    counts = (ctypes.c_int64 * num_parts)()
    with _on_device(keys):
        _check(lib().srs_partition_device(
            keys.numel(), kind, int(bool(up)), keys.data_ptr(), len(pays),
            _ptr_array([p.data_ptr() for p in pays]), _size_array([p.element_size() for p in pays]),
            int(bits), part_of_bucket.data_ptr(), int(num_parts), out[0].data_ptr(),
            _ptr_array([o.data_ptr() for o in out[1:]]), counts,
            _stream_ptr(stream, keys.device)))
    return [int(c) for c in counts]


# --------------------------------------------------------------------------
# kernel timing (HIP events around every launch, see srs_c_api.h)
# --------------------------------------------------------------------------
def set_kernel_timing(enable) -> None:
    """True / 1: HIP events around every launch; 2: around the scatter
    launches only (the timed region's roofline kernel); False / 0: off."""
    _check(lib().srs_set_kernel_timing(2 if enable == 2 else int(bool(enable))))


def reset_kernel_stats() -> None:
    _check(lib().srs_reset_kernel_stats())


def kernel_stats(name: str):
    """(launches, total_ms, elements) for a kernel family since the last reset."""
    n = ctypes.c_int64()
    ms = ctypes.c_double()
    el = ctypes.c_double()
    _check(lib().srs_kernel_stats(name.encode(), ctypes.byref(n), ctypes.byref(ms),
                                  ctypes.byref(el)))
    return n.value, ms.value, el.value


def last_fallbacks():
    """(stable, lsd): local segments the last sort on the current device
    handed to the stable / LSD fallback kernels (synchronizes the device)."""
    c = (ctypes.c_int64 * 2)()
    _check(lib().srs_debug_last_fallbacks(c))
    return int(c[0]), int(c[1])


def last_local_counts():
    """(local segments, of which handed from the direct to the fast kernel)
    of the last sort on the current device (synchronizes the device)."""
    c = (ctypes.c_int64 * 2)()
    _check(lib().srs_debug_last_local_counts(c))
    return int(c[0]), int(c[1])


def last_local_classes():
    """(small-class segments, large-class segments, of each the ones the
    direct kernel handed to the fast kernel) of the last sort on the current
    device (synchronizes the device)."""
    c = (ctypes.c_int64 * 4)()
    _check(lib().srs_debug_last_local_classes(c))
    return tuple(int(x) for x in c)


class _DeviceBlock:
    """srs_alloc_device memory exposed through __cuda_array_interface__; freed
    when the last tensor viewing it goes away."""

    def __init__(self, n, dtype, device):
        import torch
        self.device = torch.device(device)
        self.dtype = dtype
        self.n = int(n)
        nbytes = self.n * torch.empty(0, dtype=dtype).element_size()
        p = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _check(lib().srs_alloc_device(nbytes, ctypes.byref(p)))
        self.ptr = int(p.value or 0)
        typestr = {torch.int64: "<i8", torch.int32: "<i4", torch.float32: "<f4",
                   torch.float64: "<f8", torch.int16: "<i2", torch.uint8: "|u1",
                   torch.int8: "|i1"}[dtype]
        self.__cuda_array_interface__ = {"shape": (self.n,), "typestr": typestr,
                                         "data": (self.ptr, False), "version": 2,
                                         "strides": None}

    def __del__(self):
        if getattr(self, "ptr", 0):
            try:
                lib().srs_free_device(ctypes.c_void_p(self.ptr))
            except Exception:
                pass
            self.ptr = 0


def empty_device(n: int, dtype, device="cuda"):
    """A 1-D torch tensor of n elements in memory from srs_alloc_device
    (probed placement): for arrays the sort writes."""
    import torch
    blk = _DeviceBlock(n, dtype, device)
    t = torch.as_tensor(blk, device=blk.device)
    if t.data_ptr() != blk.ptr:
        raise SrsError("empty_device: torch copied the block instead of viewing it")
    t._srs_block = blk  # (keeps the memory alive as long as the tensor)
    return t


def debug_alloc(nbytes: int, mode: int = 0) -> int:
    """Raw device allocation on the current device (srs_debug_alloc; mode 0
    hipMalloc, 1 contiguous, 2 VMM at 1 GiB alignment): the address."""
    p = ctypes.c_void_p()
    _check(lib().srs_debug_alloc(int(nbytes), int(mode), ctypes.byref(p)))
    return int(p.value)


def debug_free(ptr: int) -> None:
    _check(lib().srs_debug_free(ctypes.c_void_p(ptr)))


def debug_set_super_scan(min_groups: int) -> None:
    """Scan groups from which a one-segment level takes the super-group
    column scan (srs_debug_set_super_scan; 0 = the default, 256)."""
    _check(lib().srs_debug_set_super_scan(int(min_groups)))


def debug_probe_write(ptr: int, nbytes: int) -> float:
    """ms of one pass of the scatter's write pattern over device memory."""
    ms = ctypes.c_float()
    _check(lib().srs_debug_probe_write(ctypes.c_void_p(ptr), int(nbytes), ctypes.byref(ms)))
    return float(ms.value)


def debug_workspace():
    """(tmp address, bytes, tmp2 address, bytes) of the current device."""
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    na, nb = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().srs_debug_workspace(ctypes.byref(a), ctypes.byref(na), ctypes.byref(b),
                                     ctypes.byref(nb)))
    return int(a.value or 0), int(na.value), int(b.value or 0), int(nb.value)


def release_workspace() -> None:
    _check(lib().srs_release_workspace())

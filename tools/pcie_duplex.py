"""PCIe duplex probe: H2D alone, D2H alone, and both at once (two streams,
two host threads), for pageable and pinned host memory. Decides whether the
host-pointer drop-in can overlap a column's D2H with the next column's H2D.
usage: python tools/pcie_duplex.py [GB per direction]"""
import ctypes
import sys
import threading
import time

import numpy as np
import torch

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
nbytes = int(gb * (1 << 30))
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_void_p]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
H2D, D2H = 1, 2

torch.cuda.init()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
dev_a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
dev_b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
host = {
    "pageable": (np.ones(nbytes, dtype=np.uint8), np.ones(nbytes, dtype=np.uint8)),
    "pinned": (torch.ones(nbytes, dtype=torch.uint8).pin_memory(),
               torch.ones(nbytes, dtype=torch.uint8).pin_memory()),
}


def ptr(x):
    return x.ctypes.data if isinstance(x, np.ndarray) else x.data_ptr()


def copy(kind, dst, src, stream):
    rc = hip.hipMemcpyAsync(ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, kind,
                            ctypes.c_void_p(stream.cuda_stream))
    assert rc == 0, rc
    hip.hipStreamSynchronize(ctypes.c_void_p(stream.cuda_stream))


for mem, (ha, hb) in host.items():
    jobs = {"H2D": lambda: copy(H2D, dev_a.data_ptr(), ptr(ha), s1),
            "D2H": lambda: copy(D2H, ptr(hb), dev_b.data_ptr(), s2)}
    for j in jobs.values():
        j()  # warm (first touch, staging buffers)
    for name, j in jobs.items():
        t0 = time.perf_counter()
        j()
        dt = time.perf_counter() - t0
        print(f"{mem:8s} {name} alone      {nbytes / dt / 1e9:6.1f} GB/s", flush=True)
    ths = [threading.Thread(target=j) for j in jobs.values()]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    print(f"{mem:8s} H2D+D2H together {2 * nbytes / dt / 1e9:6.1f} GB/s aggregate "
          f"({dt * 1e3:.0f} ms for {gb:g} GB each way)", flush=True)

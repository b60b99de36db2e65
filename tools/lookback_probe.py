"""Cost of a decoupled look-back in the scatter (diagnostic build
-DSRS_DIAG_LOOKBACK, tools/build_variants.sh lb:"-DSRS_DIAG_LOOKBACK").
Sorts the C1 workload with the look-back on and off (same library),
interleaved, and prints the scatter's launch time plus the check counters
(mismatches against the count pass's offsets, spin timeouts, hops).
usage: SRS_AMD_LIB=.../lb/libsrs_amd.so python tools/lookback_probe.py [n]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "simd-radix-sort_amd", "python"))
import torch  # noqa: E402

import srs_amd  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**9
keys = torch.empty(n, dtype=torch.int64, device="cuda")
pays = torch.empty(n, dtype=torch.int64, device="cuda")
srs_amd.fill_synthetic_device(keys, pays, key_kind=srs_amd.KEY_U64)
ko, po = torch.empty_like(keys), torch.empty_like(pays)
ntiles = n // 4096 + 600 * 512 + 1024
status = torch.zeros(ntiles * 512, dtype=torch.int32, device="cuda")
err = torch.zeros(4, dtype=torch.int64, device="cuda")
L = srs_amd.lib()
L.srs_debug_set_lookback.argtypes = [ctypes.c_void_p, ctypes.c_void_p]


def run(on, reps=3):
    L.srs_debug_set_lookback(status.data_ptr() if on else None, err.data_ptr() if on else None)
    srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=(ko, po))  # warm
    torch.cuda.synchronize()
    err.zero_()
    srs_amd.reset_kernel_stats()
    srs_amd.set_kernel_timing(True)
    for _ in range(reps):
        srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=(ko, po))
    torch.cuda.synchronize()
    srs_amd.set_kernel_timing(False)
    l, ms, _ = srs_amd.kernel_stats("scatter")
    lc, msc, _ = srs_amd.kernel_stats("count")
    e = err.tolist()
    print(f"lookback {'on ' if on else 'off'}: scatter {ms / l:.3f} ms/launch ({l} launches), "
          f"count {msc / lc:.3f}; mismatches {e[0]}, timeouts {e[1]}, "
          f"hops/launch(digit 0) {e[2] / max(l, 1):.0f}", flush=True)
    ok = bool((ko[1:] ^ (-2**63) >= ko[:-1] ^ (-2**63)).all().item())
    print("   sorted", ok, flush=True)


for i in range(2):
    run(False)
    run(True)

"""Per-phase cycle split of the scatter and local kernels (stamp build).

usage: SRS_AMD_LIB=.../variants/stamps/libsrs_amd.so python tools/stamps.py [n]"""
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
acc = torch.zeros(64, dtype=torch.int64, device="cuda")
L = srs_amd.lib()
L.srs_debug_set_stamp_buffer.argtypes = [ctypes.c_void_p]
srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=(ko, po))  # warm-up
torch.cuda.synchronize()
L.srs_debug_set_stamp_buffer(acc.data_ptr())
srs_amd.set_kernel_timing(True)
srs_amd.reset_kernel_stats()
srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=(ko, po))
torch.cuda.synchronize()
L.srs_debug_set_stamp_buffer(None)
a = acc.cpu().tolist()
names = {0: ["loads", "rank", "tile scan", "stage col0", "store col0+col1 (drained)"],
         1: ["keys loaded", "bucket hist+scan", "bucket scatter", "rank", "col0 moved",
             "col1 moved"]}
for kid, kname in ((0, "scatter"), (1, "local")):
    wg = a[kid * 16]
    launches, ms, el = srs_amd.kernel_stats(kname)
    tot = sum(a[kid * 16 + 1: kid * 16 + 16])
    print(f"{kname}: {wg} workgroups, {launches} launches, {ms:.2f} ms total")
    for i, nm in enumerate(names[kid]):
        c = a[kid * 16 + 1 + i]
        print(f"   {nm:28s} {c / max(wg, 1):10.0f} cyc/WG  {100 * c / max(tot, 1):5.1f}%")

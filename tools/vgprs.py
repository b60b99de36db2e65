"""Print VGPRs / scratch / occupancy per kernel from the build's remarks.
usage: python tools/vgprs.py [substring] [remarks file]"""
import re
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else ""
txt = open(sys.argv[2] if len(sys.argv) > 2 else "simd-radix-sort_amd/build/srs_kernels.remarks").read()
cur, row = None, {}
for line in txt.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        if cur and pat in cur:
            print(f"{cur[:70]:70s} {row}")
        cur, row = m.group(1), {}
        continue
    for k in ("VGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"):
        m = re.search(re.escape(k) + r": (\d+)", line)
        if m:
            row[k.split()[0]] = int(m.group(1))
if cur and pat in cur:
    print(f"{cur[:70]:70s} {row}")

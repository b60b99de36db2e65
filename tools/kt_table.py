"""Per-dispatch kernel durations from tools/kt_variants.sh output: for each
variant, the mean duration (ms) of each kernel name at each position inside a
step (e.g. the level-1 and level-2 scatter separately).
usage: python tools/kt_table.py gpurun_out/kt [kernel-substring ...]"""
import csv, glob, os, sys
from collections import defaultdict

root = sys.argv[1]
pats = sys.argv[2:] or ["scatter_kernel", "count_kernel", "local_kernel"]
for vdir in sorted(glob.glob(os.path.join(root, "*"))):
    if not os.path.isdir(vdir):
        continue
    files = glob.glob(os.path.join(vdir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        continue
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    for p in pats:
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
              for r in rows if p in r["Kernel_Name"]]
        print(f"{os.path.basename(vdir):10s} {p:16s} n={len(ds):3d} " +
              " ".join(f"{d:.3f}" for d in ds))

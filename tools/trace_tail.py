"""Per-launch kernel timeline of the last step in a rocprofv3 kernel trace.
usage: python tools/trace_tail.py <trace dir> <marker kernel substring> [min_ms]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
marker = sys.argv[2]
min_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 0.03
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
out = [(int(r["Start_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")
        .replace("srs::", "")[:60], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
       for r in rows]
idx = [i for i, o in enumerate(out) if marker in o[1]]
base = out[idx[-1]][0]
for s, n, d in out[idx[-1]:]:
    if d >= min_ms:
        print(f"{(s - base) / 1e6:9.3f} {d:8.3f} {n}")
print("end", (out[-1][0] - base) / 1e6)

"""Print the bench JSON lines of gpurun_out logs compactly.
usage: python tools/show.py gpurun_out/bench_*.log"""
import json
import sys

KEEP = ("count", "scatter", "local", "local_fast", "local_stable", "scan")
for path in sys.argv[1:]:
    path = "/dev/stdin" if path == "-" else path
    line = None
    try:
        with open(path) as f:
            for ln in f:
                if ln.startswith('{"metric"'):
                    line = json.loads(ln)
    except OSError as e:
        print(path, "missing:", e)
        continue
    if line is None:
        print(path, "no bench line")
        continue
    k = {n: (v["launches"], v["avg_ms"], v["total_ms_per_step"])
         for n, v in line.get("kernels", {}).items() if n in KEEP}
    print(f"{path}: {line['value']} {line['unit']} {line['ms_per_step']} ms "
          f"verified={line.get('verified')} kernels={k}")

"""Turn a tools/profile_round.sh output directory into committed profiles.

usage: python tools/profile_summary.py <tag> [gpurun_out/prof/<tag>]

Writes
  profiles/<tag>_kernel_stats.csv  rocprofv3 --kernel-trace --stats summary
                                   of the bench command (names shortened)
  profiles/<tag>_pmc.json          per-kernel HBM bytes per dispatch from the
                                   FETCH_SIZE / WRITE_SIZE passes, plus the
                                   bench line of the traced run
  profiles/<tag>_summary.md        the same, readable

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the
bytes of a coalesced streaming read, so read bytes = 2 x FETCH_SIZE x 1024.
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.strip('"')
    name = name.split("(")[0].replace("void ", "").replace("srs::", "")
    return name


def base_kernel(name):
    """scatter_kernel<...> -> scatter (the names bench.py reports)."""
    n = short(name).split("<")[0]
    return {"scatter_kernel": "scatter", "scatter_pair_kernel": "scatter",
            "count_kernel": "count", "local_kernel": "local_fast",
            "local_stable_kernel": "local_stable", "local_lsd_kernel": "local_lsd"}.get(n, n)


def pmc(path, counter):
    acc, cnt = defaultdict(float), defaultdict(int)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            k = short(row["Kernel_Name"])
            acc[k] += float(row["Counter_Value"])
            cnt[k] += 1
    return {k: (acc[k] / cnt[k], cnt[k]) for k in acc}


def bench_line(log):
    with open(log) as f:
        for line in f:
            if line.startswith('{"metric"'):
                return json.loads(line)
    return None


def main(tag, src):
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    out = os.path.join(ROOT, "profiles", tag)
    # 1. kernel stats
    rows = []
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            rows.append(row)
    with open(out + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for r in rows:
            w.writerow([short(r["Name"]), r["Calls"], r["TotalDurationNs"], r["AverageNs"],
                        r["Percentage"], r["MinNs"], r["MaxNs"]])
    # 2. PMC bytes
    fetch = pmc(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    line = bench_line(os.path.join(src, "bench_trace.log"))
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if k.startswith("at::") or k.startswith("__amd"):
            continue
        fk = fetch.get(k, (0.0, 0))[0] * 1024
        wk = write.get(k, (0.0, 0))[0] * 1024
        kernels[k] = {"name": base_kernel(k), "dispatches": fetch.get(k, (0, 0))[1],
                      "fetch_size_bytes_raw": fk, "read_bytes": 2 * fk, "write_bytes": wk,
                      "hbm_bytes": 2 * fk + wk}
    stats = {short(r["Name"]): {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
             for r in rows}
    doc = {"tag": tag, "command": " ".join(["python bench.py"] + sys.argv[3:]),
           "workload": (line or {}).get("config", {}).get("workload"),
           "keys_per_gpu": (line or {}).get("config", {}).get("keys_per_gpu"),
           "correction": "read_bytes = 2 x FETCH_SIZE(KiB) x 1024 (gfx950, MI355X_MICROARCH.md HBM)",
           "kernels": kernels, "kernel_stats": stats, "bench_line": line}
    with open(out + "_pmc.json", "w") as f:
        json.dump(doc, f, indent=1)
    # 3. readable summary
    L = [f"# Profile {tag}", "", f"Command: `{doc['command']}` (under rocprofv3 on one MI355X)", "",
         f"Workload: {doc['workload']}", ""]
    if line:
        L += [f"Bench line of the traced run: **{line['value']} {line['unit']}**, "
              f"{line['ms_per_step']} ms/step; dominant kernel `{line['roofline']['kernel']}` "
              f"avg {line['roofline']['avg_launch_ms']} ms (HIP events).", ""]
    L += ["## Kernel time (rocprofv3 --kernel-trace --stats)", "",
          "| kernel | calls | avg ms | % |", "|---|---:|---:|---:|"]
    torch_ms = 0.0
    for r in rows:
        if short(r["Name"]).startswith("at::"):
            torch_ms += float(r["TotalDurationNs"]) / 1e6
            continue
        if float(r["Percentage"]) < 0.01:
            continue
        L.append(f"| `{short(r['Name'])[:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} "
                 f"| {float(r['Percentage']):.1f} |")
    L += ["", f"(torch kernels, {torch_ms:.1f} ms in total, are bench.py's full-size "
          "verification after the timed region and are left out above; the CSV has every row.)"]
    L += ["", "## HBM bytes per dispatch (FETCH_SIZE x2, WRITE_SIZE)", "",
          "| kernel | read GB | write GB | total GB |", "|---|---:|---:|---:|"]
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes"])[:8]:
        L.append(f"| `{k[:90]}` | {v['read_bytes'] / 1e9:.3f} | {v['write_bytes'] / 1e9:.3f} "
                 f"| {v['hbm_bytes'] / 1e9:.3f} |")
    with open(out + "_summary.md", "w") as f:
        f.write("\n".join(L) + "\n")
    print("wrote", out + "_{kernel_stats.csv,pmc.json,summary.md}")


if __name__ == "__main__":
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof", tag)
    main(tag, src)

"""Per-step view of a rocprofv3 kernel trace (SQLite output) of
`bench.py --shard`: each step's span, its GPU idle gaps, kernel time per
kernel, and (--timeline) every launch of one step.
usage: python tools/trace_steps.py <results.db> [--step K] [--timeline]"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(n):
    return re.sub(r"\(.*", "", n).replace("void ", "").replace("srs::", "").replace(
        "unsigned long", "u64")[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--step", type=int, default=2)
    ap.add_argument("--timeline", action="store_true")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, stream_id, grid_x, workgroup_x from kernels "
                          "order by start"))
    hist = [i for i, r in enumerate(rows) if "key_hist" in r[0]]
    # a step starts with its chunk histograms (one launch per chunk, back to back)
    starts = [i for k, i in enumerate(hist) if k == 0 or i != hist[k - 1] + 1]
    for si, i0 in enumerate(starts):
        i1 = starts[si + 1] if si + 1 < len(starts) else len(rows)
        seg, t0 = rows[i0:i1], rows[i0][1]
        cur, gaps, end = t0, [], len(seg)
        for j, r in enumerate(seg):
            if r[1] - cur > 5e6:  # (> 5 ms idle: the step is over)
                end = j
                break
            if r[1] > cur:
                gaps.append((r[1] - cur) / 1e3)
            cur = max(cur, r[2])
        seg = seg[:end]
        kt = defaultdict(float)
        for r in seg:
            kt[short(r[0])] += (r[2] - r[1]) / 1e6
        print(f"step {si}: span {(cur - t0) / 1e6:.2f} ms, {len(seg)} launches, GPU idle "
              f"{sum(gaps) / 1e3:.2f} ms in {len(gaps)} gaps")
        if si == a.step:
            for k, v in sorted(kt.items(), key=lambda x: -x[1]):
                print(f"    {v:8.3f} ms  {k}")
            if a.timeline:
                for r in seg:
                    print(f"  {(r[1] - t0) / 1e6:7.3f} {(r[2] - r[1]) / 1e3:8.1f} us s{r[3]} "
                          f"wg {r[4] // max(r[5], 1):>7} {short(r[0])}")


if __name__ == "__main__":
    main()

"""Summarise rocprofv3 --pmc CSV output per kernel (mean per dispatch).

usage: python tools/pmc_summary.py <run_counter_collection.csv> [...]"""
import csv
import sys
from collections import defaultdict


def short(name):
    name = name.strip('"')
    return name.split("(")[0].replace("void ", "").replace("srs::", "")


def main(paths):
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                cnt[k][row["Counter_Name"]] += 1
    for k in sorted(acc):
        vals = {c: acc[k][c] / cnt[k][c] for c in acc[k]}
        print(k, {c: f"{v:.4g}" for c, v in sorted(vals.items())})


if __name__ == "__main__":
    main(sys.argv[1:])

"""Offline model of the sort's levels on C2's keys (BASELINE configs[2]:
1e9 float32 in [-1, 1), the bench generator: i / 2^23 - 1 for a uniform
24-bit i, so every one of the 2^24 values holds ~n / 2^24 keys).

Runs the real host planner (srs_debug_plan_table on the sort's own sample),
then replays the levels the way the kernels choose digits (make_plan: a
segment's digit is the top choose_bits(len, rbits) bits below its rbits;
the children's rbits come from the varying-bit OR) on the exact value
counts, and prints how many keys each level leaves above the LDS capacity.
No GPU.  usage: python tools/c2_levels.py [n]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "simd-radix-sort_amd", "python"))
from test_table_plan import _c2_sample, _plan, _digit  # noqa: E402

LOCAL_CAP = 8192
LOCAL_TARGET, LOCAL_CAP_TARGET, LOCAL_SMALL_TARGET, MAX_BITS = 6144, 7808, 3840, 9


def levels_for(n, target):
    need = 1
    while need < 62 and (target << need) < n:
        need += 1
    return (need + MAX_BITS - 1) // MAX_BITS, need


def choose_bits(n, rbits):
    levels, need = levels_for(n, LOCAL_TARGET)
    lc, nc = levels_for(n, LOCAL_CAP_TARGET)
    if lc < levels:
        levels, need = lc, nc
    ls, ns = levels_for(n, LOCAL_SMALL_TARGET)
    if ls == levels:
        need = ns
    bits = min(MAX_BITS, (need + levels - 1) // levels, rbits)
    return max(bits, 1)


def simulate(n=10 ** 9, verbose=True):
    """Keys left above the LDS capacity after each level: [(segments, keys)]."""
    out = []
    log = print if verbose else (lambda *a, **k: None)
    i = np.arange(1 << 24, dtype=np.int32)
    k = i.astype(np.float32) * np.float32(1.0 / 8388608.0) - np.float32(1.0)
    b = k.view(np.uint32)
    u = np.where(b >> np.uint32(31), ~b, b ^ np.uint32(1 << 31)).astype(np.uint32)
    order = np.argsort(u, kind="stable")
    u = u[order]
    cnt = np.full(u.size, n / float(1 << 24))
    hist = np.bincount(_c2_sample(n) >> np.uint32(16), minlength=65536)
    mode, groups, over, other, table, rbits = _plan(hist, n, 32)
    log(f"table mode {mode}, {groups} groups, predicted overflow {over:.0f} (other {other:.0f})")
    g = _digit(mode, table, u, 32).astype(np.int64)
    # segments: (values slice, rbits); level 1 = the table's groups
    segs = []
    for gg in np.unique(g):
        lo, hi = np.searchsorted(g, gg), np.searchsorted(g, gg, side="right")
        segs.append((lo, hi, int(rbits[gg])))
    level = 1
    while segs:
        big, keys_big, local = [], 0.0, 0
        for lo, hi, rb in segs:
            ln = cnt[lo:hi].sum()
            if level > 1:
                if ln <= LOCAL_CAP:
                    local += 1
                    continue
                bits = choose_bits(int(ln), rb)
                sh = rb - bits
                d = (u[lo:hi] >> np.uint32(sh)) & np.uint32((1 << bits) - 1)
                cuts = np.flatnonzero(np.diff(d)) + 1
                parts = np.split(np.arange(lo, hi), cuts)
                for p in parts:
                    a, z = p[0], p[-1] + 1
                    var = np.bitwise_or.reduce(u[a:z] ^ u[a]) if z - a > 1 else 0
                    nrb = int(var).bit_length()
                    big.append((a, z, min(nrb, sh)))
            else:
                big.append((lo, hi, rb))
        nxt = [(a, z, r) for a, z, r in big if cnt[a:z].sum() > LOCAL_CAP]
        keys_big = sum(cnt[a:z].sum() for a, z, _ in nxt)
        sizes = sorted((cnt[a:z].sum() for a, z, _ in nxt), reverse=True)[:8]
        out.append((len(nxt), keys_big))
        log(f"after level {level}: {len(nxt)} segments above {LOCAL_CAP} keys, "
              f"{keys_big:.0f} keys; largest {[int(s) for s in sizes]}")
        if level >= 1 and nxt:
            worst = max(nxt, key=lambda s: cnt[s[0]:s[1]].sum())
            log(f"   largest: values {u[worst[0]]:#010x}..{u[worst[1] - 1]:#010x} rbits {worst[2]}"
                  f" group {g[worst[0]]} (group rbits {rbits[g[worst[0]]]})")
        segs = nxt
        level += 1
        if level > 6:
            break
    return out


if __name__ == "__main__":
    simulate(int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9)

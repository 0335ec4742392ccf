"""Device timeline of a rocprofv3 --kernel-trace run (TEST / ANALYSIS TOOL): over the
last `--window` seconds of kernel activity, the union of all kernels' busy intervals
(device busy fraction), the time covered by the dominant kernel's launches, and per
kernel the time it runs while NO dominant-kernel launch is active (its exposed time).

    python tools/timeline.py gpurun_out/TAG/prof/run_results.db [--kernel kp_attn3] [--window 0.4]
"""
import argparse
import sqlite3
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    out = []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                out.append((cur_s, cur_e))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        out.append((cur_s, cur_e))
    return out


def covered(a, b):
    """Length of (intervals a) minus (union b), a and b sorted disjoint lists."""
    tot, j = 0, 0
    for s, e in a:
        x = s
        while j < len(b) and b[j][1] <= x:
            j += 1
        k = j
        while x < e:
            if k < len(b) and b[k][0] < e:
                if b[k][0] > x:
                    tot += b[k][0] - x
                x = max(x, b[k][1])
                k += 1
            else:
                tot += e - x
                x = e
    return tot


def short_name(n):
    n = n.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--kernel", default="kp_attn3<25, 0>")
    ap.add_argument("--window", type=float, default=0.4, help="seconds at the end of the trace")
    ap.add_argument("--skip-end", type=float, default=0.0, help="seconds cut off the end (the pipeline's drain)")
    ap.add_argument("--gaps", action="store_true", help="list the idle gaps over 1 ms with the kernels around them")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels").fetchall()
    t1 = max(e for _, _, e in rows) - a.skip_end * 1e9
    t0 = t1 - a.window * 1e9
    rows = [(n, max(s, t0), min(e, t1)) for n, s, e in rows if e > t0 and s < t1]
    busy = union([(s, e) for _, s, e in rows])
    hot = union([(s, e) for n, s, e in rows if a.kernel in n])
    span = t1 - t0
    print(f"window {span / 1e6:.1f} ms: busy {sum(e - s for s, e in busy) / span:.3f}, "
          f"{a.kernel} active {sum(e - s for s, e in hot) / span:.3f}")
    # idle gaps between busy intervals, by length
    gaps = [b[0] - a_[1] for a_, b in zip(busy, busy[1:])]
    for lo, hi in ((0, 1e4), (1e4, 1e5), (1e5, 1e6), (1e6, 1e12)):
        g = [x for x in gaps if lo <= x < hi]
        print(f"  idle gaps {lo / 1e3:g}-{hi / 1e3:g} us: {len(g)} gaps, {sum(g) / span:.3f} of the window")
    if a.gaps:
        for a_, b in zip(busy, busy[1:]):
            if b[0] - a_[1] >= 1e6:
                before = [n for n, s, e in rows if abs(e - a_[1]) < 1e3]
                after = [n for n, s, e in rows if abs(s - b[0]) < 1e3]
                print(f"  gap {(b[0] - a_[1]) / 1e3:8.1f} us at {(a_[1] - t0) / 1e6:7.2f} ms: after "
                      f"{[short_name(n)[:40] for n in before]} before {[short_name(n)[:40] for n in after]}")
    per = defaultdict(list)
    for n, s, e in rows:
        per[short_name(n)].append((s, e))
    out = []
    for n, iv in per.items():
        u = union(iv)
        out.append((covered(u, hot) / span, sum(e - s for s, e in u) / span, len(iv), n))
    for exp, act, k, n in sorted(out, reverse=True)[:12]:
        print(f"{exp:7.3f} exposed {act:7.3f} active {k:6d} launches  {n[:90]}")


if __name__ == "__main__":
    main()

"""Summarise rocprofv3 SQLite outputs into the files committed under profiles/.

    python tools/prof_summary.py --stats gpurun_out/TAG/prof/run_results.db \
        --pmc gpurun_out/TAG/pmc/run_results.db --skip-first 43 --out profiles/r01_complex-fb15k237-sufficient

writes <out>_kernel_stats.csv (the --kernel-trace --stats table: every kernel's calls,
total and average duration) and <out>_pmc.json (per-kernel FETCH_SIZE per launch,
corrected to bytes as MI355X_MICROARCH.md prescribes: KiB -> bytes, x2 for gfx950's
half-counted wide reads).  --skip-first drops each kernel's first N dispatches (the
warm-up step) from the timed-region averages it also reports.
"""
import argparse
import csv
import json
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--pmc")
    ap.add_argument("--pmc-write", help="a WRITE_SIZE pass of the same command")
    ap.add_argument("--pmc-sq", help="an SQ pass with SQ_INSTS_VALU (VALU issue of the kernels)")
    ap.add_argument("--skip-first", type=int, default=0)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    c = sqlite3.connect(a.stats)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    with open(a.out + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for r in rows:
            w.writerow([r[0], r[1], f"{r[2]:.3f}", f"{r[3]:.3f}", f"{r[4]:.2f}"])
    per = defaultdict(list)
    spans = defaultdict(list)
    for name, s, e in c.execute("select name, start, end from kernels order by start"):
        per[name].append((e - s) / 1e3)
        spans[name].append((s, e))
    timed = {n: (sum(d[a.skip_first:]) / max(1, len(d) - a.skip_first), len(d) - a.skip_first)
             for n, d in per.items() if len(d) > a.skip_first}

    def union_us(iv):
        # launches of one kernel on two streams can overlap: the time the device spent in it
        iv = sorted(iv)
        total, (s0, e0) = 0, iv[0]
        for s1, e1 in iv[1:]:
            if s1 > e0:
                total += e0 - s0
                s0, e0 = s1, e1
            else:
                e0 = max(e0, e1)
        return (total + e0 - s0) / 1e3

    summary = {"timed_avg_us": {n: {"avg_us": v[0], "launches": v[1],
                                    "union_us_per_launch": union_us(spans[n][a.skip_first:]) / v[1]}
                                for n, v in timed.items()}}
    if a.pmc:
        p = sqlite3.connect(a.pmc)
        acc = defaultdict(list)
        for name, val in p.execute("select kernel_name, value from counters_collection where counter_name='FETCH_SIZE'"):
            acc[name].append(val)
        summary["fetch_bytes_per_launch"] = {
            n: {"launches": len(v), "fetch_size_kib_avg": sum(v) / len(v),
                "hbm_bytes": 2.0 * 1024.0 * sum(v) / len(v)} for n, v in acc.items()}
        summary["fetch_note"] = ("FETCH_SIZE (KiB, L2 memory-side reads incl. Infinity-Cache hits) x 1024 x 2: "
                                 "gfx950 tallies 128-B requests at 64 B (MI355X_MICROARCH.md, HBM)")
    if a.pmc_write:
        p = sqlite3.connect(a.pmc_write)
        acc = defaultdict(list)
        for name, val in p.execute("select kernel_name, value from counters_collection where counter_name='WRITE_SIZE'"):
            acc[name].append(val)
        summary["write_bytes_per_launch"] = {
            n: {"launches": len(v), "write_size_kib_avg": sum(v) / len(v), "hbm_bytes": 1024.0 * sum(v) / len(v)}
            for n, v in acc.items()}
        summary["write_note"] = "WRITE_SIZE (KiB) x 1024: exact for 16-B-per-lane stores (MI355X_MICROARCH.md, HBM)"
    if a.pmc_sq:
        p = sqlite3.connect(a.pmc_sq)
        acc = defaultdict(lambda: defaultdict(list))
        for name, cn, val in p.execute("select kernel_name, counter_name, value from counters_collection"):
            acc[name][cn].append(val)
        summary["sq_per_launch"] = {n: {cn: sum(v) / len(v) for cn, v in d.items()} for n, d in acc.items()}
    # the library sources these passes measured (bench.py cites a pass only for the same sources)
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from kelpie_amd._lib import source_sha16
    summary["library_source_sha16"] = source_sha16()
    with open(a.out + "_pmc.json", "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

"""Per-kernel averages of every counter in a rocprofv3 --pmc SQLite output.

    python tools/pmc_dump.py gpurun_out/TAG/pmcX/run_results.db [kernel-substring]
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    c = sqlite3.connect(db)
    acc = defaultdict(list)
    for name, cn, val in c.execute("select kernel_name, counter_name, value from counters_collection"):
        if pat in name:
            acc[(name, cn)].append(val)
    for (name, cn), v in sorted(acc.items()):
        print(f"{name[:60]:60s} {cn:28s} n={len(v):4d} avg={sum(v) / len(v):.4g}")


if __name__ == "__main__":
    main()

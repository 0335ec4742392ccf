"""Summarise KELPIE_PIPELINE_TRACE output (engine.compute_relevance_pipeline).

    python tools/pipeline_trace.py gpurun_out/<tag>/trace.jsonl [--last]

Each line of the file is one pipeline call: [(seconds, event, batch), ...] with events
schedule / scheduled (scheduling thread), run / draws / ran (batch thread: start, the
batch's deferred draws complete, device call returned), joined / finish / finished
(scheduling thread: batch thread joined, results collected and finalised).  Prints the
per-batch stage durations (medians over the call's batches after the first two) and
the step period, so the bound of a host-bound pipeline can be read off.
"""
import argparse
import json
import statistics as st


def summarise(events):
    by = {}
    for t, ev, b in events:
        by.setdefault(b, {})[ev] = t
    bs = sorted(k for k in by if k >= 0)
    if len(bs) < 4:
        return None
    steady = bs[2:]
    t0 = min(t for t, _, _ in events)

    def med(a, b):
        v = [by[k][b] - by[k][a] for k in steady if a in by[k] and b in by[k]]
        return 1e3 * st.median(v) if v else float("nan")

    ends = by.pop(-1, {})
    bs = sorted(by)
    starts = [by[k]["schedule"] for k in steady]
    period = 1e3 * (starts[-1] - starts[0]) / max(1, len(starts) - 1)
    rows = {
        "period_ms": period,
        "schedule (python)": med("schedule", "scheduled"),
        "scheduled -> run start": med("scheduled", "run"),
        "draw wait (batch thread)": med("run", "draws"),
        "pack + library call": med("draws", "ran"),
        "ran -> joined": med("ran", "joined"),
        "finish (collect + finalise)": med("finish", "finished"),
        "scheduled -> next schedule": 1e3 * st.median(
            [by[k + 1]["schedule"] - by[k]["scheduled"] for k in steady if k + 1 in by]),
    }
    lines = []
    for k in bs[:8]:
        e = by[k]
        lines.append("  b%-3d " % k + "  ".join(f"{ev}={1e3 * (e[ev] - t0):8.2f}" for ev in
                                                 ("schedule", "scheduled", "run", "draws", "ran", "joined",
                                                  "finish", "finished") if ev in e))
    if "enter" in ends and "exit" in ends:
        rows["call span"] = 1e3 * (ends["exit"] - ends["enter"])
        rows["enter -> first schedule"] = 1e3 * (by[bs[0]]["schedule"] - ends["enter"])
        rows["last finished -> unwound"] = 1e3 * (ends.get("unwound", ends["exit"])
                                                  - max(e.get("finished", 0) for e in by.values()))
        rows["unwound -> exit (rng sync)"] = 1e3 * (ends["exit"] - ends.get("unwound", ends["exit"]))
    return rows, lines, len(bs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last", action="store_true", help="only the last pipeline call")
    args = ap.parse_args()
    with open(args.path) as f:
        calls = [json.loads(line) for line in f if line.strip()]
    if args.last:
        calls = calls[-1:]
    for i, ev in enumerate(calls):
        r = summarise(ev)
        if r is None:
            continue
        rows, lines, n = r
        print(f"call {i}: {n} batches")
        for k, v in rows.items():
            print(f"  {k:30s} {v:8.2f} ms")
        print("\n".join(lines))


if __name__ == "__main__":
    main()

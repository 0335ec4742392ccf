"""Host-side cost of one engine batch's scheduling (no GPU needed): the reference-order
RNG protocol, kelpie views and slot assembly of a bench workload, with the deferred
TransE draws' final wait timed separately and a cProfile of the scheduling thread.

    python tools/host_profile.py [--workload transe-fb15k237-necessary] [--preds 16]
"""
import argparse
import cProfile
import os
import pstats
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kelpie_amd import NecessaryPostTrainingEngine, SufficientPostTrainingEngine, rng as krng  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="transe-fb15k237-necessary", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--preds", type=int, default=16)
    ap.add_argument("--repeats", type=int, default=3)
    args = ap.parse_args()
    wl = bench.WORKLOADS[args.workload]
    ds, model, _ = bench.build(wl, 0, 0)
    cls = SufficientPostTrainingEngine if wl["mode"] == "sufficient" else NecessaryPostTrainingEngine
    eng = cls(model, ds, wl["hp"])
    preds = bench.pick_preds(ds, args.preds * (args.repeats + 1), seed=1234)
    random.seed(42)
    np.random.seed(42)
    torch.manual_seed(42)
    waits = []
    orig_wait = krng._lib.rng_wait

    def timed_wait():
        t = time.perf_counter()
        orig_wait()
        waits.append(time.perf_counter() - t)
    krng._lib.rng_wait = timed_wait
    calls_t = []
    orig_calls = krng._lib.transe_calls

    def timed_calls(*a, **k):
        t = time.perf_counter()
        r = orig_calls(*a, **k)
        calls_t.append(time.perf_counter() - t)
        return r
    krng._lib.transe_calls = timed_calls

    def items(ps):
        out = []
        for p in ps:
            rules = [[c] for c in bench.candidates_of(ds, p, wl["candidates"])]
            if wl["mode"] == "sufficient":
                out.append((p, rules, eng.select_entities_to_convert(p, wl["convert"], 200)))
            else:
                out.append((p, rules))
        return out
    batches = [items(preds[k * args.preds:(k + 1) * args.preds]) for k in range(args.repeats + 1)]
    for k in range(args.repeats + 1):
        eng.set_cache()
        waits.clear()
        calls_t.clear()
        prof = cProfile.Profile() if k == args.repeats else None
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        with eng.rng.deferred():
            slots, _, _ = eng._schedule_all(batches[k], None)
        if prof:
            prof.disable()
        dt = time.perf_counter() - t0
        rows = (int(eng._native_arrays(slots[0].native[0])["nrow"].sum()) if slots and slots[0].native is not None
                else sum(len(s.rows) for s in slots))
        t1 = time.perf_counter()
        eng._pack(slots)
        dp = time.perf_counter() - t1
        print(f"batch {k}: schedule {dt * 1e3:.2f} ms  final draw wait {sum(waits) * 1e3:.2f} ms  "
              f"pack {dp * 1e3:.2f} ms  kp_rng_transe_calls {sum(calls_t) * 1e3:.2f} ms  slots {len(slots)}  rows {rows}", flush=True)
    pstats.Stats(prof).sort_stats(os.environ.get("HP_SORT", "tottime")).print_stats(int(os.environ.get("HP_N", "16")))


if __name__ == "__main__":
    main()

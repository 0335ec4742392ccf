"""Host-only cost of the engine pipeline of a bench workload (no GPU needed): the device
context is replaced by a null one whose post-training returns at once (after an optional
fixed sleep standing in for the device time), so what is left is the scheduling
thread's reference-order RNG protocol, slot assembly and finalisation and the batch
threads' packing -- the bound of a host-bound line such as TransE.  Prints the period
per batch and a cProfile of the scheduling thread.  TEST/DIAGNOSTIC tool; the product
never uses the null context.

    python tools/host_pipeline.py [--workload transe-fb15k237-necessary] [--batches 12] [--device-ms 1.0]
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kelpie_amd import NecessaryPostTrainingEngine, SufficientPostTrainingEngine  # noqa: E402


class NullContext:
    def __init__(self, dim, device_ms):
        self.dim, self.device_s = dim, device_ms * 1e-3

    def posttrain_rank(self, hp, x0, row_off, rows, rng_off, rng, pred, filt_off, filt, want_x=False):
        n = len(row_off) - 1
        if self.device_s:
            time.sleep(self.device_s)  # releases the interpreter lock, as the library call does
        return np.zeros(n, np.float32), np.ones(n, np.int64), None

    def last_timing(self):
        return {}

    def convertible(self, ents, p, o, filt_off, filt):
        return np.ones(len(ents), bool)  # every candidate entity converts (host cost only)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="transe-fb15k237-necessary", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--batches", type=int, default=12)
    ap.add_argument("--device-ms", type=float, default=1.0)
    args = ap.parse_args()
    wl = bench.WORKLOADS[args.workload]
    ds, model, _ = bench.build(wl, None, 0)
    ctxs = [NullContext(model.dimension, args.device_ms) for _ in range(3)]
    model._ctx = ctxs[0]
    model.contexts = lambda n: ctxs[:max(1, n)]
    cls = SufficientPostTrainingEngine if wl["mode"] == "sufficient" else NecessaryPostTrainingEngine
    eng = cls(model, ds, wl["hp"])
    per = wl.get("preds_per_step", 1)
    preds = bench.pick_preds(ds, per * args.batches, seed=1234)
    random.seed(42)
    np.random.seed(42)
    torch.manual_seed(42)
    batches = []
    for k in range(args.batches):
        items = []
        for p in preds[k * per:(k + 1) * per]:
            rules = [[c] for c in bench.candidates_of(ds, p, wl["candidates"])]
            items.append((p, rules, eng.select_entities_to_convert(p, wl["convert"], 200))
                         if wl["mode"] == "sufficient" else (p, rules))
        batches.append(items)
    depth = int(os.environ.get("KELPIE_PIPELINE_DEPTH", wl.get("depth", 2)))
    eng.compute_relevance_pipeline(batches[:2], depth=depth)  # warm-up
    prof = cProfile.Profile()
    t0 = time.perf_counter()
    prof.enable()
    outs = eng.compute_relevance_pipeline(batches[2:], depth=depth)
    prof.disable()
    dt = time.perf_counter() - t0
    n_b = len(batches) - 2
    n_c = sum(len(o) for b in outs for o in b)
    print(f"{n_b} batches, {n_c} candidates in {dt * 1e3:.1f} ms: {dt / n_b * 1e3:.2f} ms per batch, "
          f"{n_c / dt:.0f} cand/s host-only (device {args.device_ms} ms per batch)")
    pstats.Stats(prof).sort_stats(os.environ.get("HP_SORT", "tottime")).print_stats(int(os.environ.get("HP_N", "25")))


if __name__ == "__main__":
    main()

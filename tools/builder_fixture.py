"""Full-size StochasticBuilder fixtures from the reference itself (development container
only; TEST INFRASTRUCTURE, never runs on the GPU box: it imports /root/reference through
``tests/golden/ref_harness.py``).

The north star asks for "identical explanation rankings", and the reference's recorded
metric is ``#relevances / execution_time`` over the whole ``StochasticBuilder``
(singletons, then compound rules with early exit and the stochastic stop,
ref ``src/explanation_builders/stochastic_builder.py:33-107,126-175``).  This script runs
the reference's own pipeline (ref ``src/explain.py:49-89`` ``build_pipeline``: topology
prefilter, ``StochasticBuilder`` at the default xsi -- 5 necessary, 0.9 sufficient --
then ``pipeline.explain(pred, prefilter_k=20)`` as ``explain.py:196`` calls it) on the
bench's synthetic graph and weights (``bench.build``), over a sequence of the bench's
predictions in one process, seeds 42 once before the first (``explain.py:144``), so the
generators carry over from one prediction to the next as they do in the reference.

Three variants (``tools/conditioning.py`` patches): ``fp32`` (the reference as it runs),
``fp64`` (tables, layers and optimizer state in float64, the random draws taken in
float32 exactly as the fp32 run takes them) and ``fp32_perm`` (fp32 with the reduction
order permuted: the ComplEx coordinates, or the ConvE filters).

Recorded per prediction and variant: the prefiltered candidates, every
``compute_relevance`` call in order (rule, relevance, seconds), the target rank / score
of every post-training, the ``random.random()`` values the builder consumed, and the
``output.json`` record (``rule_to_relevance``, ``#relevances``, ``execution_time``).
Written to ``tests/golden/builder/<workload>__<variant>.json`` (data only) after every
prediction.

    python tools/builder_fixture.py --workload complex-fb15k237-necessary --preds 0 1 2 --variant fp32
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import bench  # noqa: E402
import noise_floor  # noqa: E402
import ref_harness  # noqa: E402
from conditioning import _Patches, to_double  # noqa: E402
from kelpie_amd import Dataset, synth  # noqa: E402

OUT_DIR = os.path.join(ROOT, "tests", "golden", "builder")


def _jsonable(x):
    if hasattr(x, "item"):
        return x.item()
    return list(x)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True, choices=sorted(bench.WORKLOADS))
    ap.add_argument("--preds", type=int, nargs="+", required=True,
                    help="indices into bench.pick_preds(seed=1234), explained in this order")
    ap.add_argument("--variant", choices=["fp32", "fp64", "fp32_perm"], default="fp32")
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--prefilter-k", type=int, default=20)
    ap.add_argument("--max-calls", type=int, default=400,
                    help="stop the run (recorded as truncated) after this many engine calls")
    ap.add_argument("--xsi", type=float, default=None,
                    help="relevance threshold (explain.py --relevance_threshold); default the builder's")
    ap.add_argument("--name", default=None, help="fixture name (default: the workload)")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    wl = bench.WORKLOADS[args.workload]
    name = args.name or args.workload
    src = ref_harness.load_reference()
    from src.explain import build_pipeline

    g = synth.make_graph(wl["shape"], seed=0)
    w = synth.make_weights(wl["model"], g.num_entities, g.num_relations, wl["dim"], seed=0)
    ds = Dataset(g.num_entities, g.num_relations, g.train, g.valid, g.test, name=wl["shape"])
    n_pick = max(args.preds) + 1
    all_preds = bench.pick_preds(ds, n_pick, seed=1234)
    preds = [all_preds[i] for i in args.preds]

    cols = None
    if args.variant == "fp32_perm":
        # the same function with other reduction orders (tools/conditioning.py): ComplEx
        # coordinates permuted in the tables and the kelpie init, ConvE filters permuted
        from conditioning import permuted_weights
        w, cols = permuted_weights(wl, w)
    dataset, model = noise_floor.reference_model(src, wl, g, w)
    if wl["mode"] == "sufficient":
        # synthetic graphs have entities with no training triple; the reference's degree
        # lookup (engine.py:73) is a plain dict (tools/conditioning.py, same fix)
        import collections
        dataset.entity_to_degree = collections.defaultdict(int, dataset.entity_to_degree)
    D = wl["dim"] * (2 if wl["model"] == "ComplEx" else 1)
    patches = None
    if args.variant == "fp64":
        patches = _Patches(fp64=True, dim=D).__enter__()
        to_double(model)
    elif cols is not None:
        patches = _Patches(init_cols=cols, dim=D).__enter__()

    ref_harness.seed_all(42)  # explain.py:144, once for the whole sequence
    pipeline = build_pipeline(model, dataset, wl["hp"], wl["mode"], None, None, args.xsi, None)
    engine = pipeline.builder.engine

    calls, draws, pts = [], [], []
    orig_rel = engine.compute_relevance
    orig_res = engine.get_triple_results
    orig_random = random.random

    class Truncated(Exception):
        pass

    def rel_logged(pred, rule):
        if len(calls) >= args.max_calls:
            raise Truncated()
        pts.clear()
        t0 = time.time()
        r = orig_rel(pred, rule)
        calls.append({"rule": [[int(v) for v in t] for t in rule], "relevance": float(r),
                      "seconds": time.time() - t0, "results": list(pts)})
        if len(calls) % 10 == 0:
            print(f"  {len(calls)} calls, last {r:.4f} ({calls[-1]['seconds']:.1f}s)", flush=True)
        return r

    def res_logged(m, triple):
        r = orig_res(m, triple)
        pts.append({"rank": int(r["target_rank"]), "score": float(r["target_score"])})
        return r

    def random_logged():
        v = orig_random()
        draws.append(v)
        return v

    engine.compute_relevance = rel_logged
    engine.get_triple_results = res_logged
    random.random = random_logged

    path = os.path.join(OUT_DIR, f"{name}__{args.variant}.json")
    os.makedirs(OUT_DIR, exist_ok=True)
    rec = {}
    rec.update({"workload": args.workload, "pred_indices": args.preds, "preds": [list(p) for p in preds],
                "prefilter_k": args.prefilter_k, "xsi": pipeline.builder.xsi, "seed": 42,
                "generator": "tools/builder_fixture.py (reference pipeline imported through "
                             "tests/golden/ref_harness.py, CPU)"})
    runs = rec.setdefault("runs", {})
    out = runs[args.variant] = {"threads": args.threads, "explanations": [], "truncated": False}
    try:
        for pred in preds:
            calls.clear()
            draws.clear()
            t0 = time.time()
            print(f"pred {pred}", flush=True)
            ex = pipeline.explain(pred=tuple(pred), prefilter_k=args.prefilter_k)
            ex = json.loads(json.dumps(ex, default=_jsonable))
            ex["pred"] = list(pred)
            ex["candidates"] = [c["rule"][0] for c in calls[:len(calls)] if len(c["rule"]) == 1]
            ex["entities_to_convert"] = ([int(e) for e in engine.entities_to_convert]
                                         if wl["mode"] == "sufficient" else None)
            ex["calls"] = list(calls)
            ex["random_draws"] = list(draws)
            ex["wall_seconds"] = time.time() - t0
            out["explanations"].append(ex)
            print(f"  -> #relevances {ex['#relevances']}, {len(draws)} draws, {ex['wall_seconds']:.0f}s, "
                  f"top {ex['rule_to_relevance'][0]}", flush=True)
            with open(path, "w") as f:
                json.dump(rec, f)
    except Truncated:
        out["truncated"] = True
        out["truncated_pred"] = list(pred)
        out["truncated_calls"] = list(calls)
        print(f"TRUNCATED at {args.max_calls} calls on pred {pred}", flush=True)
    finally:
        random.random = orig_random
        if patches is not None:
            patches.__exit__(None, None, None)
    with open(path, "w") as f:
        json.dump(rec, f)


if __name__ == "__main__":
    main()

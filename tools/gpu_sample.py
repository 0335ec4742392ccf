"""Run the HIP engine on the sample of a reference noise-floor record (GPU box).

    python tools/gpu_sample.py profiles/noise_floor_<workload>.json [run-name]

Reads the prediction, candidates and conversion entities that
``tools/noise_floor.py`` ran through the reference (development container),
evaluates them with the MI355X engine on the same synthetic graph, weights and
seeds, and adds a ``"gpu"`` run (relevances, rank deltas, per post-training
target score / rank) plus the GPU-vs-reference match rates to the same file.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main(path, name="gpu"):
    with open(path) as f:
        rec = json.load(f)
    wl = bench.WORKLOADS[rec["workload"]]
    ds, model, _ = bench.build(wl, 0, 0)
    from kelpie_amd import NecessaryPostTrainingEngine, SufficientPostTrainingEngine
    pred = tuple(rec["pred"])
    cands = [tuple(c) for c in rec["candidates"]]
    bench.seed_all(42)
    if wl["mode"] == "sufficient":
        eng = SufficientPostTrainingEngine(model, ds, wl["hp"])
        eng.entities_to_convert = list(rec["entities_to_convert"])
    else:
        eng = NecessaryPostTrainingEngine(model, ds, wl["hp"])
    rels = eng.compute_relevance_batch(pred, [[c] for c in cands])
    pairs = [pb for rj in eng.last_results for pb in rj] if wl["mode"] == "sufficient" else eng.last_results
    deltas = [pt["target_rank"] - b["target_rank"] for pt, b in pairs]
    rec["runs"][name] = {"relevances": [float(r) for r in rels], "rank_deltas": deltas,
                          "results": [{"pt": pt, "base": b} for pt, b in pairs]}
    for other, run in rec["runs"].items():
        if other == name:
            continue
        d = run["rank_deltas"]
        rec.setdefault("rank_delta_match_rates", {})[f"{name} vs {other}"] = float(np.mean([a == b for a, b in zip(deltas, d)]))
        rec.setdefault("rank_delta_max_abs_diff", {})[f"{name} vs {other}"] = int(
            max(abs(a - b) for a, b in zip(deltas, d)))
    print(json.dumps({name: rec["runs"][name]["rank_deltas"], "rates": rec["rank_delta_match_rates"],
                      "scores": [(pt["target_score"], b["target_score"]) for pt, b in pairs]}))
    with open(path, "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:3])

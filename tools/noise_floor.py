"""Rank-delta noise floor of the reference itself (development container only).

TEST INFRASTRUCTURE: imports the read-only reference through
``tests/golden/ref_harness.py`` and never runs on the GPU box.

The bench's ``rank_delta_match_rate`` compares the HIP engine with the CPU
oracle on a sample of the bench workload.  With the reference's random
initialisers the post-training targets are dense (ConvE sigmoid outputs
0.5 +- 0.02 over 123k entities), and Adam turns last-bit gradient differences
into visible kelpie-row differences, so two correct fp32 implementations can
rank the target a few places apart.  This script measures how far the
reference disagrees WITH ITSELF when only the CPU thread count changes (torch
re-blocks its GEMM reductions), and how far the oracle is from both, on the
bench's own workload and sample:

    python tools/noise_floor.py --workload conve-yago310-necessary --threads 1 8

Writes ``profiles/noise_floor_<workload>.json``: per run the base / pt target
score and rank of each sampled candidate, and the pairwise rank-delta match
rates.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import bench  # noqa: E402
import ref_harness  # noqa: E402
from kelpie_amd import synth  # noqa: E402


def reference_model(src, wl, g, w):
    from src.data import Dataset
    from src.link_prediction import MODEL_REGISTRY
    name = "noise_" + wl["shape"]
    ref_harness.register_dataset(name, g.num_entities, g.num_relations, g.train, g.valid, g.test)
    dataset = Dataset(name)
    cls = MODEL_REGISTRY[wl["model"]]["class"]
    mp = {"dimension": wl["dim"]}
    if wl["model"] == "ComplEx":
        mp["init_scale"] = 1e-3
    elif wl["model"] == "TransE":
        mp["norm"] = 2
    else:
        mp.update({"input_dropout_rate": wl.get("input_dropout", 0.0),
                   "hidden_dropout_rate": wl.get("hidden_dropout", 0.0),
                   "feature_map_dropout_rate": wl.get("fmap_dropout", 0.0), "hidden_layer_size": 9728})
    model = cls(dataset=dataset, hp=cls.get_hyperparams_class()(**mp))
    with torch.no_grad():
        model.entity_embeddings.data = torch.from_numpy(w["entity_embeddings"].copy())
        model.relation_embeddings.data = torch.from_numpy(w["relation_embeddings"].copy())
        if wl["model"] == "ConvE":
            model.convolutional_layer.weight.data = torch.from_numpy(w["conv_weight"].copy())
            model.convolutional_layer.bias.data = torch.from_numpy(w["conv_bias"].copy())
            model.hidden_layer.weight.data = torch.from_numpy(w["fc_weight"].copy())
            model.hidden_layer.bias.data = torch.from_numpy(w["fc_bias"].copy())
            for i, bn in ((1, model.batch_norm_1), (2, model.batch_norm_2), (3, model.batch_norm_3)):
                bn.weight.data = torch.from_numpy(w[f"bn{i}_weight"].copy())
                bn.bias.data = torch.from_numpy(w[f"bn{i}_bias"].copy())
                bn.running_mean.data = torch.from_numpy(w[f"bn{i}_mean"].copy())
                bn.running_var.data = torch.from_numpy(w[f"bn{i}_var"].copy())
    model.eval()
    return dataset, model


def run_reference(src, wl, dataset, model, pred, cands, ents):
    from src.relevance_engines import NecessaryPostTrainingEngine, SufficientPostTrainingEngine
    ref_harness.seed_all(42)
    cls = SufficientPostTrainingEngine if wl["mode"] == "sufficient" else NecessaryPostTrainingEngine
    eng = cls(model, dataset, wl["hp"])
    eng.set_cache()
    if ents is not None:
        eng.entities_to_convert = list(ents)
    log = []
    orig = eng.get_triple_results

    def wrapped(m, triple):
        r = orig(m, triple)
        log.append({"triple": [int(v) for v in triple], "target_score": float(r["target_score"]),
                    "target_rank": int(r["target_rank"])})
        return r

    eng.get_triple_results = wrapped
    rels, calls = [], []
    run_reference.cand_seconds = []
    for c in cands:
        log.clear()
        t0 = time.time()
        rels.append(float(eng.compute_relevance(pred, [c])))
        run_reference.cand_seconds.append(time.time() - t0)
        calls.append(list(log))
    return rels, calls


def deltas_of(calls, mode=None):
    """(pt_rank - base_rank) per post-training, in call order.  The first call logs
    (base, pt) per conversion entity (one for necessary mode); the base results are
    cached afterwards, so later calls log the pt results only."""
    first = calls[0]
    base = [r["target_rank"] for r in first[0::2]]
    out = [pt["target_rank"] - b for pt, b in zip(first[1::2], base)]
    for c in calls[1:]:
        out += [pt["target_rank"] - b for pt, b in zip(c, base)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="conve-yago310-necessary", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--candidates", type=int, default=3)
    ap.add_argument("--no-oracle", action="store_true")
    args = ap.parse_args()
    wl = bench.WORKLOADS[args.workload]
    src = ref_harness.load_reference()
    g = synth.make_graph(wl["shape"], seed=0)
    w = synth.make_weights(wl["model"], g.num_entities, g.num_relations, wl["dim"], seed=0)
    from kelpie_amd import Dataset
    ds = Dataset(g.num_entities, g.num_relations, g.train, g.valid, g.test, name=wl["shape"])
    pred = bench.pick_preds(ds, 1, seed=1234)[0]
    cands = bench.candidates_of(ds, pred, wl["candidates"])[:args.candidates]
    dataset, model = reference_model(src, wl, g, w)
    ents = None
    if wl["mode"] == "sufficient":
        from src.relevance_engines import SufficientPostTrainingEngine
        ref_harness.seed_all(42)
        se = SufficientPostTrainingEngine(model, dataset, wl["hp"])
        se.select_entities_to_convert(pred, wl["convert"], 200)  # sets entities_to_convert (engine.py:125)
        ents = [int(e) for e in se.entities_to_convert]
    out = {"workload": args.workload, "pred": list(pred), "candidates": [list(c) for c in cands],
           "entities_to_convert": ents, "runs": {}}
    for t in args.threads:
        torch.set_num_threads(t)
        t0 = time.time()
        rels, log = run_reference(src, wl, dataset, model, pred, cands, ents)
        out["runs"][f"reference_threads{t}"] = {"relevances": rels, "results": log,
                                                "rank_deltas": deltas_of(log, wl["mode"]),
                                                "seconds": time.time() - t0}
        print(f"reference threads={t}: {rels} deltas {deltas_of(log, wl['mode'])} ({time.time() - t0:.0f}s)",
              flush=True)
    if not args.no_oracle:
        from oracle import kelpie_oracle as ko
        om = ko.OracleModel(wl["model"], w, wl["dim"],
                            {"init_scale": 1e-3, "hidden_dropout_rate": wl.get("hidden_dropout", 0.0),
                             "input_dropout_rate": wl.get("input_dropout", 0.0),
                             "feature_map_dropout_rate": wl.get("fmap_dropout", 0.0)})
        ods = ko.OracleDataset(ds.num_entities, ds.num_relations, ds.training_triples, ds.validation_triples,
                               ds.testing_triples)
        bench.seed_all(42)
        oeng = ko.OracleEngine(om, ods, wl["hp"])
        rels, deltas = [], []
        for c in cands:
            if wl["mode"] == "sufficient":
                r, det = oeng.sufficient_relevance(pred, [c], ents)
                deltas += [pt["target_rank"] - b["target_rank"] for pt, b in det]
            else:
                r, pt, b = oeng.necessary_relevance(pred, [c])
                deltas.append(pt["target_rank"] - b["target_rank"])
            rels.append(float(r))
        out["runs"]["oracle"] = {"relevances": rels, "rank_deltas": deltas}
        print(f"oracle: {rels} deltas {deltas}", flush=True)
    names = list(out["runs"])
    rates, diffs = {}, {}
    for i, a in enumerate(names):
        for b in names[i + 1:]:
            da, db = out["runs"][a]["rank_deltas"], out["runs"][b]["rank_deltas"]
            rates[f"{a} vs {b}"] = float(np.mean([x == y for x, y in zip(da, db)])) if da else None
            diffs[f"{a} vs {b}"] = int(max(abs(x - y) for x, y in zip(da, db))) if da else None
    out["rank_delta_match_rates"] = rates
    out["rank_delta_max_abs_diff"] = diffs
    print(json.dumps(rates, indent=1))
    with open(os.path.join(ROOT, "profiles", f"noise_floor_{args.workload}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

"""Golden vectors for edge-case engine calls (empty / total edits).

TEST INFRASTRUCTURE, run once in the development container through ref_harness.
For three golden cases, on a low-degree subject:
  * necessary, the rule removes every training triple of the subject (the kelpie
    entity post-trains on zero rows);
  * necessary, an empty rule (the reference raises "No removal to undo." from
    KelpieDataset.undo_removal after the post-training);
  * a regular call afterwards (checks the random stream stays in sync after both);
  * sufficient mode, "stale conversion entities": select_entities_to_convert on
    prediction A, then on prediction B with a degree cap no entity meets; the
    reference returns [] WITHOUT resetting ``entities_to_convert``
    (engine.py:90-91), so B's relevance is computed on A's entities.

    python tests/golden/make_edge_golden.py
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import ref_harness  # noqa: E402
from make_golden import CASES, build_case  # noqa: E402

EDGE_CASES = ["complex_tiny", "transe_tiny", "conve60_tiny"]


def main():
    src = ref_harness.load_reference()
    from src.relevance_engines import NecessaryPostTrainingEngine

    out = {}
    for name in EDGE_CASES:
        out.setdefault("_stale_entities", {})[name] = stale_entities(src, name)
        g, _, dataset, model = build_case(src, name, CASES[name])
        ref_harness.seed_all(42)
        eng = NecessaryPostTrainingEngine(model, dataset, CASES[name]["hp"])
        eng.set_cache()
        subj = min((e for e in dataset.entity_to_training_triples if len(dataset.entity_to_training_triples[e]) >= 2),
                   key=lambda e: (len(dataset.entity_to_training_triples[e]), e))
        trip = [tuple(int(v) for v in t) for t in dataset.entity_to_training_triples[subj]]
        t0 = trip[0]
        pred = (int(subj), t0[1], t0[2] if t0[0] == subj else t0[0])
        rec = {"pred": list(pred), "all_rows": [list(t) for t in trip], "calls": []}
        for label, rule in (("all_removed", trip), ("empty", []), ("regular", trip[:1])):
            try:
                rel = eng.compute_relevance(pred, list(rule))
                rec["calls"].append({"label": label, "rule": [list(t) for t in rule], "relevance": float(rel)})
            except Exception as e:  # the reference's own error
                rec["calls"].append({"label": label, "rule": [list(t) for t in rule], "error": type(e).__name__,
                                     "message": str(e)})
        out[name] = rec
        print(name, rec["calls"], flush=True)
    with open(os.path.join(HERE, "edge_golden.json"), "w") as f:
        json.dump(out, f)


def stale_entities(src, name):
    from src.relevance_engines import SufficientPostTrainingEngine
    g, _, dataset, model = build_case(src, name, CASES[name])
    ref_harness.seed_all(42)
    eng = SufficientPostTrainingEngine(model, dataset, CASES[name]["hp"])
    eng.set_cache()
    deg = dataset.entity_to_degree
    test = [tuple(int(v) for v in t) for t in g.test if 3 <= deg.get(int(t[0]), 0) <= 20]
    pa, pb = test[0], next(t for t in test[1:] if t[0] != test[0][0])
    ret_a = eng.select_entities_to_convert(pa, 3, 200)
    ents_a = [int(e) for e in eng.entities_to_convert]
    ret_b = eng.select_entities_to_convert(pb, 3, 0.5)  # truthy cap below every degree: no candidate
    ents_b = [int(e) for e in eng.entities_to_convert]
    rule = [tuple(int(v) for v in dataset.entity_to_training_triples[pb[0]][0])]
    rel = float(eng.compute_relevance(pb, rule))
    rec = {"pred_a": list(pa), "pred_b": list(pb), "entities_a": ents_a, "returned_b": ret_b,
           "entities_after_b": ents_b, "returned_a_is_none": ret_a is None, "rule": [list(t) for t in rule],
           "relevance": rel}
    print(name, "stale entities", rec, flush=True)
    return rec


if __name__ == "__main__":
    main()

"""Golden vectors for the baseline relevance engines.

Run in the development container only (needs ``/root/reference``):

    python tests/golden/make_baseline_golden.py

Imports the reference through ``ref_harness`` (CPU redirect + import
placeholders) and, on the ``complex_tiny`` / ``conve60_tiny`` cases of
``make_golden.py`` (same graph, weights and seeds), records

* ``NecessaryDPEngine`` / ``SufficientDPEngine.compute_relevance(pred,
  perspective, triple)`` (``src/relevance_engines/data_poisoning_engine.py``)
  for the head and tail perspectives, ComplEx (the only model of the three with
  ``score_embeddings``; TransE and ConvE raise ``AttributeError``, recorded);
* ``NecessaryCriageEngine`` / ``SufficientCriageEngine.compute_relevance(pred,
  triple, perspective)`` (``src/relevance_engines/criage_engine.py``) for ComplEx
  and ConvE, on perspective entities with at least D + 8 tail triples (D the
  model dimension), so that the float64 Hessian the reference inverts has full
  rank (with fewer tail triples it is singular and numpy's inverse
  returns rounding-dominated values);
* ``CriagePreFilter.select_triples`` (``src/prefilters/criage_prefilter.py``).

Output: ``tests/golden/baseline_golden.json`` (data only; no reference source).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import make_golden  # noqa: E402
import ref_harness  # noqa: E402


def _f(x):
    if x is None:
        return None
    return float(np.asarray(x).reshape(-1)[0])


def dp_cases(src, name):
    from src.relevance_engines import NecessaryDPEngine, SufficientDPEngine
    cfg = make_golden.CASES[name]
    g, w, dataset, model = make_golden.build_case(src, name, cfg)
    eps = cfg["hp"].get("lr", 0.01)
    preds = make_golden.pick_preds(dataset, g)
    out = {"case": name, "epsilon": eps, "necessary": [], "sufficient": []}
    nec = NecessaryDPEngine(model, dataset, eps)
    for pred in preds:
        s, _, o = pred
        for persp, ent in (("head", s), ("tail", o)):
            trip = sorted(dataset.entity_to_training_triples.get(ent, []))[:5]
            rels = [_f(nec.compute_relevance(tuple(pred), persp, tuple(t))) for t in trip]
            out["necessary"].append({"pred": list(map(int, pred)), "perspective": persp,
                                     "triples": [list(map(int, t)) for t in trip], "relevance": rels})
    ref_harness.seed_all(42)
    suf = SufficientDPEngine(model, dataset, eps)
    pred = preds[0]
    suf.select_entities_to_convert(pred, 4, 200)
    ents = [int(e) for e in suf.entities_to_convert]
    s, _, o = pred
    for persp in ("head", "tail"):
        trip = sorted(dataset.entity_to_training_triples.get(s, []))[:4]
        rels = [_f(suf.compute_relevance(tuple(pred), persp, tuple(t))) for t in trip]
        out["sufficient"].append({"pred": list(map(int, pred)), "perspective": persp, "entities_to_convert": ents,
                                  "triples": [list(map(int, t)) for t in trip], "relevance": rels})
    return out


def dp_unsupported(src, name):
    from src.relevance_engines import NecessaryDPEngine
    cfg = make_golden.CASES[name]
    g, w, dataset, model = make_golden.build_case(src, name, cfg)
    pred = make_golden.pick_preds(dataset, g)[0]
    trip = sorted(dataset.entity_to_training_triples[pred[0]])[0]
    try:
        NecessaryDPEngine(model, dataset, 0.01).compute_relevance(tuple(pred), "head", tuple(trip))
        return {"case": name, "error": None}
    except Exception as e:  # noqa: BLE001
        return {"case": name, "error": type(e).__name__, "message": str(e)}


def criage_cases(src, name):
    from src.prefilters import CriagePreFilter
    from src.relevance_engines import NecessaryCriageEngine, SufficientCriageEngine
    cfg = make_golden.CASES[name]
    g, w, dataset, model = make_golden.build_case(src, name, cfg)
    D = int(model.dimension)
    tails = {}
    for h, r, t in dataset.training_triples:
        tails.setdefault(int(t), []).append((int(h), int(r), int(t)))
    rich = {e for e, ts in tails.items() if len(ts) >= D + 8}
    test = [tuple(int(v) for v in t) for t in g.test]
    out = {"case": name, "dimension": D, "necessary": [], "sufficient": [], "prefilter": []}
    pf = CriagePreFilter(dataset)
    nec = NecessaryCriageEngine(model, dataset)
    picked = 0
    for pred in test:
        s, p, o = pred
        for persp, ent in (("tail", o), ("head", s)):
            if ent not in rich or picked >= 4:
                continue
            cands = pf.select_triples(pred=pred, k=3)
            out["prefilter"].append({"pred": list(pred), "k": 3, "triples": [list(map(int, t)) for t in cands]})
            trip = [t for t in cands if t[2] == ent][:3] or sorted(tails[ent])[:3]
            rels = [_f(nec.compute_relevance(pred, tuple(int(v) for v in t), persp)) for t in trip]
            out["necessary"].append({"pred": list(pred), "perspective": persp,
                                     "triples": [list(map(int, t)) for t in trip], "relevance": rels})
            picked += 1
    # sufficient: conversion entities drawn among the well-conditioned ones
    ref_harness.seed_all(42)
    suf = SufficientCriageEngine(model, dataset)
    for pred in test:
        s, p, o = pred
        if o not in rich:
            continue
        ents = sorted(rich - {s, o})[:3]
        if len(ents) < 2:
            continue
        suf.entities_to_convert = ents
        trip = sorted(tails[o])[:3]
        rels = [_f(suf.compute_relevance(pred, tuple(t), "tail")) for t in trip]
        out["sufficient"].append({"pred": list(pred), "perspective": "tail", "entities_to_convert": ents,
                                  "triples": [list(map(int, t)) for t in trip], "relevance": rels})
        break
    return out


def main():
    src = ref_harness.load_reference()
    import builtins
    _print = builtins.print
    rec = {"dp": [], "dp_unsupported": [], "criage": []}
    builtins.print = lambda *a, **k: None  # the reference prints per rule
    try:
        rec["dp"].append(dp_cases(src, "complex_tiny"))
        rec["dp_unsupported"] = [dp_unsupported(src, n) for n in ("transe_tiny", "conve60_tiny")]
        rec["criage"].append(criage_cases(src, "complex_tiny"))
        rec["criage"].append(criage_cases(src, "conve60_tiny"))
    finally:
        builtins.print = _print
    with open(os.path.join(HERE, "baseline_golden.json"), "w") as f:
        json.dump(rec, f, indent=1)
    for c in rec["dp"]:
        print("dp", c["case"], [r["relevance"] for r in c["necessary"][:2]], [r["relevance"] for r in c["sufficient"]])
    print("dp unsupported", rec["dp_unsupported"])
    for c in rec["criage"]:
        print("criage", c["case"], [r["relevance"] for r in c["necessary"]], [r["relevance"] for r in c["sufficient"]])


if __name__ == "__main__":
    main()

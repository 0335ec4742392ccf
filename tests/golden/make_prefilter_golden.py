"""Golden vectors for the candidate prefilters.

TEST INFRASTRUCTURE, run once in the development container (the reference is
imported through ``ref_harness``; nothing here runs on the GPU box).  It runs the
reference's ``TopologyPreFilter`` and ``WeightedTopologyPreFilter``
(``src/prefilters/topology_prefilter.py``, ``weighted_topology_prefilter.py``,
networkx under the hood) on a sparse synthetic graph with self loops and
several components, and on synthetic entity classes drawn from a small
vocabulary (so Jaccard costs repeat and equal-length paths exist).

Writes ``prefilter_golden.npz`` (training triples, class CSR) and
``prefilter_golden.json`` (per prediction: the selected triples for several k
and each candidate's distance).

    python tests/golden/make_prefilter_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import ref_harness  # noqa: E402

from kelpie_amd import synth  # noqa: E402

N_CLASSES = 6


def make_inputs(seed=5):
    g = synth.make_graph("tiny", seed=seed, n_ent=600, n_rel=8, n_train=800, n_valid=40, n_test=80)
    rng = np.random.default_rng(seed)
    loops = np.array([[e, int(rng.integers(8)), e] for e in rng.choice(600, 6, replace=False)], np.int64)
    train = np.concatenate([g.train, loops])
    classes = [sorted(rng.choice(N_CLASSES, int(rng.integers(0, 4)), replace=False).tolist()) for _ in range(600)]
    return g, train, classes


def main():
    src = ref_harness.load_reference()
    import pandas as pd
    from src.data import Dataset as RefDataset
    from src.prefilters import TopologyPreFilter, WeightedTopologyPreFilter

    g, train, classes = make_inputs()
    ref_harness.register_dataset("prefilter_synth", 600, 8, train, g.valid, g.test)
    ds = RefDataset(dataset="prefilter_synth")
    ds.entities_semantic_impl = pd.DataFrame({"entity": list(range(600)),
                                              "classes": [{f"c{c}" for c in cl} for cl in classes]})
    topo = TopologyPreFilter(ds)
    wtopo = WeightedTopologyPreFilter(ds)

    test = [tuple(int(v) for v in t) for t in g.test]
    preds = [t for t in test if len(ds.entity_to_training_triples.get(t[0], [])) >= 2][:12]
    out = {"n_ent": 600, "n_rel": 8, "preds": []}
    for pred in preds:
        rec = {"pred": list(pred)}
        for name, pf in (("topology", topo), ("weighted", wtopo)):
            pf.pred_s, _, pf.pred_o = pred
            cands = sorted(ds.entity_to_training_triples[pred[0]])
            rec[name + "_dist"] = {",".join(map(str, t)): float(pf.analyze_triple(t)) for t in cands}
            for k in (3, 50, -1):
                rec[f"{name}_k{k}"] = [list(map(int, t)) for t in pf.select_triples(pred=pred, k=k)]
        out["preds"].append(rec)
        print(pred, rec["topology_k3"], rec["weighted_k3"], flush=True)

    off = np.zeros(601, np.int64)
    off[1:] = np.cumsum([len(c) for c in classes])
    cls = np.array([c for cl in classes for c in cl], np.int32)
    np.savez(os.path.join(HERE, "prefilter_golden.npz"), train=train, valid=g.valid, test=g.test,
             class_off=off, class_ids=cls)
    with open(os.path.join(HERE, "prefilter_golden.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()

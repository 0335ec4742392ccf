"""Candidate prefilters vs the reference's golden vectors.

The fixtures come from the reference's TopologyPreFilter and
WeightedTopologyPreFilter run on a sparse synthetic graph with self loops and
repeated Jaccard costs (tests/golden/make_prefilter_golden.py).  The searches
run in the library's host C++ (kp_graph_*), so these tests need no GPU.
"""
import json
import os

import numpy as np
import pytest

import kelpie_amd as ka
from kelpie_amd.prefilters import NoPreFilter, TopologyPreFilter, WeightedTopologyPreFilter

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def case():
    arr = np.load(os.path.join(HERE, "prefilter_golden.npz"))
    with open(os.path.join(HERE, "prefilter_golden.json")) as f:
        rec = json.load(f)
    ds = ka.Dataset(rec["n_ent"], rec["n_rel"], arr["train"], arr["valid"], arr["test"])
    off, ids = arr["class_off"], arr["class_ids"]
    classes = {e: {f"c{c}" for c in ids[off[e]:off[e + 1]]} for e in range(rec["n_ent"])}
    return rec, ds, classes


def test_topology_prefilter_matches_reference(case):
    rec, ds, _ = case
    pf = TopologyPreFilter(ds)
    for p in rec["preds"]:
        pred = tuple(p["pred"])
        for k in (3, 50, -1):
            assert pf.select_triples(pred, k=k) == [tuple(t) for t in p[f"topology_k{k}"]], (pred, k)
    # batched selection == per-prediction selection
    preds = [tuple(p["pred"]) for p in rec["preds"]]
    assert pf.select_triples_batch(preds, 50) == [pf.select_triples(q, 50) for q in preds]


def test_topology_distances_match_reference(case):
    rec, ds, _ = case
    pf = TopologyPreFilter(ds)
    for p in rec["preds"]:
        s, _, o = p["pred"]
        d = pf.graph.bfs([o])[0]
        for key, ref in p["topology_dist"].items():
            t = tuple(int(v) for v in key.split(","))
            e = t[2] if t[0] == s else t[0]
            got = 1e6 if d[e] < 0 else float(d[e])
            assert got == ref, (p["pred"], t, got, ref)


def test_weighted_prefilter_matches_reference_bitwise(case):
    rec, ds, classes = case
    pf = WeightedTopologyPreFilter(ds, classes)
    for p in rec["preds"]:
        pred = tuple(p["pred"])
        s, _, o = pred
        keys = list(p["weighted_dist"].items())
        ends = []
        for key, _ in keys:
            t = tuple(int(v) for v in key.split(","))
            ends.append(t[2] if t[0] == s else t[0])
        got = pf.graph.dijkstra_pairs(ends, [o] * len(ends))
        for (key, ref), g in zip(keys, got):
            g = 1e6 if np.isinf(g) else float(g)
            assert g == ref, (pred, key, g, ref)  # bit-exact float64 path sums
        for k in (3, 50, -1):
            assert pf.select_triples(pred, k=k) == [tuple(t) for t in p[f"weighted_k{k}"]], (pred, k)


def test_no_prefilter(case):
    _, ds, _ = case
    pf = NoPreFilter(ds)
    s = int(ds.training_triples[0][0])
    assert pf.select_triples((s, 0, 0)) == ds.entity_to_training_triples[s]


def test_graph_rejects_bad_ids(case):
    _, ds, _ = case
    from kelpie_amd._lib import Graph, KelpieHipError
    with pytest.raises(KelpieHipError):
        Graph(10, [[0, 0, 11]])
    g = Graph(ds.num_entities, ds.training_triples)
    with pytest.raises(KelpieHipError):
        g.bfs([ds.num_entities])

"""Edge-case engine calls vs the reference (tests/golden/make_edge_golden.py):
a rule that removes every training triple of the subject (post-training on zero
rows), an empty rule (the reference raises "No removal to undo." after the
post-training, and its draws stay consumed), and a regular call afterwards."""
import json
import os

import pytest

from engine_cases import TOL, build_product
from golden_io import seed_all

import kelpie_amd as ka

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(HERE, "edge_golden.json")) as f:
    GOLD = json.load(f)
STALE = GOLD.pop("_stale_entities")


def _run(name, backend):
    rec = GOLD[name]
    gold_rec, ds, model = build_product(name, backend)
    seed_all(gold_rec["seed"])
    eng = ka.NecessaryPostTrainingEngine(model, ds, gold_rec["hp"])
    eng.set_cache()
    pred = tuple(rec["pred"])
    for call in rec["calls"]:
        rule = [tuple(t) for t in call["rule"]]
        if "error" in call:
            with pytest.raises(Exception, match=call["message"]):
                eng.compute_relevance(pred, rule)
        else:
            rel = eng.compute_relevance(pred, rule)
            assert abs(rel - call["relevance"]) <= TOL, (name, call["label"], rel, call["relevance"])


@pytest.mark.parametrize("name", sorted(GOLD))
def test_edge_calls_host_protocol(name):
    _run(name, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLD))
def test_edge_calls_gpu(name):
    _run(name, "gpu")


def _stale(name, backend):
    """select_entities_to_convert with no surviving candidate leaves the previous
    prediction's entities in place (engine.py:90-91), and the sufficient relevance
    of the next call uses them."""
    rec = STALE[name]
    gold_rec, ds, model = build_product(name, backend)
    seed_all(gold_rec["seed"])
    eng = ka.SufficientPostTrainingEngine(model, ds, gold_rec["hp"])
    eng.set_cache()
    eng.select_entities_to_convert(tuple(rec["pred_a"]), 3, 200)
    assert [int(e) for e in eng.entities_to_convert] == rec["entities_a"]
    assert eng.select_entities_to_convert(tuple(rec["pred_b"]), 3, 0.5) == rec["returned_b"] == []
    assert [int(e) for e in eng.entities_to_convert] == rec["entities_after_b"] == rec["entities_a"]
    rel = eng.compute_relevance(tuple(rec["pred_b"]), [tuple(t) for t in rec["rule"]])
    assert abs(rel - rec["relevance"]) <= TOL * max(1.0, abs(rec["relevance"])), (name, rel, rec["relevance"])


@pytest.mark.parametrize("name", sorted(STALE))
def test_stale_conversion_entities_host_protocol(name):
    _stale(name, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(STALE))
def test_stale_conversion_entities_gpu(name):
    _stale(name, "gpu")

"""BASELINE.json configs[0] on real data: TransE, DBpedia50, necessary mode, the first
10 predictions of the reference's ``preds/TransE_DBpedia50.csv`` and its explanation
config (d = 256, 65 epochs), end to end: labels -> ``Dataset.from_directory`` ->
``read_preds`` -> ``build_pipeline`` (topology prefilter k = 20, StochasticBuilder,
xsi 5) -> ``explain_preds`` -> ``output.json``, against the reference's own pipeline
run on the same triples and seeded weights (tests/golden/make_dbpedia50_golden.py).

The DBpedia50 triples travel as data under tests/golden/dbpedia50/ (the reference's
own data files, copied by the generator); /root/reference is not read here.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from engine_cases import TOL

import kelpie_amd as ka
from kelpie_amd import synth
from kelpie_amd.pipeline import read_preds, run_explain

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GOLD_PATH = os.path.join(HERE, "dbpedia50_transe.json")
# the same reference pipeline run in float64 (make_dbpedia50_golden.py --fp64): the second
# variant of the element-wise rule of tests/test_fullsize_reference.py
GOLD64_PATH = os.path.join(HERE, "dbpedia50_transe_fp64.json")
DATA = os.path.join(HERE, "dbpedia50")
pytestmark = pytest.mark.skipif(not os.path.exists(GOLD_PATH), reason="DBpedia50 golden not generated")


def _load():
    with open(GOLD_PATH) as f:
        rec = json.load(f)
    ds = ka.Dataset.from_directory(DATA, name="DBpedia50")
    w = synth.make_weights("TransE", ds.num_entities, ds.num_relations, rec["model_params"]["dimension"],
                           seed=rec["weights_seed"])
    return rec, ds, w


def test_dbpedia50_loader_and_weights():
    """from_directory reproduces the golden's dataset (sizes, every pred maps to ids) and
    the seeded weights are the ones the reference ran with (sha256)."""
    rec, ds, w = _load()
    assert (ds.num_entities, ds.num_relations, len(ds.training_triples)) == \
        (rec["num_entities"], rec["num_relations"], rec["n_train"])
    for k, v in w.items():
        assert hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() == rec["weights_sha256"][k], k
    preds = read_preds(os.path.join(HERE, rec["preds_file"]))
    assert len(preds) == 10
    for p, ex in zip(preds, rec["explanations"]):
        s, r, o = ds.ids_triple(p)
        assert 0 <= s < ds.num_entities and 0 <= o < ds.num_entities and 0 <= r < ds.num_relations
        assert list(ex["triple"]) == list(p)


def _run(backend, tmpdir, n_preds):
    """explain.py's main loop through ``run_explain`` (seeds, the reference model
    construction's draws, the checkpoint as a state dict, pipeline, output.json)."""
    rec, ds, w = _load()
    out_path = os.path.join(str(tmpdir), "output.json")
    preds = read_preds(os.path.join(HERE, rec["preds_file"]))[:n_preds]
    state = {"entity_embeddings": w["entity_embeddings"], "relation_embeddings": w["relation_embeddings"]}
    if backend == "cpu":
        from cpu_backend import OracleBackedContext
        orig = ka.models.TransE.__init__

        def init_with_standin(self, *a, **k):
            orig(self, *a, **k)
            self._ctx = OracleBackedContext(self)

        ka.models.TransE.__init__ = init_with_standin
    try:
        run_explain("TransE", ds, state, rec["model_params"], rec["hp"], "necessary", preds,
                    prefilter_k=rec["prefilter_k"], xsi=rec["xsi"], output_path=out_path)
    finally:
        if backend == "cpu":
            ka.models.TransE.__init__ = orig
    with open(out_path) as f:
        got = json.load(f)
    assert len(got) == n_preds
    ex64 = [None] * n_preds
    if os.path.exists(GOLD64_PATH):
        with open(GOLD64_PATH) as f:
            ex64 = json.load(f)["explanations"][:n_preds]
    for g, e, e64 in zip(got, rec["explanations"][:n_preds], ex64):
        assert set(g) == {"triple", "rule_to_relevance", "#relevances", "execution_time"}
        assert list(g["triple"]) == list(e["triple"])
        assert g["#relevances"] == e["#relevances"], (g["triple"], g["#relevances"], e["#relevances"])
        assert len(g["rule_to_relevance"]) == len(e["rule_to_relevance"])
        rel64 = {json.dumps(r): v for r, v in e64["rule_to_relevance"]} if e64 else {}
        for (rule, rel), (erule, erel) in zip(g["rule_to_relevance"], e["rule_to_relevance"]):
            assert [list(t) for t in rule] == [list(t) for t in erule]
            tol = TOL * max(1.0, abs(erel))
            if abs(rel - erel) <= tol:
                continue
            # element-wise rule: where the reference's float32 and float64 runs disagree (a
            # near-tie the ranks resolve differently), the engine may lie anywhere between them
            v64 = rel64.get(json.dumps(erule))
            assert v64 is not None and abs(v64 - erel) > tol, (rule, rel, erel, v64)
            assert min(erel, v64) - tol <= rel <= max(erel, v64) + tol, (rule, rel, erel, v64)


def test_dbpedia50_pipeline_host_protocol(tmp_path):
    """The host protocol (oracle-backed stand-in for the HIP context), all 10 predictions."""
    _run("cpu", tmp_path, 10)


@pytest.mark.gpu
def test_dbpedia50_pipeline_gpu(tmp_path):
    """All 10 predictions through the HIP engine."""
    _run("gpu", tmp_path, 10)

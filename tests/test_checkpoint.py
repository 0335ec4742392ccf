"""f1: the reference's checkpoint format (``torch.save(model.state_dict())``, loaded at
explain.py:169-176) through ``kelpie_amd.models.from_state_dict``.

tests/golden/make_ckpt_golden.py saved the reference models of three golden cases
and recorded their ``all_scores``; here each checkpoint is loaded with
``torch.load(..., weights_only=True)``, turned into a frozen model, scored against the
reference's scores (1e-6 relative), and run through the engine against the case's
reference relevances (the same goldens as the in-memory model)."""
import json
import os

import numpy as np
import pytest
import torch

from engine_cases import TOL, _close
from golden_io import load_case, seed_all

import kelpie_amd as ka
from kelpie_amd.models import from_state_dict

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(HERE, "ckpt_golden.json")) as f:
    GOLD = json.load(f)


def _model(name, backend):
    rec, arrays, _ = load_case(name)
    ds = ka.Dataset(rec["num_entities"], rec["num_relations"], arrays["train"], arrays["valid"], arrays["test"])
    state = torch.load(os.path.join(HERE, f"ckpt_{name}.pt"), weights_only=True)
    assert sorted(state) == GOLD[name]["keys"]
    model = from_state_dict(rec["model"], ds, state, rec["model_params"])
    if backend == "cpu":
        from cpu_backend import OracleBackedContext
        model._ctx = OracleBackedContext(model)
    return rec, ds, model


def _check(name, backend):
    rec, ds, model = _model(name, backend)
    g = GOLD[name]
    got = model.all_scores(np.asarray(g["triples"], dtype=np.int64))
    ref = np.asarray(g["all_scores"])
    assert got.shape == ref.shape
    assert np.max(np.abs(got - ref)) <= 1e-6 * max(1.0, float(np.max(np.abs(ref)))), name
    # the engine on the loaded model reproduces the reference relevances of the case
    seed_all(rec["seed"])
    eng = ka.NecessaryPostTrainingEngine(model, ds, rec["hp"])
    block = rec["necessary"][0]
    eng.set_cache()
    rels = eng.compute_relevance_batch(tuple(block["pred"]), [[tuple(t) for t in c["rule"]] for c in block["calls"]])
    for call, rel, (pt, _) in zip(block["calls"], rels, eng.last_results):
        assert abs(rel - call["relevance"]) <= TOL, (name, rel, call["relevance"])
        assert pt["target_rank"] == call["results"][-1]["target_rank"]
        assert _close(pt["target_score"], call["results"][-1]["target_score"])


@pytest.mark.parametrize("name", sorted(GOLD))
def test_checkpoint_roundtrip_host(name):
    _check(name, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLD))
def test_checkpoint_roundtrip_gpu(name):
    _check(name, "gpu")

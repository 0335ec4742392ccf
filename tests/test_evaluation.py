"""Link-prediction evaluation vs the reference's goldens.

tests/golden/eval_golden.json holds the reference's Model.predict_triples ranks and
Evaluator metrics on the test triples of three golden cases (make_eval_golden.py).
CPU tests pin the oracle restatement and the host Evaluator (through the oracle
stand-in); the GPU test runs kp_predict_tails.
"""
import json
import os

import numpy as np
import pytest

from engine_cases import build_product
from kelpie_amd.evaluation import Evaluator

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(HERE, "eval_golden.json")) as f:
    GOLD = json.load(f)
CASES = sorted(GOLD)


def _check(name, backend, tmp_path=None):
    rec = GOLD[name]
    _, ds, model = build_product(name, backend)
    triples = np.array(rec["triples"], dtype=np.int64)
    res = model.predict_triples(triples)
    tail = [r["rank"]["tail"] for r in res]
    head = [r["rank"]["head"] for r in res]
    assert tail == rec["tail_rank"], (name, [(a, b) for a, b in zip(tail, rec["tail_rank"]) if a != b][:5])
    assert head == rec["head_rank"], (name, [(a, b) for a, b in zip(head, rec["head_rank"]) if a != b][:5])
    for a, b in zip([r["score"]["tail"] for r in res] + [r["score"]["head"] for r in res],
                    rec["tail_score"] + rec["head_score"]):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), (name, a, b)
    out = os.path.join(str(tmp_path), "ranks.csv") if tmp_path else "ranks.csv"
    m = Evaluator(model).evaluate(triples, write_output=tmp_path is not None, output_path=out)
    for k, v in rec["metrics"].items():
        assert abs(m[k] - v) <= 1e-9 * max(1.0, abs(v)), (name, k, m[k], v)
    if tmp_path is not None:
        with open(out) as f:
            lines = f.read().strip().split("\n")
        assert lines[0] == "head;relation;tail;head_rank;tail_rank" and len(lines) == len(triples) + 1


@pytest.mark.parametrize("name", CASES)
def test_oracle_predict_tails_matches_reference(name):
    """Pins oracle.kelpie_oracle.predict_tails against the reference's ranks."""
    from oracle import kelpie_oracle as ko
    from cpu_backend import OracleBackedContext
    rec = GOLD[name]
    _, ds, model = build_product(name, "cpu")
    om = model.ctx.om if isinstance(model.ctx, OracleBackedContext) else None
    sc, rk = ko.predict_tails(om, ds, np.array(rec["triples"]))
    assert rk == rec["tail_rank"]


@pytest.mark.parametrize("name", CASES)
def test_evaluator_host_protocol(name, tmp_path):
    _check(name, "cpu", tmp_path)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_predict_tails_gpu_vs_reference(name, tmp_path):
    _check(name, "gpu", tmp_path)

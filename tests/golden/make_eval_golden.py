"""Golden vectors for link-prediction evaluation.

TEST INFRASTRUCTURE, run once in the development container through ref_harness
(nothing here runs on the GPU box).  For three of the tiny golden cases it runs
the reference's ``Model.predict_triples`` (model.py:25-68, conve.py:160-184) and
``Evaluator.evaluate`` (link_prediction/evaluation.py:16-48) on the test triples
and records per-triple tail / head scores and filtered ranks plus MRR / Hits@k.
Weights are the cases' own (regenerated from their seed by make_golden.build_case).

    python tests/golden/make_eval_golden.py
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
from make_golden import CASES, build_case  # noqa: E402

EVAL_CASES = ["transe_tiny", "complex_tiny", "conve60_tiny"]


def main():
    src = ref_harness.load_reference()
    from src.link_prediction.evaluation import Evaluator

    out = {}
    for name in EVAL_CASES:
        g, _, dataset, model = build_case(src, name, CASES[name])
        test = np.asarray(dataset.testing_triples)[:60]
        res = model.predict_triples(test)
        metrics = Evaluator(model).evaluate(test)
        out[name] = {
            "triples": test.astype(int).tolist(),
            "tail_rank": [int(r["rank"]["tail"]) for r in res],
            "head_rank": [int(r["rank"]["head"]) for r in res],
            "tail_score": [float(r["score"]["tail"]) for r in res],
            "head_score": [float(r["score"]["head"]) for r in res],
            "metrics": {k: float(v) for k, v in metrics.items()},
        }
        print(name, out[name]["metrics"], flush=True)
    with open(os.path.join(HERE, "eval_golden.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()

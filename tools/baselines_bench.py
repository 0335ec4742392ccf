"""Throughput of the baseline engines on the FB15k-237 shape.

    python tools/baselines_bench.py [--preds 8]

ComplEx d = 200 (D = 400) with the reference random init on the synthetic
FB15k-237 graph.  Per prediction (head perspective):
  * data poisoning: every training triple of the subject;
  * CRIAGE: the CriagePreFilter candidates (k = 20 per side), the float64
    Hessians of the perspective entities included;
all predictions' candidates in one launch (compute_relevance_multi).
The CPU oracle is timed on a bounded sample of the same work.  Prints one JSON
line per engine.  (With random weights most Hessians are rank-deficient, so
CRIAGE values are not meaningful here: this measures time only; parity is in
tests/test_baselines.py.)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preds", type=int, default=8)
    ap.add_argument("--dump", default=None, help="save the CRIAGE relevances (float64, .npy) here")
    a = ap.parse_args()
    import kelpie_amd.baselines as kb
    wl = bench.WORKLOADS["complex-fb15k237-necessary"]
    ds, model, w = bench.build(wl, 0, 0)
    preds = bench.pick_preds(ds, a.preds, seed=1234)
    dp = kb.NecessaryDPEngine(model, ds, 0.043)
    cr = kb.NecessaryCriageEngine(model, ds)
    pf = kb.CriagePreFilter(ds)
    jobs_dp = [(p, sorted(ds.entity_to_training_triples[p[0]])) for p in preds]
    jobs_cr = [(p, pf.select_triples(p, 20)) for p in preds]
    # warm-up
    dp.compute_relevance_batch(jobs_dp[0][0], "head", jobs_dp[0][1][:2])
    cr.compute_relevance_batch(jobs_cr[0][0], jobs_cr[0][1][:1], "head")
    out = {}
    for name, eng, jobs in (("dp", dp, jobs_dp), ("criage", cr, jobs_cr)):
        jobs = [(p, c) for p, c in jobs if c]
        n = sum(len(c) for _, c in jobs)
        t0 = time.perf_counter()
        res = eng.compute_relevance_multi(jobs, "head")  # every prediction's candidates in one launch
        dt = time.perf_counter() - t0
        out[name] = (n, dt)
        if name == "criage" and a.dump:
            np.save(a.dump, np.array([np.nan if v is None else float(v) for r in res for v in r], dtype=np.float64))
    # CPU oracle on a bounded sample (the first prediction's first candidates)
    from oracle import kelpie_oracle as ko
    om = ko.OracleModel("ComplEx", w, wl["dim"], {"init_scale": 1e-3})
    ods = ko.OracleDataset(ds.num_entities, ds.num_relations, ds.training_triples, ds.validation_triples,
                           ds.testing_triples)
    from collections import defaultdict
    tails = defaultdict(list)
    for h, r, t in ods.training_triples.tolist():
        tails[t].append((h, r, t))
    cpu = {}
    p, cands = jobs_dp[0]
    t0 = time.perf_counter()
    for c in cands[:20]:
        ko.dp_relevance(om, p, "head", c, 0.043, "necessary")
    cpu["dp"] = (min(20, len(cands)), time.perf_counter() - t0)
    p, cands = next((j for j in jobs_cr if j[1]))
    t0 = time.perf_counter()
    k = 0
    for c in cands[:3]:
        try:
            ko.criage_relevance(om, ods, p, c, "head", "necessary", tails=tails)
        except np.linalg.LinAlgError:
            pass
        k += 1
    cpu["criage"] = (k, time.perf_counter() - t0)
    for name in ("dp", "criage"):
        n, dt = out[name]
        cn, cdt = cpu[name]
        print(json.dumps({"engine": name, "workload": "ComplEx FB15k-237 (synthetic), d=200, head perspective",
                          "candidates": n, "predictions": len(preds), "seconds": dt, "value": n / dt,
                          "unit": "candidates/s", "includes": "host packing, H2D/D2H copies, per-call Hessians",
                          "cpu_baseline": {"value": cn / cdt, "unit": "candidates/s", "kind": "port",
                                           "sample": f"{cn} candidates of 1 prediction, oracle numpy"}}),
              flush=True)


if __name__ == "__main__":
    main()

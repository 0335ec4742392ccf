"""The regularised full-width ComplEx case against the reference itself.

``tests/golden/complex200_reg_fullwidth.json`` (``make_reg_fullwidth_golden.py``): the
reference run, fp32 as it runs and in fp64, on exactly the inputs of
``test_gpu_parity.py::test_complex_vs_oracle_full_width`` -- D = 400, the 2,000-entity
graph, two predictions and a multi-minibatch hub, Adagrad for 20 epochs -- without a
regulariser and with N3 or N2 at weight 0.05 (ref ``regularizers.py:25-46``).

The host test pins the oracle: on every post-training it equals the reference's fp64
run, ranks exactly and scores within 1e-5 relative (the oracle computes the whole step
in fp64).  The reference's own fp32 run is up to 1.5e-3 away from its fp64 run there (N3,
the first prediction's second candidate: a near-cancelling coordinate that Adagrad's
normalised first step turns into a full step), which is what the device test allows.

The GPU test holds the device to the reference element by element, as the full-size
fixtures are held (tests/test_fullsize_reference.py): ranks equal to the reference where
its fp32 and fp64 runs agree, else between them; scores within 1e-4 relative of the fp64
run where the fp32 run is within 1e-4 of it, else no farther from it than the fp32 run.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "complex200_reg_fullwidth.json")
REGS = ["none", "N3", "N2"]
pytestmark = pytest.mark.skipif(not os.path.exists(GOLD), reason="golden not generated")


def _case():
    import kelpie_amd as ka
    from kelpie_amd import synth
    with open(GOLD) as f:
        rec = json.load(f)
    g = synth.make_graph(rec["graph"]["shape"], seed=rec["graph"]["seed"])
    ds = ka.Dataset(g.num_entities, g.num_relations, g.train, g.valid, g.test)
    w = synth.make_weights("ComplEx", g.num_entities, g.num_relations, rec["weights"]["dim"],
                           seed=rec["weights"]["seed"], trained_scale=rec["weights"]["trained_scale"])
    return rec, ds, w


def _ref(rec, reg, variant):
    """[(pt rank, pt score, base rank, base score)] per call, in call order."""
    out = []
    for blk in rec["runs"][f"{reg}_{variant}"]:
        base = blk["calls"][0]["results"][0]
        for c in blk["calls"]:
            pt = c["results"][-1]
            out.append((pt["rank"], pt["score"], base["rank"], base["score"]))
    return out


def _run(rec, ds, w, reg, backend):
    import kelpie_amd as ka
    from golden_io import seed_all
    hp = dict(rec["hp"]) if reg == "none" else dict(rec["hp"], regularizer_name=reg, regularizer_weight=0.05)
    model = ka.ComplEx(ds, w["entity_embeddings"], w["relation_embeddings"], init_scale=rec["init_scale"])
    if backend == "cpu":
        from cpu_backend import OracleBackedContext
        model._ctx = OracleBackedContext(model)
    seed_all(rec["seed"])
    eng = ka.NecessaryPostTrainingEngine(model, ds, hp)
    out = []
    for pred, cands in zip(rec["preds"], rec["candidates"]):
        eng.set_cache()
        eng.compute_relevance_batch(tuple(pred), [[tuple(c)] for c in cands])
        out += [(pt["target_rank"], pt["target_score"], b["target_rank"], b["target_score"]) for pt, b in eng.last_results]
    return out


def misses(got, r32, r64, tol=1e-4):
    """Elements of ``got`` outside the reference's own fp32 / fp64 spread."""
    bad = []
    for i, (g, a, b) in enumerate(zip(got, r32, r64)):
        for k in (0, 2):  # ranks
            lo, hi = min(a[k], b[k]), max(a[k], b[k])
            if not lo <= g[k] <= hi:
                bad.append((i, "rank", g[k], a[k], b[k]))
        for k in (1, 3):  # scores, against fp64
            err, ref_err = abs(g[k] - b[k]) / abs(b[k]), abs(a[k] - b[k]) / abs(b[k])
            if err > max(tol, ref_err):
                bad.append((i, "score", g[k], a[k], b[k]))
    return bad


@pytest.mark.slow
def test_oracle_equals_reference_fp64():
    rec, ds, w = _case()
    for reg in ("N3", "N2"):  # the regularised cases (the plain one is the oracle goldens' business)
        got = _run(rec, ds, w, reg, "cpu")
        r64 = _ref(rec, reg, "fp64")
        for g, b in zip(got, r64):
            assert g[0] == b[0] and g[2] == b[2], (reg, g, b)
            assert abs(g[1] - b[1]) <= 1e-5 * abs(b[1]) and abs(g[3] - b[3]) <= 1e-5 * abs(b[3]), (reg, g, b)


@pytest.mark.gpu
@pytest.mark.parametrize("reg", REGS)
def test_device_within_reference_spread(reg):
    rec, ds, w = _case()
    got = _run(rec, ds, w, reg, "gpu")
    r32, r64 = _ref(rec, reg, "fp32"), _ref(rec, reg, "fp64")
    print(json.dumps({"reg": reg, "gpu": got, "ref_fp32": r32, "ref_fp64": r64}))
    assert not misses(got, r32, r64), misses(got, r32, r64)
    # and the ranks match the fp64 reference on all but at most one element
    assert sum(g[0] == b[0] and g[2] == b[2] for g, b in zip(got, r64)) >= len(got) - 1

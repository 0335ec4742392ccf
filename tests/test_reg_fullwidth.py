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
its variants (fp32, fp64, fp32 with a permuted reduction order) agree, else between them;
scores within 1e-4 relative of the fp64 run, or no farther from it than an fp32 variant.
Where the reference itself misses 1e-4 (an fp32 variant more than 1e-4 from fp64: one
post-training of the 36, N3's, whose fp32 run is 1.5e-3 off) the score is held to that
spread and the rank to one place around the variants' ranks -- the rank an exact fp64
count gives for a score inside that spread.
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


def ill_conditioned(rec, reg, tol=1e-4):
    """Post-trainings where the reference cannot meet the north star's 1e-4 itself: one of
    its fp32 runs (as it runs, or with a permuted reduction order) lies more than ``tol``
    (relative) from its fp64 run in the pt or base score."""
    r64 = _ref(rec, reg, "fp64")
    fp32s = [_ref(rec, reg, v) for v in ("fp32", "fp32_perm") if f"{reg}_{v}" in rec["runs"]]
    out = set()
    for i, b in enumerate(r64):
        for r in fp32s:
            if abs(r[i][1] - b[1]) > tol * abs(b[1]) or abs(r[i][3] - b[3]) > tol * abs(b[3]):
                out.add(i)
    return out


def misses(got, r32, r64, tol=1e-4, others=(), loose=()):
    """Elements of ``got`` outside the reference's own spread: ranks between the smallest
    and the largest of the reference variants (fp32, fp64, and the fp32 run with a
    permuted reduction order when recorded), scores within ``tol`` of fp64 or no farther
    from it than the farthest fp32 variant."""
    bad = []
    for i, (g, a, b) in enumerate(zip(got, r32, r64)):
        vs = [a, b] + [o[i] for o in others]
        slack = 1 if i in loose else 0  # an ill-conditioned post-training: one place either way
        for k in (0, 2):  # ranks
            lo, hi = min(v[k] for v in vs), max(v[k] for v in vs)
            if not lo - slack <= g[k] <= hi + slack:
                bad.append((i, "rank", g[k], [v[k] for v in vs]))
        for k in (1, 3):  # scores, against fp64
            err = abs(g[k] - b[k]) / abs(b[k])
            ref_err = max(abs(v[k] - b[k]) / abs(b[k]) for v in vs)
            if err > max(tol, ref_err):
                bad.append((i, "score", g[k], [v[k] for v in vs]))
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
    others = [_ref(rec, reg, "fp32_perm")] if f"{reg}_fp32_perm" in rec["runs"] else []
    print(json.dumps({"reg": reg, "gpu": got, "ref_fp32": r32, "ref_fp64": r64, "ref_other": others}))
    loose = ill_conditioned(rec, reg)
    bad = misses(got, r32, r64, others=others, loose=loose)
    assert not bad, bad
    # and the ranks match the fp64 reference on all but at most one element
    assert sum(g[0] == b[0] and g[2] == b[2] for g, b in zip(got, r64)) >= len(got) - 1

"""Baseline relevance engines: data poisoning and CRIAGE.

Golden vectors: ``tests/golden/baseline_golden.json`` (``make_baseline_golden.py``, the
reference run on CPU).  The CPU tests pin the oracle restatement; the GPU tests run
the HIP engines (``kp_dp_relevance``, ``kp_criage_relevance``) through the C ABI.
Relevances within 1e-4 (CRIAGE: relative 1e-4 as well, its values come out of a
float64 solve of a float32-assembled system).
"""
import json
import os

import numpy as np
import pytest

from golden_io import GOLDEN, load_case
from oracle import kelpie_oracle as ko

TOL = 1e-4


def _golden():
    with open(os.path.join(GOLDEN, "baseline_golden.json")) as f:
        return json.load(f)


def _oracle(name):
    rec, arrays, weights = load_case(name)
    ds = ko.OracleDataset(rec["num_entities"], rec["num_relations"], arrays["train"], arrays["valid"], arrays["test"])
    model = ko.OracleModel(rec["model"], weights, rec["model_params"]["dimension"], rec["model_params"])
    return ds, model


def _close(a, b):
    return abs(a - b) <= TOL * max(1.0, abs(b))


def test_oracle_dp_vs_reference():
    g = _golden()
    for case in g["dp"]:
        ds, om = _oracle(case["case"])
        eps = case["epsilon"]
        for blk in case["necessary"]:
            for t, exp in zip(blk["triples"], blk["relevance"]):
                got = ko.dp_relevance(om, tuple(blk["pred"]), blk["perspective"], tuple(t), eps, "necessary")
                assert _close(float(got), exp), (blk["pred"], t, got, exp)
        for blk in case["sufficient"]:
            for t, exp in zip(blk["triples"], blk["relevance"]):
                got = ko.dp_relevance(om, tuple(blk["pred"]), blk["perspective"], tuple(t), eps, "sufficient",
                                      blk["entities_to_convert"])
                assert _close(float(got), exp), (blk["pred"], t, got, exp)


@pytest.mark.parametrize("name", ["transe_tiny", "conve60_tiny"])
def test_oracle_dp_unsupported_models_raise_like_reference(name):
    exp = next(c for c in _golden()["dp_unsupported"] if c["case"] == name)
    ds, om = _oracle(name)
    with pytest.raises(AttributeError) as ei:
        ko.dp_relevance(om, (0, 0, 1), "head", (0, 0, 1), 0.01, "necessary")
    assert exp["error"] == "AttributeError" and str(ei.value) == exp["message"]


def test_oracle_criage_vs_reference():
    g = _golden()
    for case in g["criage"]:
        ds, om = _oracle(case["case"])
        for blk in case["prefilter"]:
            assert [list(t) for t in ko.criage_prefilter(ds, tuple(blk["pred"]), blk["k"])] == blk["triples"]
        for mode in ("necessary", "sufficient"):
            for blk in case[mode]:
                for t, exp in zip(blk["triples"], blk["relevance"]):
                    got = ko.criage_relevance(om, ds, tuple(blk["pred"]), tuple(t), blk["perspective"], mode,
                                              blk.get("entities_to_convert"))
                    assert _close(float(got), exp), (case["case"], mode, blk["pred"], t, got, exp)


# ---------------------------------------------------------------------------- product engines
from engine_cases import build_product  # noqa: E402

import kelpie_amd.baselines as kb  # noqa: E402


def _check_dp(backend):
    g = _golden()
    for case in g["dp"]:
        rec, ds, model = build_product(case["case"], backend)
        eps = case["epsilon"]
        nec = kb.NecessaryDPEngine(model, ds, eps)
        for blk in case["necessary"]:
            got = nec.compute_relevance_batch(tuple(blk["pred"]), blk["perspective"], [tuple(t) for t in blk["triples"]])
            for t, v, exp in zip(blk["triples"], got, blk["relevance"]):
                assert isinstance(v, np.float32) and _close(float(v), exp), (blk["pred"], t, v, exp)
            one = nec.compute_relevance(tuple(blk["pred"]), blk["perspective"], tuple(blk["triples"][0]))
            assert one == got[0]
        suf = kb.SufficientDPEngine(model, ds, eps)
        for blk in case["sufficient"]:
            suf.entities_to_convert = blk["entities_to_convert"]
            got = suf.compute_relevance_batch(tuple(blk["pred"]), blk["perspective"], [tuple(t) for t in blk["triples"]])
            for t, v, exp in zip(blk["triples"], got, blk["relevance"]):
                assert _close(float(v), exp), (blk["pred"], t, v, exp)
    for exp in g["dp_unsupported"]:
        rec, ds, model = build_product(exp["case"], backend)
        with pytest.raises(AttributeError) as ei:
            kb.NecessaryDPEngine(model, ds, 0.01).compute_relevance((0, 0, 1), "head", (0, 0, 1))
        assert str(ei.value) == exp["message"]


def _check_criage(backend):
    g = _golden()
    for case in g["criage"]:
        rec, ds, model = build_product(case["case"], backend)
        pf = kb.CriagePreFilter(ds)
        for blk in case["prefilter"]:
            assert [list(t) for t in pf.select_triples(tuple(blk["pred"]), blk["k"])] == blk["triples"]
        nec = kb.NecessaryCriageEngine(model, ds)
        for blk in case["necessary"]:
            got = nec.compute_relevance_batch(tuple(blk["pred"]), [tuple(t) for t in blk["triples"]], blk["perspective"])
            for t, v, exp in zip(blk["triples"], got, blk["relevance"]):
                assert _close(v, exp), (case["case"], blk["pred"], t, v, exp)
        suf = kb.SufficientCriageEngine(model, ds)
        for blk in case["sufficient"]:
            suf.entities_to_convert = blk["entities_to_convert"]
            got = suf.compute_relevance_batch(tuple(blk["pred"]), [tuple(t) for t in blk["triples"]], blk["perspective"])
            for t, v, exp in zip(blk["triples"], got, blk["relevance"]):
                assert _close(v, exp), (case["case"], blk["pred"], t, v, exp)
    rec, ds, model = build_product("transe_tiny", backend)
    with pytest.raises(Exception, match="Criage does not support this model."):
        kb.NecessaryCriageEngine(model, ds)


def test_dp_engine_host_protocol_cpu():
    _check_dp("cpu")


def test_criage_engine_host_protocol_cpu():
    _check_criage("cpu")


@pytest.mark.gpu
def test_dp_engine_gpu_vs_reference_goldens():
    _check_dp("gpu")


@pytest.mark.gpu
def test_criage_engine_gpu_vs_reference_goldens():
    _check_criage("gpu")


def test_multi_equals_batch_cpu():
    g = _golden()
    case = g["criage"][0]
    rec, ds, model = build_product(case["case"], "cpu")
    nec = kb.NecessaryCriageEngine(model, ds)
    jobs = [(tuple(b["pred"]), [tuple(t) for t in b["triples"]]) for b in case["necessary"] if b["perspective"] == "tail"]
    multi = nec.compute_relevance_multi(jobs, "tail")
    for (p, ts), m in zip(jobs, multi):
        assert m == nec.compute_relevance_batch(p, ts, "tail")
    dcase = g["dp"][0]
    rec, ds, model = build_product(dcase["case"], "cpu")
    dp = kb.NecessaryDPEngine(model, ds, dcase["epsilon"])
    jobs = [(tuple(b["pred"]), [tuple(t) for t in b["triples"]]) for b in dcase["necessary"] if b["perspective"] == "head"]
    multi = dp.compute_relevance_multi(jobs, "head")
    for (p, ts), m in zip(jobs, multi):
        assert m == dp.compute_relevance_batch(p, "head", ts)


# ---------------------------------------------------------------------------- CRIAGE at production size
def _criage_fullrank(dim, backend):
    """A ComplEx model of dimension ``dim`` (D = 2 dim float64 systems: 400 pads to the
    blocked solver's 416 with an identity border, 320 needs none) whose perspective
    entity 0 has D + 60 tail triples, so H_0 has full rank; the engine's relevances
    against the oracle's (numpy.linalg.inv, as the reference): float64 solves of systems
    built in float32 (x = E_h * R_r, sigma(e . z)), whose dot products sum in another
    order on the device, so the systems differ in their last float32 bits: relative 1e-5."""
    rng = np.random.default_rng(dim)
    ne, nr, D = 700, 6, 2 * dim
    heads = rng.choice(np.arange(1, ne), size=D + 60, replace=False)
    train = np.array([(int(h), int(rng.integers(nr)), 0) for h in heads] +
                     [(int(rng.integers(1, ne)), int(rng.integers(nr)), int(rng.integers(1, ne))) for _ in range(400)])
    test = np.array([(int(heads[0]), 0, 0)])
    E = (0.3 * rng.standard_normal((ne, D))).astype(np.float32)
    R = (0.3 * rng.standard_normal((2 * nr, D))).astype(np.float32)
    ds = ka.Dataset(ne, nr, train, test[:0], test)
    model = ka.ComplEx(ds, E, R, init_scale=1e-3)
    if backend == "cpu":
        from cpu_backend import OracleBackedContext
        model._ctx = OracleBackedContext(model)
    om = ko.OracleModel("ComplEx", {"entity_embeddings": E, "relation_embeddings": R}, dim, {"init_scale": 1e-3})
    ods = ko.OracleDataset(ne, nr, train, test[:0], test)
    pred = (int(heads[1]), 1, 0)
    cands = [tuple(int(v) for v in t) for t in train[:12]]
    got = kb.NecessaryCriageEngine(model, ds).compute_relevance_batch(pred, cands, "tail")
    for t, v in zip(cands, got):
        exp = float(ko.criage_relevance(om, ods, pred, t, "tail", "necessary"))
        assert v is not None and abs(v - exp) <= 1e-5 * max(1e-3, abs(exp)), (dim, t, v, exp)


import kelpie_amd as ka  # noqa: E402


@pytest.mark.parametrize("dim", [200, 160])
def test_criage_fullrank_host_protocol_cpu(dim):
    _criage_fullrank(dim, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [200, 160])
def test_criage_fullrank_gpu_vs_oracle(dim):
    _criage_fullrank(dim, "gpu")

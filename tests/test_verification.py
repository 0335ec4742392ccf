"""f3, second half: explanation verification (src/verify_explanations.py) and its
metrics (src/compute_metrics.py) against the reference's own end-to-end runs
(tests/golden/verify_golden.json, tests/golden/make_verify_golden.py).

The retraining is a fresh model trained for three epochs (ComplEx: Adagrad + N3, and
Adam; TransE: Adam + margin ranking + L2; ConvE: Adam + BCE with label smoothing, the
three dropouts and train-mode batch norms, every layer trained), so the scores after it carry fp32
summation-order noise: new scores are compared to a
relative 1e-3 and new ranks to within one place; everything before the retraining
(the explained model's ranks, the edited triples, the JSON schema; its scores exactly on
the CPU stand-in, to fp32 summation order on the device) and the random protocol
(which rows each epoch visits) must match exactly."""
import json
import os

import numpy as np
import pytest

import kelpie_amd as ka
from kelpie_amd import verification as kv

from engine_cases import build_product

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "verify_golden.json")))
CASES = [(c, t, m) for c, g in GOLD["cases"].items() for t in g["training"] for m in ("necessary", "sufficient")]
TRAINERS = [(c, t) for c, g in GOLD["cases"].items() for t in g["training"]]


def _context_factory(backend):
    if backend == "cpu":
        from cpu_backend import OracleBackedContext
        return OracleBackedContext
    return None


def _check(backend, case, tname, mode):
    G = GOLD["cases"][case]
    rec, ds, model = build_product(case, backend)
    cfg = {"model": G["model"], "model_params": G["model_params"], "training": G["training"][tname]}
    got = kv.verify_explanations(G["explanations"][mode], ds, model, cfg, mode,
                                 context_factory=_context_factory(backend))
    exp = G["runs"][f"{tname}/{mode}"]
    assert len(got) == len(exp)

    def same(g, e):
        # before the retraining: the explained model's scores to fp32 summation order
        # (exact strings for ComplEx on the CPU stand-in; TransE's L2 norm there sums in
        # another order than torch.norm), ranks exact
        if backend == "cpu" and G["model"] == "ComplEx":
            assert g["score"] == e["score"]
        assert abs(float(g["score"]) - float(e["score"])) <= 1e-5 * max(1.0, abs(float(e["score"])))
        assert g["rank"] == e["rank"]
        ns, ne = float(g["new_score"]), float(e["new_score"])
        assert abs(ns - ne) <= 1e-3 * max(1.0, abs(ne)), (g, e)
        assert abs(int(g["new_rank"]) - int(e["new_rank"])) <= 1, (g, e)

    for g, e in zip(got, exp):
        assert [list(x) for x in [g["triple_to_explain"]]] == [e["triple_to_explain"]]
        if mode == "necessary":
            assert [list(t) for t in g["rule"]] == e["rule"]
            same(g, e)
        else:
            assert len(g["conversions"]) == len(e["conversions"])
            for gc, ec in zip(g["conversions"], e["conversions"]):
                assert [list(t) for t in gc["triples_to_add"]] == ec["triples_to_add"]
                same(gc, ec)
    m_got, m_exp = kv.compute_metrics(got, mode), kv.compute_metrics(exp, mode)
    assert m_got["mrr"] == m_exp["mrr"] and m_got["h1"] == m_exp["h1"]
    assert abs(m_got["new_mrr"] - m_exp["new_mrr"]) <= 0.01


def _check_direct(backend, case, tname):
    """The trainer alone: seed 42, a fresh model, optimizer.train on the training set."""
    G = GOLD["cases"][case]
    rec, ds, _ = build_product(case, "cpu")
    kv.set_seeds(42)
    m = kv.retrain(G["model"], ds, G["model_params"], G["training"][tname],
                   context_factory=_context_factory(backend))
    d = G["direct"][tname]
    E, R = m.entity_embeddings, m.relation_embeddings
    # ConvE: Adam divides by sqrt(v) + eps, so a row whose gradient is small in every step
    # moves by up to ~lr * g / eps on rounding-level gradient differences (measured for the
    # oracle trainer against the reference: 5e-5 on R row 0)
    atol = 1e-4 if G["model"] == "ConvE" else 1e-5
    assert np.allclose(E[:4], np.array(d["E_rows"]), rtol=1e-3, atol=atol)
    assert np.allclose(R[:2], np.array(d["R_rows"]), rtol=1e-3, atol=atol)
    assert abs(np.abs(E.astype(np.float64)).sum() - d["E_abs_sum"]) <= 1e-4 * d["E_abs_sum"]
    assert abs(np.abs(R.astype(np.float64)).sum() - d["R_abs_sum"]) <= 1e-4 * d["R_abs_sum"]
    if G["model"] == "ConvE":
        # the layers the BCEOptimizer trains with the tables, and the batch norms' running
        # statistics (momentum 0.1 over every train-mode batch)
        L, T = d["layers"], m.trained_layers
        c3 = 33 + E.shape[1]
        sl = {1: slice(0, 1), 2: slice(1, 33), 3: slice(33, c3)}
        assert abs(np.abs(T["conv_w"].astype(np.float64)).sum() - L["conv_w_abs_sum"]) <= 1e-4 * L["conv_w_abs_sum"]
        assert abs(np.abs(T["fc_w"].astype(np.float64)).sum() - L["fc_w_abs_sum"]) <= 1e-4 * L["fc_w_abs_sum"]
        assert np.allclose(T["fc_b"], L["fc_b"], rtol=1e-3, atol=1e-5)
        # the conv bias feeds a train-mode batch norm that subtracts it again: its exact
        # gradient is zero, so it (and BN2's running mean, which tracks it) walks on Adam's
        # normalised rounding residue; the oracle trainer lands within 1.1e-3 of the
        # reference, bounded here by lr (0.003); the bias minus the running mean, what eval
        # mode scores with, agrees to 4.4e-4
        lr0 = float(G["training"][tname]["lr"])
        assert np.allclose(T["conv_b"], L["conv_b"], rtol=0, atol=lr0)
        assert np.allclose(T["conv_b"] - T["bn_m"][sl[2]], np.array(L["conv_b"]) - L["bn2_running_mean"], rtol=0,
                           atol=lr0)
        for i in (1, 2, 3):
            for k, key in (("bn_w", "weight"), ("bn_b", "bias"), ("bn_m", "running_mean"), ("bn_v", "running_var")):
                tol = lr0 if (i, k) == (2, "bn_m") else 1e-4
                assert np.allclose(T[k][sl[i]], L[f"bn{i}_{key}"], rtol=1e-3, atol=tol), (i, key)


@pytest.mark.parametrize("case,tname", TRAINERS)
def test_oracle_trainer_vs_reference(case, tname):
    _check_direct("cpu", case, tname)


@pytest.mark.parametrize("case,tname,mode", CASES)
def test_verify_host_protocol_vs_reference(case, tname, mode):
    _check("cpu", case, tname, mode)


def test_compute_metrics_matches_reference_rounding():
    ev = [{"rank": "1", "new_rank": "3"}, {"rank": "4", "new_rank": "1"}, {"rank": "2", "new_rank": "2"}]
    m = kv.compute_metrics(ev, "necessary", explanations=[{"#relevances": 5}, {"#relevances": 7}])
    assert m == {"mrr": 0.583, "h1": 0.333, "new_mrr": 0.611, "new_h1": 0.333, "mrr_delta": 0.028,
                 "h1_delta": 0.0, "rels": 12}


def test_unsupported_models_raise():
    with pytest.raises(NotImplementedError):
        kv.retrain("DistMult", None, {}, {})


@pytest.mark.gpu
@pytest.mark.parametrize("case,tname", TRAINERS)
def test_device_trainer_vs_reference(case, tname):
    _check_direct("gpu", case, tname)


@pytest.mark.gpu
@pytest.mark.parametrize("case,tname,mode", CASES)
def test_verify_on_device_vs_reference(case, tname, mode):
    _check("gpu", case, tname, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("tname", ["adagrad_n3", "adam"])
def test_device_trainer_padded_rows(tname):
    """ComplEx dimension 12: rows of 24 floats stored at a 32-float stride, so the
    per-row gradient buffers have pad columns that the scatter sums into the table
    gradient (kp_train.hip kp_tr_rowgrads).  The device trainer must equal the oracle
    trainer and the tables stay finite."""
    from cpu_backend import OracleBackedContext
    G = GOLD["cases"]["complex_tiny"]
    _, ds, _ = build_product("complex_tiny", "cpu")
    mp = dict(G["model_params"], dimension=12)
    tr = G["training"][tname]
    kv.set_seeds(42)
    dev = kv.retrain("ComplEx", ds, mp, tr)
    kv.set_seeds(42)
    ref = kv.retrain("ComplEx", ds, mp, tr, context_factory=OracleBackedContext)
    assert np.isfinite(dev.entity_embeddings).all() and np.isfinite(dev.relation_embeddings).all()
    assert np.allclose(dev.entity_embeddings, ref.entity_embeddings, rtol=1e-3, atol=1e-5)
    assert np.allclose(dev.relation_embeddings, ref.relation_embeddings, rtol=1e-3, atol=1e-5)
    s = dev.ctx.all_scores(np.arange(4), np.zeros(4))
    assert np.isfinite(s).all()


@pytest.mark.gpu
@pytest.mark.parametrize("drop", [True, False])
def test_device_conve_trainer_matches_oracle_trainer(drop):
    """kp_conve_train_step against the oracle trainer (torch autograd on the CPU) for one
    epoch whose last batch holds a single pair (batch norms in eval mode for it), with
    and without the three dropouts (no noise drawn for rate 0)."""
    from cpu_backend import OracleBackedContext
    G = GOLD["cases"]["conve60_tiny"]
    _, ds, _ = build_product("conve60_tiny", "cpu")
    train = ds.training_triples
    stack = np.vstack([train, ds.invert_triples(train)])
    P = len({(int(h), int(r)) for h, r, _ in stack})
    bs = max(b for b in range(2, 400) if (P - 1) % b == 0 and b < P - 1)
    mp = dict(G["model_params"])
    if not drop:
        mp.update(input_dropout_rate=0.0, feature_map_dropout_rate=0.0, hidden_dropout_rate=0.0)
    tr = dict(G["training"]["bce"], batch_size=bs, epochs=1)
    kv.set_seeds(42)
    dev = kv.retrain("ConvE", ds, mp, tr)
    kv.set_seeds(42)
    ref = kv.retrain("ConvE", ds, mp, tr, context_factory=OracleBackedContext)
    assert P % bs == 1
    assert np.allclose(dev.entity_embeddings, ref.entity_embeddings, rtol=1e-3, atol=1e-4)
    assert np.allclose(dev.relation_embeddings, ref.relation_embeddings, rtol=1e-3, atol=1e-4)
    lr0 = float(tr["lr"])
    # biases that feed a train-mode batch norm directly have a zero exact gradient and
    # walk on rounding residue (see _check_direct): the conv bias always, the FC bias when
    # no hidden dropout sits between it and BN3; their running means track them
    # (and BN1's bias without input dropout: the unpadded conv turns it into a uniform
    # per-channel shift that BN2 removes)
    walk = ("conv_b", "bn_m") if drop else ("conv_b", "fc_b", "bn_m")
    for k in ("conv_w", "fc_w", "fc_b", "bn_w", "bn_b", "bn_v"):
        if k not in walk:
            a, b = dev.trained_layers[k], ref.trained_layers[k]
            if k == "bn_b" and not drop:
                assert abs(a[0] - b[0]) <= lr0
                a, b = a[1:], b[1:]
            assert np.allclose(a, b, rtol=1e-3, atol=1e-4), k
    for k in walk:
        assert np.allclose(dev.trained_layers[k], ref.trained_layers[k], rtol=0, atol=lr0), k

"""The library's host scheduler (csrc/kp_sched.cpp: kelpie view edits, rank filters and
the batch packing of TransE calls) against the Python KelpieView path it replaces
(kelpie_amd/data.py: removed / added / filter_for, the generic per-slot schedule).

Both paths run the same calls from the same generator states; the arrays they hand
to kp_posttrain_rank (x0, rows, draws, rank triples, filters) must be identical, and
the generator states after each batch equal.  Covers multi-triple rules, a triple
listed twice, self loops, training triples that are also validation / test triples,
sufficient-mode additions, and the three errors the reference's edits raise (a triple
without the entity: AssertionError, a triple that is not a training triple: KeyError,
a removal the filter cannot take: ValueError), with the draws made before each.
No GPU: the device call is replaced by a recorder."""
import numpy as np
import pytest
import torch

import kelpie_amd as ka
from kelpie_amd import models as kmodels

HP = {"batch_size": 64, "epochs": 3, "lr": 0.01, "margin": 2, "negative_triples_ratio": 2,
      "regularizer_weight": 0.0, "optimizer_name": "Adam", "regularizer_name": "L2"}


def _dataset():
    rng = np.random.default_rng(7)
    n_ent, n_rel = 40, 4
    trip = set()
    while len(trip) < 260:
        h, r, t = int(rng.integers(n_ent)), int(rng.integers(n_rel)), int(rng.integers(n_ent))
        trip.add((h, r, t))
    for e in (3, 5, 8):  # self loops of subjects used below
        trip.add((e, 1, e))
    train = sorted(trip)
    valid = [(3, 0, 11), (5, 2, 3), train[10]]
    test = [(8, 3, 3), (3, 1, 3), (5, 0, 5)]
    return ka.Dataset(n_ent, n_rel, np.array(train), np.array(valid), np.array(test))


def _run(ds, native, items, mode):
    w = np.random.default_rng(1).normal(size=(ds.num_entities, 16)).astype(np.float32)
    r = np.random.default_rng(2).normal(size=(ds.num_relations * 2, 16)).astype(np.float32)
    model = ka.TransE(ds, w, r)
    cls = ka.NecessaryPostTrainingEngine if mode == "necessary" else ka.SufficientPostTrainingEngine
    torch.manual_seed(5)
    np.random.seed(6)
    eng = cls(model, ds, HP)
    packs = []

    def run(slots, ctx=None):
        packs.append(eng._pack(slots))
        for s in slots:
            s.result = {"target_score": 0.5, "target_rank": 1}
        eng.last_batch_stats = {}
        return {}

    eng._run = run
    eng._collect = lambda slots, stats: None
    err = None
    try:
        for it in items:
            eng.set_cache()
            if mode == "sufficient":
                eng.compute_relevance_multi([(it[0], it[1], it[2])])
            else:
                eng.compute_relevance_multi([it])
    except Exception as e:  # noqa: BLE001
        err = e
    return packs, err, torch.get_rng_state().numpy().copy(), np.random.get_state()[1].copy()


def _both(monkeypatch, items, mode="necessary"):
    ds = _dataset()
    out = {}
    for native in (True, False):
        if not native:
            monkeypatch.setattr(kmodels.TransE, "fused_call_draws", property(lambda self: False))
        out[native] = _run(ds, native, items, mode)
    return out


def _assert_same(out):
    (pa, ea, ta, na), (pb, eb, tb, nb) = out[True], out[False]
    assert len(pa) == len(pb)
    for a, b in zip(pa, pb):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    assert type(ea) is type(eb) and (ea is None or ea.args == eb.args), (ea, eb)
    np.testing.assert_array_equal(ta, tb)
    np.testing.assert_array_equal(na, nb)


def _subject_triples(ds, e):
    return sorted(ds.entity_to_training_triples[e])


def test_native_necessary_matches_python(monkeypatch):
    ds = _dataset()
    items = []
    for e in (3, 5, 8, 12):
        tr = _subject_triples(ds, e)
        pred = tr[0]
        rules = [[t] for t in tr[:6]] + [tr[1:4], [tr[2], tr[2]] if False else [tr[2], tr[3]], []]
        items.append((pred, rules[:-1]))
    _assert_same(_both(monkeypatch, items))


def test_native_sufficient_matches_python(monkeypatch):
    ds = _dataset()
    items = []
    for e in (3, 5):
        tr = _subject_triples(ds, e)
        pred = tr[0]
        rules = [[t] for t in tr[1:4]] + [[tr[1], tr[2]]]
        items.append((pred, rules, [7, 9, 11]))
    _assert_same(_both(monkeypatch, items, "sufficient"))


@pytest.mark.parametrize("case", ["assert", "keyerror", "valueerror"])
def test_native_edit_errors_match_python(monkeypatch, case):
    ds = _dataset()
    tr = _subject_triples(ds, 3)
    pred = tr[0]
    good = [[t] for t in tr[1:4]]
    bad = {"assert": [(20, 0, 21)],                               # no subject
           "keyerror": [(3, 3, 39) if (3, 3, 39) not in tr else (3, 2, 38)],  # not a training triple
           "valueerror": [tr[1], tr[1]]}[case]                   # removed twice
    items = [(pred, good + [bad] + good)]
    out = _both(monkeypatch, items)
    assert out[True][1] is not None
    _assert_same(out)

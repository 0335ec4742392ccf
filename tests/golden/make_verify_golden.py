"""Reference goldens for explanation verification (f3: verify_explanations.py and
compute_metrics.py), development container only.

On the complex_tiny and transe_tiny graphs and weights of make_golden.py (300 entities,
2,400 training triples), with three explained predictions per mode, the reference's own
``verify_explanations.main`` runs end to end (its set_seeds(42), the original model's
init_random construction, the edited dataset, a fresh model trained by its optimizer's
train, predict_triples before and after) for the training configurations below
(ComplEx: Adagrad + N3, Adam; TransE: Adam + L2); its ``output_end_to_end.json`` is
recorded.
A direct training run (set_seeds(42), ComplEx(init_random=True), optimizer.train on
the unedited training set) records the trained tables, to pin the trainer itself.

    python tests/golden/make_verify_golden.py [case ...]   -> tests/golden/verify_golden.json
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import ref_harness  # noqa: E402
from make_golden import CASES, build_case  # noqa: E402

CASES_VERIFY = {
    "complex_tiny": {
        "model": "ComplEx",
        "model_params": {"dimension": 8, "init_scale": 1e-3},
        "training": {
            "adagrad_n3": {"optimizer_name": "Adagrad", "batch_size": 100, "epochs": 3, "lr": 0.1, "decay1": 0.9,
                           "decay2": 0.999, "regularizer_name": "N3", "regularizer_weight": 0.05},
            "adam": {"optimizer_name": "Adam", "batch_size": 128, "epochs": 3, "lr": 0.01, "decay1": 0.9,
                     "decay2": 0.999, "regularizer_name": "N3", "regularizer_weight": 0.0},
        },
    },
    "conve60_tiny": {
        "model": "ConvE",
        # the explained model's shape (make_golden.py), every dropout of the reference
        # configs switched on for the retraining (ConvE_*_training.json use 0.2 / 0.3 / 0.1-0.2)
        "model_params": {"dimension": 60, "input_dropout_rate": 0.2, "feature_map_dropout_rate": 0.3,
                         "hidden_dropout_rate": 0.2, "hidden_layer_size": 1216},
        "training": {
            "bce": {"batch_size": 256, "label_smoothing": 0.1, "lr": 0.003, "decay": 0.995, "epochs": 3},
        },
    },
    "transe_tiny": {
        "model": "TransE",
        "model_params": {"dimension": 16, "norm": 2},
        "training": {
            "adam_l2": {"batch_size": 512, "epochs": 3, "lr": 0.01, "margin": 5, "negative_triples_ratio": 5,
                        "regularizer_weight": 1.0},
        },
    },
    # the L1 score norm (TransEHyperParams.norm = 1, transe.py:46; tune.py:19 searches {1, 2})
    "transe_l1_tiny": {
        "model": "TransE",
        "model_params": {"dimension": 16, "norm": 1},
        "training": {
            "adam_l1": {"batch_size": 512, "epochs": 3, "lr": 0.01, "margin": 5, "negative_triples_ratio": 5,
                        "regularizer_weight": 1.0},
        },
    },
}


def explanations_for(dataset, g):
    """Three test predictions with a one- or two-triple best rule from the subject's
    training triples, and (sufficient) two conversion entities."""
    lab = dataset.labels_triple
    out_n, out_s = [], []
    deg = dataset.entity_to_degree
    picked = 0
    for t in g.test:
        s, p, o = (int(v) for v in t)
        tr = sorted(dataset.entity_to_training_triples.get(s, []))
        tr = [x for x in tr if x[0] == s]
        if len(tr) < 3 or picked >= 3:
            continue
        rule = tr[:1 + picked % 2]
        conv = [e for e in range(dataset.num_entities) if e != s and deg.get(e, 0) >= 2][3 * picked:3 * picked + 2]
        out_n.append({"triple": list(lab((s, p, o))), "rule_to_relevance": [[[list(lab(x)) for x in rule], 1.5]]})
        out_s.append({"triple": list(lab((s, p, o))), "entities_to_convert": [dataset.id_to_entity[e] for e in conv],
                      "rule_to_relevance": [[[list(lab(x)) for x in rule], 0.7]]})
        picked += 1
    return out_n, out_s


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


def run_case(src, name, spec, ver, MODEL_REGISTRY):
    g, w, dataset, model = build_case(src, name, CASES[name])
    out = {"model": spec["model"], "model_params": spec["model_params"], "training": spec["training"], "runs": {}}
    with tempfile.TemporaryDirectory() as tmp:
        pt = os.path.join(tmp, "model.pt")
        torch.save(model.state_dict(), pt)
        ex_n, ex_s = explanations_for(dataset, g)
        out["explanations"] = {"necessary": ex_n, "sufficient": ex_s}
        for tname, training in spec["training"].items():
            cfg = {"model": spec["model"], "model_path": pt, "model_params": spec["model_params"],
                   "training": training}
            cfg_path = os.path.join(tmp, f"{tname}.json")
            with open(cfg_path, "w") as f:
                json.dump(cfg, f)
            for mode, ex in (("necessary", ex_n), ("sufficient", ex_s)):
                d = os.path.join(tmp, f"{tname}_{mode}")
                os.makedirs(d)
                with open(os.path.join(d, "output.json"), "w") as f:
                    json.dump(ex, f)
                ver.main.callback(dataset=name, explanations_path=d, model_config=cfg_path, mode=mode)
                with open(os.path.join(d, "output_end_to_end.json")) as f:
                    out["runs"][f"{tname}/{mode}"] = json.load(f)
                print(name, tname, mode, json.dumps(out["runs"][f"{tname}/{mode}"])[:200], flush=True)
    # the trainer alone on the unedited training set
    from src.data import Dataset
    direct = {}
    for tname, training in spec["training"].items():
        ref_harness.seed_all(42)
        ds = Dataset(name)
        cls = MODEL_REGISTRY[spec["model"]]["class"]
        m = cls(dataset=ds, hp=cls.get_hyperparams_class()(**spec["model_params"]), init_random=True)
        opt_cls = MODEL_REGISTRY[spec["model"]]["optimizer"]
        opt = opt_cls(model=m, hp=opt_cls.get_hyperparams_class()(**training), verbose=False)
        opt.train(training_triples=ds.training_triples)
        E = m.entity_embeddings.detach().cpu().numpy()
        R = m.relation_embeddings.detach().cpu().numpy()
        direct[tname] = {"E_rows": E[:4].astype(np.float64).tolist(), "R_rows": R[:2].astype(np.float64).tolist(),
                         "E_abs_sum": float(np.abs(E.astype(np.float64)).sum()),
                         "R_abs_sum": float(np.abs(R.astype(np.float64)).sum()),
                         "E_sha256": digest(E), "R_sha256": digest(R)}
        if spec["model"] == "ConvE":
            # the frozen layers the retraining also trains, and the batch-norm running statistics
            f64 = lambda t: t.detach().cpu().numpy().astype(np.float64)  # noqa: E731
            direct[tname]["layers"] = {
                "conv_w_abs_sum": float(np.abs(f64(m.convolutional_layer.weight)).sum()),
                "conv_b": f64(m.convolutional_layer.bias).tolist(),
                "fc_w_abs_sum": float(np.abs(f64(m.hidden_layer.weight)).sum()),
                "fc_b": f64(m.hidden_layer.bias).tolist(),
                **{f"bn{i}_{k}": f64(getattr(bn, k)).tolist()
                   for i, bn in ((1, m.batch_norm_1), (2, m.batch_norm_2), (3, m.batch_norm_3))
                   for k in ("weight", "bias", "running_mean", "running_var")}}
    out["direct"] = direct
    return out


def main():
    src = ref_harness.load_reference()
    import src.verify_explanations as ver
    from src.link_prediction import MODEL_REGISTRY
    # utils.set_seeds (utils/utils.py:15-21) without its torch.cuda state touch: the
    # same three CPU seeds
    ver.set_seeds = ref_harness.seed_all
    path = os.path.join(HERE, "verify_golden.json")
    only = sys.argv[1:]  # case names to (re)generate; the others are kept as recorded
    out = {"cases": {}}
    if only and os.path.exists(path):
        with open(path) as f:
            out = json.load(f)
    for name, spec in CASES_VERIFY.items():
        if not only or name in only:
            out["cases"][name] = run_case(src, name, spec, ver, MODEL_REGISTRY)
    with open(path, "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()

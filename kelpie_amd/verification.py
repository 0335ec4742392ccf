"""End-to-end verification of explanations (``src/verify_explanations.py``): retrain
the model from scratch on the training set with the explanations removed (necessary)
or added for every conversion entity (sufficient), then compare the predictions.

The retraining runs on the device (``kp_train_epoch``, ``csrc/kp_train.hip``); the
host keeps the reference's random protocol (RNG-as-input): after ``set_seeds(42)``
the original model's ``init_random=True`` construction (verify_explanations.py:59,
its draws are consumed before ``load_state_dict``), the new model's initialisation
(complex.py:28-36: ``torch.rand`` tables scaled by ``init_scale``) and one
``torch.randperm`` per epoch (multiclass_nll_optimizer.py:102) come from the same
torch CPU generator, in that order (TransE: its xavier_normal_ tables and per epoch the
numpy shuffle and torch.randint negatives of pairwise_ranking_optimizer.py:102-118).
Supported: ComplEx with its MultiClassNLLOptimizer (Adagrad / Adam / SGD, N3),
TransE with its PairwiseRankingOptimizer (Adam, margin ranking, L2) and ConvE with its
BCEOptimizer (Adam on every layer, train-mode batch norms, the three dropouts; the
dropout noise is drawn here from the torch generator in the forward's order, the numpy
shuffle of the (head, relation) pairs once per epoch; ``kp_conve_train_step``,
``csrc/kp_train_conve.hip``).
"""
from __future__ import annotations

import random
from collections import defaultdict

import numpy as np
import torch

from .data import MANY_TO_ONE, ONE_TO_ONE, Dataset
from .models import ComplEx, ConvE, TransE


def set_seeds(seed: int = 42):
    """utils.set_seeds (src/utils/utils.py:16-21) for the CPU generators."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def _complex_init(dataset: Dataset, dimension: int, init_scale: float):
    """ComplEx(dataset, hp, init_random=True) tables (complex.py:28-36), float32."""
    D = 2 * int(dimension)
    E = torch.rand(dataset.num_entities, D)
    R = torch.rand(2 * dataset.num_relations, D)
    E *= init_scale
    R *= init_scale
    return E.numpy(), R.numpy()


def _transe_init(dataset: Dataset, dimension: int):
    """TransE(dataset, hp, init_random=True) tables (transe.py:26-33): torch.rand draws,
    then xavier_normal_ over each whole table."""
    E = torch.rand(dataset.num_entities, int(dimension))
    R = torch.rand(2 * dataset.num_relations, int(dimension))
    torch.nn.init.xavier_normal_(E)
    torch.nn.init.xavier_normal_(R)
    return E.numpy(), R.numpy()


def _conve_init(dataset: Dataset, model_params: dict):
    """ConvE(dataset, hp, init_random=True) (conve.py:23-61): the Conv2d(1, 32, 3x3) and
    Linear(hidden_layer_size, dimension) default initialisations, then the torch.rand
    tables and xavier_normal_ over each, all from the CPU generator in that order."""
    d, hidden = int(model_params["dimension"]), int(model_params["hidden_layer_size"])
    conv = torch.nn.Conv2d(1, 32, (3, 3), 1, 0, bias=True)
    fc = torch.nn.Linear(hidden, d)
    E = torch.rand(dataset.num_entities, d)
    R = torch.rand(2 * dataset.num_relations, d)
    torch.nn.init.xavier_normal_(E)
    torch.nn.init.xavier_normal_(R)
    f = lambda t: t.detach().numpy().copy()  # noqa: E731
    return E.numpy(), R.numpy(), {"conv_w": f(conv.weight).reshape(32, 3, 3), "conv_b": f(conv.bias),
                                  "fc_w": f(fc.weight), "fc_b": f(fc.bias)}


def model_init(model_name: str, dataset: Dataset, model_params: dict):
    """The parameters of ``MODEL_REGISTRY[model_name](dataset, hp, init_random=True)``:
    (E, R) for ComplEx / TransE, (E, R, layers) for ConvE."""
    if model_name == "ComplEx":
        return _complex_init(dataset, model_params["dimension"], model_params["init_scale"])
    if model_name == "TransE":
        return _transe_init(dataset, model_params["dimension"])
    if model_name == "ConvE":
        return _conve_init(dataset, model_params)
    raise NotImplementedError(f"device retraining supports ComplEx, TransE and ConvE, not {model_name}")


def _dropout_noise(shape, p: float):
    """nn.Dropout / nn.Dropout2d's CPU multiplier (torch _dropout_impl): nothing drawn for
    p == 0, zeros for p == 1, else ``empty(shape).bernoulli_(1 - p).div_(1 - p)``."""
    if p == 0:
        return None
    if p == 1:
        return np.zeros(shape, np.float32)
    return torch.empty(shape).bernoulli_(1 - p).div_(1 - p).numpy()


def _retrain_conve(dataset: Dataset, model_params: dict, training: dict, device, context_factory):
    """BCEOptimizer.train (bce_optimizer.py:45-150) for a fresh ConvE on the device."""
    E, R, L = _conve_init(dataset, model_params)
    d = E.shape[1]
    h = d // 20
    model = ConvE(dataset, E, R, L["conv_w"], L["conv_b"], L["fc_w"], L["fc_b"], device=device)
    if context_factory is not None:
        model._ctx = context_factory(model)
    ctx = model.ctx
    c3 = 33 + d
    ctx.conve_train_begin(np.ones(c3, np.float32), np.zeros(c3, np.float32), np.zeros(c3, np.float32),
                          np.ones(c3, np.float32))
    train = dataset.training_triples
    stack = np.vstack([train, dataset.invert_triples(train)]).astype(np.int64)
    # extract_er_vocab: (head, relation) keys in first-occurrence order, tails in row order
    keys, inv = np.unique(stack[:, 0] * (2 * dataset.num_relations) + stack[:, 1], return_inverse=True)
    first = np.full(len(keys), len(stack), np.int64)
    np.minimum.at(first, inv, np.arange(len(stack)))
    key_order = np.argsort(first, kind="stable")  # pair index -> key index
    rank_of_key = np.empty(len(keys), np.int64)
    rank_of_key[key_order] = np.arange(len(keys))
    pair_of_row = rank_of_key[inv]
    by_pair = np.argsort(pair_of_row, kind="stable")
    counts = np.bincount(pair_of_row, minlength=len(keys))
    off = np.concatenate([[0], np.cumsum(counts)])
    tails_sorted = stack[by_pair, 2].astype(np.int32)
    pairs = stack[by_pair[off[:-1]], :2].astype(np.int32)  # [P][2] in er_vocab order
    P = len(pairs)
    order = np.arange(P)
    bs = int(training["batch_size"])
    ls = float(training["label_smoothing"])
    lr, decay = float(training["lr"]), float(training["decay"])
    pin = float(model_params["input_dropout_rate"])
    pfm = float(model_params["feature_map_dropout_rate"])
    phid = float(model_params["hidden_dropout_rate"])
    for _ in range(int(training["epochs"])):
        np.random.shuffle(order)  # the in-place shuffle of er_vocab_pairs, epoch after epoch
        for b0 in range(0, P, bs):
            idx = order[b0:b0 + bs]
            B = len(idx)
            cnt = counts[idx]
            toff = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
            tails = np.concatenate([tails_sorted[off[i]:off[i + 1]] for i in idx]) if B else np.zeros(0, np.int32)
            nin = _dropout_noise((B, 1, 40, h), pin)
            nfm = _dropout_noise((B, 32, 1, 1), pfm)
            nhid = _dropout_noise((B, d), phid)
            ctx.conve_train_step(pairs[idx], toff, tails, nin, nfm, nhid, lr, ls, B > 1)
        if decay:
            lr = lr * decay  # ExponentialLR.step
    E2, R2 = ctx.read_tables(2 * dataset.num_relations)
    T = ctx.conve_train_read()
    sl = [(0, 1), (1, 33), (33, c3)]
    bn = {i + 1: {"weight": T["bn_w"][a:b], "bias": T["bn_b"][a:b], "running_mean": T["bn_m"][a:b],
                  "running_var": T["bn_v"][a:b]} for i, (a, b) in enumerate(sl)}
    out = ConvE(dataset, E2, R2, T["conv_w"].reshape(32, 3, 3), T["conv_b"], T["fc_w"], T["fc_b"], bn=bn,
                device=device)
    if context_factory is not None:
        out._ctx = context_factory(out)
    out.trained_layers = T
    return out


def _transe_epoch_rows(stack: np.ndarray, ratio: int, n_entities: int):
    """PairwiseRankingOptimizer.epoch's draws and rows (pairwise_ranking_optimizer.py:102-118):
    the in-place shuffle of the stack, randint(2) then randint(N) over ratio * n, and of
    the repeated rows the first n, i.e. row i of the batch loop is stack[i // ratio]."""
    np.random.shuffle(stack)
    n = len(stack)
    size = (n * ratio,)
    head_or_tail = torch.randint(high=2, size=size).numpy()[:n]
    ents = torch.randint(high=n_entities, size=size).numpy()[:n]
    pos = stack[np.arange(n) // ratio]
    neg = pos.copy()
    mh = head_or_tail == 1
    neg[mh, 0] = ents[mh]
    neg[~mh, 2] = ents[~mh]
    return pos.astype(np.int32), neg.astype(np.int32)


def retrain(model_name: str, dataset: Dataset, model_params: dict, training: dict, device: int = 0,
            context_factory=None):
    """A fresh model (``init_random=True``) trained by its optimizer on
    ``dataset.training_triples`` (``optimizer.train``: multiclass_nll_optimizer.py:57-99,
    pairwise_ranking_optimizer.py:55-100), on the device.  Consumes the torch / numpy
    generators like the reference.  ``context_factory(model)``, if given, supplies the
    model's context (tests)."""
    if model_name == "ConvE":
        return _retrain_conve(dataset, model_params, training, device, context_factory)
    E, R = model_init(model_name, dataset, model_params)
    if model_name == "ComplEx":
        model = ComplEx(dataset, E, R, init_scale=model_params["init_scale"], device=device)
    else:
        model = TransE(dataset, E, R, norm=model_params.get("norm", 2), device=device)
    if context_factory is not None:
        model._ctx = context_factory(model)
    hp = model.kp_hp(training)
    train = dataset.training_triples
    stack = np.vstack([train, dataset.invert_triples(train)])
    ctx = model.ctx
    for epoch in range(int(training["epochs"])):
        if model_name == "ComplEx":
            perm = torch.randperm(stack.shape[0]).numpy()
            ctx.train_epoch(hp, stack.astype(np.int32), perm, epoch)
        else:
            pos, neg = _transe_epoch_rows(stack, int(training["negative_triples_ratio"]), dataset.num_entities)
            ctx.train_epoch(hp, pos, neg, epoch)
    E2, R2 = ctx.read_tables(2 * dataset.num_relations)
    model.entity_embeddings, model.relation_embeddings = E2, R2
    return model


def _fmt(score) -> str:
    """str() of the reference's float32 numpy score (verify_explanations.py:190-193)."""
    return str(np.float32(score))


def _best_rule(explanation, dataset):
    tmp = explanation["rule_to_relevance"][0]
    best = tmp[1] if len(tmp) == 3 else tmp[0]
    return [dataset.ids_triple(t) for t in best]


def verify_explanations(explanations: list, dataset: Dataset, model, model_config: dict, mode: str,
                        device: int = 0, context_factory=None) -> list:
    """``verify_explanations.main`` (verify_explanations.py:42-268) after its file loading:
    ``explanations`` is the pipeline's ``output.json`` list, ``model`` the trained
    model being explained, ``model_config`` the reference config (``model``,
    ``model_params``, ``training``).  Returns the ``output_end_to_end.json`` list."""
    if mode not in ("necessary", "sufficient"):
        raise ValueError(mode)
    name = model_config["model"]
    if name not in ("ComplEx", "TransE", "ConvE"):
        raise NotImplementedError(f"device retraining supports ComplEx, TransE and ConvE, not {name}")
    set_seeds(42)
    # the original model's init_random=True construction (verify_explanations.py:59)
    model_init(name, dataset, model_config["model_params"])
    preds = []
    if mode == "sufficient":
        convert_set, best = {}, {}
        for ex in explanations:
            pred = dataset.ids_triple(ex["triple"])
            preds.append(pred)
            convert_set[pred] = [dataset.entity_to_id[e] for e in ex["entities_to_convert"]]
            best[pred] = _best_rule(ex, dataset)
        to_add, to_convert, added_for = [], [], {}
        for pred in preds:
            s = pred[0]
            cur = []
            for e in convert_set[pred]:
                tc = Dataset.replace_entity_in_triple(pred, s, e)
                cur.append(tc)
                adds = Dataset.replace_entity_in_triples(best[pred], s, e)
                to_add.extend(adds)
                added_for[tc] = adds
            to_convert.extend(cur)
            convert_set[pred] = cur
        new_ds = dataset.copy()
        for s, p, o in to_add:
            if new_ds.relation_to_type[p] in (MANY_TO_ONE, ONE_TO_ONE):
                # iterates the list it removes from, like the reference (:114-116)
                for existing_o in new_ds.train_to_filter[(s, p)]:
                    new_ds.remove_training_triple((s, p, existing_o))
        new_ds.add_training_triples(to_add)
        results = dict(zip(to_convert, model.predict_triples(np.array(to_convert))))
        new_model = retrain(name, new_ds, model_config["model_params"], model_config["training"], device,
                            context_factory)
        new_results = dict(zip(to_convert, new_model.predict_triples(np.array(to_convert))))
        evaluations = []
        for pred in preds:
            conversions = []
            for tc in convert_set[pred]:
                r, nr = results[tc], new_results[tc]
                conversions.append({
                    "triples_to_add": [dataset.labels_triple(t) for t in added_for[tc]],
                    "score": _fmt(r["score"]["tail"]), "rank": str(r["rank"]["tail"]),
                    "new_score": _fmt(nr["score"]["tail"]), "new_rank": str(nr["rank"]["tail"]),
                })
            evaluations.append({"triple_to_explain": dataset.labels_triple(pred), "conversions": conversions})
        return evaluations
    best = defaultdict(list)
    for ex in explanations:
        pred = dataset.ids_triple(ex["triple"])
        preds.append(pred)
        best[pred] = _best_rule(ex, dataset)
    to_remove = []
    for pred in preds:
        to_remove += best[pred]
    new_ds = dataset.copy()
    new_ds.remove_training_triples(to_remove)
    results = dict(zip(preds, model.predict_triples(np.array(preds))))
    new_model = retrain(name, new_ds, model_config["model_params"], model_config["training"], device,
                            context_factory)
    new_results = dict(zip(preds, new_model.predict_triples(np.array(preds))))
    evaluations = []
    for pred in preds:
        r, nr = results[pred], new_results[pred]
        evaluations.append({
            "triple_to_explain": dataset.labels_triple(pred),
            "rule": [dataset.labels_triple(t) for t in best[pred]],
            "score": _fmt(r["score"]["tail"]), "rank": str(r["rank"]["tail"]),
            "new_score": _fmt(nr["score"]["tail"]), "new_rank": str(nr["rank"]["tail"]),
        })
    return evaluations


def compute_metrics(evaluations: list, mode: str, explanations: list | None = None) -> dict:
    """``compute_metrics.main`` (compute_metrics.py:27-85): MRR and H@1 of the explained
    predictions before and after the retraining, their deltas (each rounded to 3
    decimals, the deltas of the rounded values), and ``rels`` = the summed
    ``#relevances`` of ``output.json`` when ``explanations`` is given."""
    def hits1(ranks):
        return round(sum(1.0 for r in ranks if r <= 1) / float(len(ranks)), 3)

    def mrr(ranks):
        acc = 0.0
        for r in ranks:
            acc += 1.0 / float(r)
        return round(acc / float(len(ranks)), 3)

    if mode == "necessary":
        ranks = [float(d["rank"]) for d in evaluations]
        new_ranks = [float(d["new_rank"]) for d in evaluations]
    else:
        ranks = [float(c["rank"]) for d in evaluations for c in d["conversions"]]
        new_ranks = [float(c["new_rank"]) for d in evaluations for c in d["conversions"]]
    out = {"mrr": mrr(ranks), "h1": hits1(ranks), "new_mrr": mrr(new_ranks), "new_h1": hits1(new_ranks)}
    out["mrr_delta"] = round(out["new_mrr"] - out["mrr"], 3)
    out["h1_delta"] = round(out["new_h1"] - out["h1"], 3)
    if explanations is not None:
        out["rels"] = sum(x["#relevances"] for x in explanations)
    return out

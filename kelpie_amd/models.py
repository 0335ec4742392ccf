"""Frozen link-prediction models as seen by the relevance engine.

These classes keep the reference ``Model`` surface the engine uses
(``name``, ``dimension``, ``is_minimizer()``, ``all_scores(triples)``,
``MODEL_REGISTRY``; src/link_prediction/models/model.py:8-78,
src/link_prediction/__init__.py:5-9) and hold the HIP context with the
frozen tables.  The per-candidate ``Kelpie*`` model construction of the
reference (transe.py:84-99, complex.py:144-159, conve.py:193-237) is reduced
to the kelpie-row initialisation below plus the RNG it consumes; the tables
themselves are never cloned.
"""
from __future__ import annotations

import math

import numpy as np

from . import _lib
from .rng import ReferenceRNG


class FrozenModel:
    name = "?"

    def __init__(self, dataset, entity_embeddings, relation_embeddings, device=0):
        self.dataset = dataset
        self.entity_embeddings = np.ascontiguousarray(entity_embeddings, dtype=np.float32)
        self.relation_embeddings = np.ascontiguousarray(relation_embeddings, dtype=np.float32)
        assert self.entity_embeddings.shape[0] == dataset.num_entities
        assert self.relation_embeddings.shape[0] == 2 * dataset.num_relations
        self.device = device
        self._ctx = None

    # ------------------------------------------------------------ reference surface
    @property
    def dimension(self):
        return self.entity_embeddings.shape[1]

    def is_minimizer(self):
        return False

    def eval(self):
        return self

    @property
    def ctx(self) -> _lib.Context:
        if self._ctx is None:
            self._ctx = self._make_ctx()
        return self._ctx

    def _make_ctx(self):
        return _lib.Context(self.name, self.entity_embeddings, self.relation_embeddings, device=self.device)

    def contexts(self, n: int) -> list:
        """``n`` device contexts over replicas of the frozen tables (the first is
        :attr:`ctx`), for batches in flight at once; a stand-in context (tests) is
        never replicated."""
        if not isinstance(self.ctx, _lib.Context):
            return [self.ctx]
        extra = self.__dict__.setdefault("_ctx_extra", [])
        while len(extra) < n - 1:
            extra.append(self._make_ctx())
        return [self.ctx] + extra[:n - 1]

    def all_scores(self, triples):
        """``Model.all_scores`` over the frozen entities (model.py:19): float32 [B, |E|]."""
        t = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
        return self.ctx.all_scores(t[:, 0], t[:, 1])

    def predict_tails(self, triples):
        """``Model.predict_tails`` (model.py:42-68; ConvE conve.py:160-184): target
        scores and filtered ranks against ``dataset.to_filter``, on the device."""
        t = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
        flt = [self.dataset.to_filter.get((int(h), int(r)), []) for h, r, _ in t.tolist()]
        off = np.zeros(len(t) + 1, np.int32)
        off[1:] = np.cumsum([len(f) for f in flt])
        filt = np.array([e for f in flt for e in f], np.int32)
        score, rank = self.ctx.predict_tails(t, off, filt)
        return [float(x) for x in score], [int(x) for x in rank]

    def predict_triples(self, triples):
        """``Model.predict_triples`` (model.py:25-40): tail prediction on the triples,
        head prediction on their inverses."""
        direct = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
        assert np.all(direct[:, 1] < self.dataset.num_relations)
        direct_scores, tail_ranks = self.predict_tails(direct)
        inverse_scores, head_ranks = self.predict_tails(self.dataset.invert_triples(direct))
        return [{"score": {"tail": direct_scores[i], "head": inverse_scores[i]},
                 "rank": {"tail": int(tail_ranks[i]), "head": int(head_ranks[i])}} for i in range(len(direct))]

    # ------------------------------------------------------------ kelpie hooks
    def kelpie_init(self, init: np.ndarray, rng: ReferenceRNG) -> np.ndarray:
        raise NotImplementedError

    def kp_hp(self, hp: dict) -> _lib.HP:
        raise NotImplementedError

    def posttrain_draws(self, rows: np.ndarray, hp: dict, rng: ReferenceRNG) -> np.ndarray:
        """Random draws of one post-training over ``rows`` (kelpie rows + inverses)."""
        raise NotImplementedError

    # Slots another rank post-trains (kelpie_amd.distributed): consume the same draws
    # without producing what only the post-training needs.  The defaults make the draws
    # and drop them; models override with a bare generator advance where they can.
    skip_needs_rows = True  # posttrain_skip needs the edited rows, not only their count

    def kelpie_skip(self, rng: ReferenceRNG):
        """The draws of a KelpieModel construction (kelpie_init) whose row is not needed."""
        self.kelpie_init(np.zeros(self.dimension, np.float32), rng)

    def posttrain_skip(self, rows, n_rows: int, hp: dict, rng: ReferenceRNG):
        self.posttrain_draws(rows, hp, rng)


class ComplEx(FrozenModel):
    """ComplEx (complex.py:17-142): rows [Re | Im], maximizer."""

    name = "ComplEx"

    def __init__(self, dataset, entity_embeddings, relation_embeddings, init_scale=1e-3, device=0):
        super().__init__(dataset, entity_embeddings, relation_embeddings, device)
        assert self.dimension % 2 == 0
        self.real_dimension = self.dimension // 2
        self.init_scale = float(init_scale)

    def kelpie_init(self, init, rng):
        # KelpieComplEx: Parameter(init.cuda()) *= init_scale (complex.py:155-157), float32
        return (init.astype(np.float32) * np.float32(self.init_scale)).astype(np.float32)

    def kp_hp(self, hp):
        name = hp["optimizer_name"]
        if name not in _lib.KP_OPT:
            raise ValueError(f"unknown optimizer {name}")
        reg = hp.get("regularizer_name", "N3")
        if reg not in _lib.KP_REG:  # multiclass_nll_optimizer.py:45-48: {"N3", "N2"}[name]
            raise KeyError(reg)
        return _lib.HP(optimizer=_lib.KP_OPT[name], epochs=int(hp["epochs"]), batch_size=int(hp["batch_size"]),
                       lr=float(hp["lr"]), beta1=float(hp.get("decay1", 0.9)), beta2=float(hp.get("decay2", 0.999)),
                       eps=1e-10 if name == "Adagrad" else 1e-8, reg_weight=float(hp.get("regularizer_weight", 0.0)),
                       reg_kind=_lib.KP_REG[reg])

    def posttrain_draws(self, rows, hp, rng):
        return rng.complex_epochs(len(rows), int(hp["epochs"]), int(hp["batch_size"]))

    skip_needs_rows = False

    def kelpie_skip(self, rng):
        pass  # KelpieComplEx draws nothing at construction

    def posttrain_skip(self, rows, n_rows, hp, rng):
        rng.complex_epochs(int(n_rows), int(hp["epochs"]), int(hp["batch_size"]), want=False)


class TransE(FrozenModel):
    """TransE (transe.py:17-82): L_p distance (p = ``norm``, 2 or 1: transe.py:46,
    tune.py:19), minimizer."""

    name = "TransE"

    def __init__(self, dataset, entity_embeddings, relation_embeddings, norm=2, device=0):
        super().__init__(dataset, entity_embeddings, relation_embeddings, device)
        if int(norm) not in (1, 2):
            raise ValueError(f"TransE: norm must be 1 or 2, got {norm!r}")
        self.norm = int(norm)

    def _make_ctx(self):
        return _lib.Context(self.name, self.entity_embeddings, self.relation_embeddings, device=self.device,
                            norm_p=self.norm)

    def is_minimizer(self):
        return True

    def kelpie_init(self, init, rng):
        # KelpieTransE: xavier_normal_ overwrites the init copy (transe.py:93-95)
        return rng.xavier_row(self.dimension)

    @property
    def fused_call_draws(self):
        """Every draw of a compute_relevance call can come from one library call
        (ReferenceRNG.transe_call): its normal_ replica needs rows of >= 16 values."""
        return self.dimension >= 16

    def kp_hp(self, hp):
        return _lib.HP(optimizer=_lib.KP_OPT["Adam"], epochs=int(hp["epochs"]), batch_size=int(hp["batch_size"]),
                       lr=float(hp["lr"]), beta1=0.9, beta2=0.999, eps=1e-8,
                       reg_weight=float(hp["regularizer_weight"]), margin=float(hp["margin"]),
                       neg_ratio=int(hp["negative_triples_ratio"]))

    def posttrain_draws(self, rows, hp, rng):
        return rng.transe_epochs(len(rows), int(hp["epochs"]), int(hp["negative_triples_ratio"]),
                                 self.dataset.num_entities + 1)


class ConvE(FrozenModel):
    """ConvE (conve.py:23-191): 20 x (d/20) images, 32 3x3 filters, sigmoid scores."""

    name = "ConvE"

    def __init__(self, dataset, entity_embeddings, relation_embeddings, conv_weight, conv_bias, fc_weight, fc_bias,
                 bn=None, input_dropout_rate=0.0, feature_map_dropout_rate=0.0, hidden_dropout_rate=0.0, device=0):
        super().__init__(dataset, entity_embeddings, relation_embeddings, device)
        d = self.dimension
        if d % 20 or d // 20 < 3:
            raise ValueError("ConvE dimension must be 20*h with h >= 3")
        for rate in (input_dropout_rate, feature_map_dropout_rate, hidden_dropout_rate):
            if not 0.0 <= float(rate) <= 1.0:
                raise ValueError(f"dropout probability has to be between 0 and 1, but got {rate}")
        self.hidden_layer_size = 32 * 38 * (d // 20 - 2)
        self.conv_weight = np.asarray(conv_weight, np.float32).reshape(32, 3, 3)
        self.conv_bias = np.asarray(conv_bias, np.float32).reshape(32)
        self.fc_weight = np.asarray(fc_weight, np.float32).reshape(d, self.hidden_layer_size)
        self.fc_bias = np.asarray(fc_bias, np.float32).reshape(d)
        # the three dropouts stay in train mode during post-training (model.py:114-125)
        self.input_dropout_rate = float(input_dropout_rate)
        self.feature_map_dropout_rate = float(feature_map_dropout_rate)
        self.hidden_dropout_rate = float(hidden_dropout_rate)
        alpha, beta = [], []
        for i, c in ((1, 1), (2, 32), (3, d)):
            b = (bn or {}).get(i, {})
            w = np.asarray(b.get("weight", np.ones(c)), np.float32)
            bias = np.asarray(b.get("bias", np.zeros(c)), np.float32)
            mean = np.asarray(b.get("running_mean", np.zeros(c)), np.float32)
            var = np.asarray(b.get("running_var", np.ones(c)), np.float32)
            inv = (1.0 / np.sqrt(var.astype(np.float64) + 1e-5)).astype(np.float32)
            a = (inv * w).astype(np.float32)
            alpha.append(a)
            beta.append((bias - mean * a).astype(np.float32))
        self.bn_alpha = np.concatenate(alpha)
        self.bn_beta = np.concatenate(beta)

    def _make_ctx(self):
        return _lib.Context("ConvE", self.entity_embeddings, self.relation_embeddings, device=self.device,
                            conve={"conv_w": self.conv_weight, "conv_b": self.conv_bias, "fc_w": self.fc_weight,
                                   "fc_b": self.fc_bias, "bn_alpha": self.bn_alpha, "bn_beta": self.bn_beta})

    def kelpie_init(self, init, rng):
        rng.conve_construction(self.hidden_layer_size, self.dimension)
        return init.astype(np.float32).copy()

    def kp_hp(self, hp):
        return _lib.HP(optimizer=_lib.KP_OPT["Adam"], epochs=int(hp["epochs"]), batch_size=int(hp["batch_size"]),
                       lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, label_smoothing=float(hp["label_smoothing"]),
                       hidden_dropout=self.hidden_dropout_rate, input_dropout=self.input_dropout_rate,
                       fmap_dropout=self.feature_map_dropout_rate)

    def er_vocab_sizes(self, rows: np.ndarray, batch_size: int, epochs: int):
        # the distinct (head, relation) pairs of the rows (BCEOptimizer's er_vocab keys)
        rows = np.asarray(rows, dtype=np.int64).reshape(-1, 3)
        P = int(np.unique(rows[:, 0] * (int(rows[:, 1].max()) + 1) + rows[:, 1]).size) if len(rows) else 0
        per_epoch = [min(batch_size, P - s) for s in range(0, P, batch_size)]
        return per_epoch * epochs

    def dropout_segments(self):
        """(elements per pair, rate) of each dropout in the forward's draw order: the
        input dropout over the stacked 40 x (d/20) image, the feature-map Dropout2d over
        the 32 channels, the hidden dropout over d (conve.py:142,147,151)."""
        return [(2 * self.dimension, self.input_dropout_rate), (32, self.feature_map_dropout_rate),
                (self.dimension, self.hidden_dropout_rate)]

    def posttrain_draws(self, rows, hp, rng):
        steps = self.er_vocab_sizes(rows, int(hp["batch_size"]), int(hp["epochs"]))
        return rng.conve_masks(steps, self.dropout_segments())

    def kelpie_skip(self, rng):
        rng.conve_construction(self.hidden_layer_size, self.dimension)

    def posttrain_skip(self, rows, n_rows, hp, rng):
        # bernoulli_: one random64 (two outputs) per element; rate 0 and rate 1 draw nothing
        per_pair = sum(n for n, p in self.dropout_segments() if 0.0 < p < 1.0)
        if per_pair:
            steps = self.er_vocab_sizes(rows, int(hp["batch_size"]), int(hp["epochs"]))
            rng.discard(2 * per_pair * int(sum(steps)))


MODEL_REGISTRY = {"ComplEx": ComplEx, "TransE": TransE, "ConvE": ConvE}


def from_state_dict(name, dataset, state, model_params, device=0):
    """Build a frozen model from a reference checkpoint state dict (``torch.save(
    model.state_dict())``, pairwise_ranking_optimizer.py:96-98 etc.), loaded by
    the caller with ``torch.load(path, weights_only=True)``."""

    def arr(k):
        v = state[k]
        return v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)

    from .hparams import model_params as _validated
    model_params = _validated(name, model_params)  # explain.py:169-170, the reference's hp class
    E, R = arr("entity_embeddings"), arr("relation_embeddings")
    if name == "ComplEx":
        return ComplEx(dataset, E, R, init_scale=model_params.get("init_scale", 1e-3), device=device)
    if name == "TransE":
        return TransE(dataset, E, R, norm=model_params.get("norm", 2), device=device)
    if name == "ConvE":
        bn = {}
        for i in (1, 2, 3):
            bn[i] = {k: arr(f"batch_norm_{i}.{k}") for k in ("weight", "bias", "running_mean", "running_var")}
        return ConvE(dataset, E, R, arr("convolutional_layer.weight"), arr("convolutional_layer.bias"),
                     arr("hidden_layer.weight"), arr("hidden_layer.bias"), bn=bn,
                     input_dropout_rate=model_params.get("input_dropout_rate", 0.0),
                     feature_map_dropout_rate=model_params.get("feature_map_dropout_rate", 0.0),
                     hidden_dropout_rate=model_params.get("hidden_dropout_rate", 0.0), device=device)
    raise ValueError(name)

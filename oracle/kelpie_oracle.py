"""CPU restatement of the Kelpie relevance-engine hot path (TEST INFRASTRUCTURE).

This module is the parity ORACLE.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker /
the timed CPU baseline; the product package ``kelpie_amd`` never imports it.

It restates, in plain numpy (float32 arrays, the dtype the reference trains
in) plus the torch CPU generator for the random draws, the reference's
post-training relevance path:

* dataset indices and filters ............ ``src/data/dataset.py:104-141,319-352``
* per-entity kelpie view ................. ``src/data/kelpie_dataset.py:10-203``
* engine, relevance formulas, rank ....... ``src/relevance_engines/post_training_engine.py:17-207``
* conversion-entity selection ............ ``src/relevance_engines/engine.py:22-126``
* TransE / ComplEx / ConvE scorers ....... ``src/link_prediction/models/{transe,complex,conve}.py``
* Kelpie optimizers (one trainable row) .. ``src/link_prediction/optimization/*.py``
* stochastic explanation builder ......... ``src/explanation_builders/stochastic_builder.py:33-192``

Gradients are the hand-derived single-row gradients of SURVEY.md Appendix C,
computed from the FULL score matrices (no algebraic shortcuts), so the oracle
is an independent check of the decompositions the HIP kernels use.

Parity pinning: every function here is checked against golden vectors that
``tests/golden/make_golden.py`` captured by running the reference itself
(CPU-redirected import) in the development container; see
``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math
import random
from collections import Counter, OrderedDict, defaultdict
from itertools import combinations

import numpy as np
import torch

ONE_TO_ONE, ONE_TO_MANY, MANY_TO_ONE, MANY_TO_MANY = "1-1", "1-N", "N-1", "N-N"
F32 = np.float32


# =============================================================================
# data layer
# =============================================================================
class OracleDataset:
    """Index / filter semantics of ``Dataset.__init__`` (dataset.py:104-141)."""

    def __init__(self, num_entities, num_relations, train, valid, test):
        self.num_entities = int(num_entities)
        self.num_relations = int(num_relations)
        self.training_triples = np.asarray(train, dtype=np.int64).reshape(-1, 3)
        self.validation_triples = np.asarray(valid, dtype=np.int64).reshape(-1, 3)
        self.testing_triples = np.asarray(test, dtype=np.int64).reshape(-1, 3)
        e2tr, e2va, e2te = defaultdict(list), defaultdict(list), defaultdict(list)
        for dst, arr in ((e2tr, self.training_triples), (e2va, self.validation_triples),
                         (e2te, self.testing_triples)):
            for s, p, o in arr.tolist():
                dst[s].append((s, p, o))
                dst[o].append((s, p, o))
        # dataset.py:114-125 -- the three dedup loops all rewrite the TRAINING lists
        for e in list(e2tr):
            e2tr[e] = list(set(e2tr[e]))
        for e in list(e2va):
            e2tr[e] = list(set(e2tr[e]))
        for e in list(e2te):
            e2tr[e] = list(set(e2tr[e]))
        self.entity_to_training_triples = e2tr
        self.entity_to_validation_triples = e2va
        self.entity_to_testing_triples = e2te
        self.entity_to_degree = {e: len(t) for e, t in e2tr.items()}
        R = self.num_relations
        self.train_to_filter = defaultdict(list)
        for s, p, o in self.training_triples.tolist():
            self.train_to_filter[(s, p)].append(o)
            self.train_to_filter[(o, p + R)].append(s)
        self.to_filter = defaultdict(list)
        for arr in (self.training_triples, self.validation_triples, self.testing_triples):
            for s, p, o in arr.tolist():
                self.to_filter[(s, p)].append(o)
                self.to_filter[(o, p + R)].append(s)
        self._relation_types()

    def _relation_types(self):
        # dataset.py:282-317
        s_num, o_num = defaultdict(list), defaultdict(list)
        for (e, r) in self.train_to_filter:
            n = len(self.to_filter[(e, r)])
            if r >= self.num_relations:
                s_num[r - self.num_relations].append(n)
            else:
                o_num[r].append(n)
        self.relation_to_type = {}
        for r in s_num:
            a_s = np.average(s_num[r])
            a_o = np.average(o_num[r])
            if a_s > 1.2 and a_o > 1.2:
                t = MANY_TO_MANY
            elif a_s > 1.2 and a_o <= 1.2:
                t = MANY_TO_ONE
            elif a_s <= 1.2 and a_o > 1.2:
                t = ONE_TO_MANY
            else:
                t = ONE_TO_ONE
            self.relation_to_type[r] = t

    def invert_triples(self, triples):
        # dataset.py:319-331
        t = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
        out = t.copy()
        out[:, 0] = t[:, 2]
        out[:, 2] = t[:, 0]
        out[:, 1] += self.num_relations
        return out


def replace_entity(triple, old, new):
    # dataset.py:333-341
    s, p, o = triple
    return (new if s == old else s, p, new if o == old else o)


class OracleKelpieView:
    """The per-entity view of ``KelpieDataset`` (kelpie_dataset.py:10-203).

    Filters are multisets (``to_filter`` lists of the reference, where
    ``list.remove`` drops one occurrence)."""

    def __init__(self, ds: OracleDataset, entity: int):
        self.ds = ds
        self.original_entity = entity
        self.kelpie_entity = ds.num_entities
        self.num_entities = ds.num_entities + 1
        k = self.kelpie_entity
        self.base_training = [replace_entity(t, entity, k) for t in ds.entity_to_training_triples[entity]]
        kva = [replace_entity(t, entity, k) for t in ds.entity_to_validation_triples.get(entity, [])]
        kte = [replace_entity(t, entity, k) for t in ds.entity_to_testing_triples.get(entity, [])]
        R = ds.num_relations
        self.filter = defaultdict(Counter)  # only keys touched by kelpie triples
        for s, p, o in self.base_training + kva + kte:
            self.filter[(s, p)][o] += 1
            self.filter[(o, p + R)][s] += 1
        self.index = {t: i for i, t in enumerate(self.base_training)}

    def as_kelpie(self, triple):
        if self.original_entity not in triple:
            raise Exception(f"Could not find the original entity {self.original_entity} in {triple}")
        return replace_entity(triple, self.original_entity, self.kelpie_entity)

    def removed(self, triples):
        """(training rows, filter for ranking) after ``remove_training_triples`` (:130-158)."""
        k = self.kelpie_entity
        R = self.ds.num_relations
        conv = [replace_entity(tuple(t), self.original_entity, k) for t in triples]
        idx = [self.index[x] for x in conv]  # KeyError like the reference
        keep = np.ones(len(self.base_training), bool)
        keep[idx] = False
        rows = [t for t, f in zip(self.base_training, keep) if f]
        filt = defaultdict(Counter, {key: Counter(v) for key, v in self.filter.items()})
        for s, p, o in conv:
            for key, val in (((s, p), o), ((o, p + R), s)):
                if filt[key][val] <= 0:
                    raise ValueError("list.remove(x): x not in list")
                filt[key][val] -= 1
        return rows, filt

    def added(self, triples):
        """(training rows, filter) after ``add_training_triples`` (:92-128)."""
        k = self.kelpie_entity
        R = self.ds.num_relations
        conv = [replace_entity(tuple(t), self.original_entity, k) for t in triples]
        rows = list(self.base_training) + conv
        filt = defaultdict(Counter, {key: Counter(v) for key, v in self.filter.items()})
        for s, p, o in conv:
            filt[(s, p)][o] += 1
            filt[(o, p + R)][s] += 1
        return rows, filt


def filter_list(filt, s, p):
    c = filt.get((s, p))
    if not c:
        return []
    return [e for e, n in c.items() if n > 0]


# =============================================================================
# models (frozen tables; scoring)
# =============================================================================
class OracleModel:
    """Frozen weights of one reference model family."""

    def __init__(self, name, weights: dict, dim: int, model_params: dict | None = None):
        self.name = name
        self.E = np.ascontiguousarray(weights["entity_embeddings"], dtype=F32)
        self.R = np.ascontiguousarray(weights["relation_embeddings"], dtype=F32)
        self.w = {k: np.asarray(v, dtype=F32) for k, v in weights.items()}
        self.dim = dim  # hp dimension (ComplEx: real dimension)
        self.params = dict(model_params or {})
        if name == "ComplEx":
            self.dimension = 2 * dim
            self.init_scale = float(self.params.get("init_scale", 1e-3))
        else:
            self.dimension = dim
        # TransE score norm p (transe.py:46; tune.py:19 searches p in {1, 2})
        self.norm = int(self.params.get("norm", 2)) if name == "TransE" else 2
        if name == "ConvE":
            self.hidden_dropout = float(self.params.get("hidden_dropout_rate", 0.0))
            self.input_dropout = float(self.params.get("input_dropout_rate", 0.0))
            self.fmap_dropout = float(self.params.get("feature_map_dropout_rate", 0.0))
            self.ew, self.eh = 20, dim // 20
            self.bn = {}
            for i in (1, 2, 3):
                inv = (1.0 / np.sqrt(self.w[f"bn{i}_var"].astype(np.float64) + 1e-5)).astype(F32)
                alpha = (inv * self.w[f"bn{i}_weight"]).astype(F32)
                beta = (self.w[f"bn{i}_bias"] - self.w[f"bn{i}_mean"] * alpha).astype(F32)
                self.bn[i] = (alpha, beta)

    def is_minimizer(self):
        return self.name == "TransE"

    # ------------------------------------------------------------ scorers
    def complex_query(self, lhs, rel):
        d = self.dim
        a, b = lhs[..., :d], lhs[..., d:]
        c, dd = rel[..., :d], rel[..., d:]
        return np.concatenate([a * c - b * dd, a * dd + b * c], axis=-1).astype(F32)

    def conve_encode(self, lhs, rel, hidden_mask=None, in_mask=None, fm_mask=None):
        """ConvE encoder (conve.py:133-153).  Returns (x, cache for backward).

        The three dropout multipliers (conve.py:142,147,151; ``None``: not drawn) are
        ``in_mask`` (b, 40, eh) on the BN1 image, ``fm_mask`` (b, 32) per feature-map
        channel after the ReLU and ``hidden_mask`` (b, d) on the FC output."""
        b = lhs.shape[0]
        d = self.dim
        img = np.concatenate([lhs.reshape(b, 20, self.eh), rel.reshape(b, 20, self.eh)], axis=1)  # (b,40,eh)
        a1, b1 = self.bn[1]
        img_bn = (img * a1[0] + b1[0]).astype(F32)
        if in_mask is not None:
            img_bn = (img_bn * in_mask.reshape(b, 40, self.eh)).astype(F32)
        W = self.w["conv_weight"][:, 0]  # (32,3,3)
        H, Wd = 38, self.eh - 2
        # per channel: the nine taps accumulated in (ky, kx) order on cache-sized arrays
        # (the same float32 operations, in the same order, as one pass per tap)
        patches = [np.ascontiguousarray(img_bn[:, ky:ky + H, kx:kx + Wd]) for ky in range(3) for kx in range(3)]
        conv = np.empty((b, 32, H, Wd), F32)
        tmp = np.empty((b, H, Wd), F32)
        for ch in range(32):
            acc = np.zeros((b, H, Wd), F32)
            for k in range(9):
                np.multiply(patches[k], W[ch, k // 3, k % 3], out=tmp)
                acc += tmp
            conv[:, ch] = acc
        conv += self.w["conv_bias"][None, :, None, None]
        a2, b2 = self.bn[2]
        c_bn = (conv * a2[None, :, None, None] + b2[None, :, None, None]).astype(F32)
        c_relu = np.maximum(c_bn, 0).astype(F32)
        if fm_mask is not None:
            c_relu = (c_relu * fm_mask.reshape(b, 32, 1, 1)).astype(F32)
        flat = c_relu.reshape(b, -1)
        fc = (flat @ self.w["fc_weight"].T + self.w["fc_bias"]).astype(F32)
        if hidden_mask is not None:
            fc_d = (fc * hidden_mask).astype(F32)
        else:
            fc_d = fc
        a3, b3 = self.bn[3]
        h_bn = (fc_d * a3 + b3).astype(F32)
        x = np.maximum(h_bn, 0).astype(F32)
        return x, (c_bn, h_bn, hidden_mask, in_mask, fm_mask)

    def conve_backward_lhs(self, dx, cache):
        """d loss / d lhs-embedding through the frozen encoder (ConvE)."""
        c_bn, h_bn, mask, in_mask, fm_mask = cache
        b = dx.shape[0]
        a3, _ = self.bn[3]
        g = dx * (h_bn > 0)
        g = g * a3
        if mask is not None:
            g = g * mask
        dflat = (g @ self.w["fc_weight"]).astype(F32)  # (b, hidden)
        H, Wd = 38, self.eh - 2
        dc = dflat.reshape(b, 32, H, Wd)
        if fm_mask is not None:
            dc = dc * fm_mask.reshape(b, 32, 1, 1)
        dc = dc * (c_bn > 0)
        a2, _ = self.bn[2]
        dc = dc * a2[None, :, None, None]
        W = self.w["conv_weight"][:, 0]
        dimg = np.zeros((b, 40, self.eh), F32)
        for ky in range(3):
            for kx in range(3):
                dimg[:, ky:ky + H, kx:kx + Wd] += np.einsum("bchw,c->bhw", dc, W[:, ky, kx])
        if in_mask is not None:
            dimg = dimg * in_mask.reshape(b, 40, self.eh)
        a1, _ = self.bn[1]
        dimg = dimg * a1[0]
        return dimg[:, :20, :].reshape(b, self.dim).astype(F32)

    def all_scores(self, triples, kelpie_row=None):
        """``Model.all_scores`` over the entity table (+ optional kelpie row at index |E|)."""
        t = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
        E = self.E if kelpie_row is None else np.vstack([self.E, kelpie_row[None].astype(F32)])
        lhs = E[t[:, 0]]
        rel = self.R[t[:, 1]]
        if self.name == "TransE":
            tr = (lhs + rel).astype(F32)
            diff = (tr[:, None, :] - E[None, :, :]).astype(np.float64)
            if self.norm == 1:
                return np.abs(diff).sum(-1).astype(F32)
            return np.sqrt((diff ** 2).sum(-1)).astype(F32)
        if self.name == "ComplEx":
            q = self.complex_query(lhs, rel)
            return (q @ E.T).astype(F32)
        x, _ = self.conve_encode(lhs, rel)
        s = (x @ E.T).astype(F32)
        return sigmoid_f32(s)


def sigmoid_f32(s):
    """torch.sigmoid on a float32 tensor (conve.py:157): 1 / (1 + exp(-x)) in float32
    arithmetic.  Near 1 its outputs step by 2^-23 and reach 1.0 at x ~ 16.64 (a float64
    sigmoid rounded once to float32 stays below 1.0 up to x ~ 17.33): the saturated ties
    the reference's rank counts (post_training_engine.py:117-121)."""
    s = np.asarray(s, dtype=F32)
    with np.errstate(over="ignore"):
        return (F32(1.0) / (F32(1.0) + np.exp(-s))).astype(F32)


def predict_tails(om, dataset, triples):
    """Model.predict_tails (model.py:42-68) / ConvE.predict_tails (conve.py:160-184):
    target score and filtered rank of each triple's tail (f3, link-prediction eval)."""
    t = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
    sc = om.all_scores(t)
    scores, ranks = [], []
    for i, (h, r, o) in enumerate(t.tolist()):
        row = sc[i].copy()
        tgt = row[o]
        F = list(dataset.to_filter.get((h, r), []))
        if om.name == "ConvE":
            row[F] = F32(0.0)
            row[o] = tgt
            rank = 1 + int((row > tgt).sum())  # descending-sort position (ties with o unordered)
        elif om.name == "TransE":
            row[F] = F32(1e6)
            row[o] = tgt
            rank = int((row <= tgt).sum())
        else:
            row[F] = F32(-1e6)
            row[o] = tgt
            rank = int((row >= tgt).sum())
        scores.append(float(tgt))
        ranks.append(rank)
    return scores, ranks


# =============================================================================
# optimizers (torch semantics, float32)
# =============================================================================
class AdagradState:
    # torch.optim.Adagrad, lr_decay 0, eps 1e-10, initial accumulator 0
    def __init__(self, n, lr, eps=1e-10):
        self.sum = np.zeros(n, F32)
        self.lr, self.eps = F32(lr), F32(eps)

    def step(self, x, g):
        self.sum = (self.sum + g * g).astype(F32)
        std = (np.sqrt(self.sum) + self.eps).astype(F32)
        return (x - self.lr * (g / std)).astype(F32)


class AdamState:
    # torch.optim.Adam (single-tensor path), weight_decay 0, amsgrad False
    def __init__(self, n, lr, betas=(0.9, 0.999), eps=1e-8):
        self.m = np.zeros(n, F32)
        self.v = np.zeros(n, F32)
        self.t = 0
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps

    def step(self, x, g):
        self.t += 1
        self.m = (self.m + F32(1 - self.b1) * (g - self.m)).astype(F32)
        self.v = (self.v * F32(self.b2) + F32(1 - self.b2) * g * g).astype(F32)
        bc1 = 1 - self.b1 ** self.t
        bc2 = 1 - self.b2 ** self.t
        step_size = self.lr / bc1
        denom = (np.sqrt(self.v) / F32(math.sqrt(bc2)) + F32(self.eps)).astype(F32)
        return (x - F32(step_size) * (self.m / denom)).astype(F32)


class SGDState:
    def __init__(self, n, lr):
        self.lr = F32(lr)

    def step(self, x, g):
        return (x - self.lr * g).astype(F32)


# =============================================================================
# full-model training (the retraining of verify_explanations.py:141-143,230-232)
# =============================================================================
class ComplExTrainer:
    """MultiClassNLLOptimizer.train / epoch / step_on_batch
    (src/link_prediction/optimization/multiclass_nll_optimizer.py:57-135) for ComplEx
    (models/complex.py:58-86 forward, regularizers.py N3), numpy float32 over the whole
    tables.  The gradients come from the full score matrix and autograd's rules written
    out: CE(mean) -> (softmax - onehot) / B, the complex product's partials, and
    d |f|^3 through f = sqrt(re^2 + im^2)."""

    def __init__(self, E, R, hp: dict):
        self.E = np.array(E, dtype=F32)
        self.R = np.array(R, dtype=F32)
        self.hp = hp
        self.half = self.E.shape[1] // 2
        name = hp["optimizer_name"]
        mk = {"Adagrad": lambda n: AdagradState(n, hp["lr"]),
              "Adam": lambda n: AdamState(n, hp["lr"], (hp.get("decay1", 0.9), hp.get("decay2", 0.999))),
              "SGD": lambda n: SGDState(n, hp["lr"])}[name]
        self.oE, self.oR = mk(self.E.size), mk(self.R.size)

    def _step(self, batch):
        E, R, h = self.E, self.R, self.half
        B = len(batch)
        lhs, rel, rhs = E[batch[:, 0]], R[batch[:, 1]], E[batch[:, 2]]
        a, b, c, e = lhs[:, :h], lhs[:, h:], rel[:, :h], rel[:, h:]
        Q = np.hstack([a * c - b * e, a * e + b * c]).astype(F32)
        S = (Q[:, :h] @ E[:, :h].T + Q[:, h:] @ E[:, h:].T).astype(F32)
        S = S - S.max(1, keepdims=True)
        P = np.exp(S)
        P = (P / P.sum(1, keepdims=True)).astype(F32)
        P[np.arange(B), batch[:, 2]] -= F32(1)
        dS = (P / F32(B)).astype(F32)
        dQ = (dS @ E).astype(F32)
        gE = (dS.T @ Q).astype(F32)
        dr, di = dQ[:, :h], dQ[:, h:]
        gl = np.hstack([dr * c + di * e, di * c - dr * e]).astype(F32)
        gr = np.hstack([dr * a + di * b, di * a - dr * b]).astype(F32)
        gt = np.zeros_like(gl)
        w = F32(self.hp.get("regularizer_weight", 0.0))
        if w != 0:
            k = F32(3) * w / F32(B)
            for g, (x, y) in ((gl, (a, b)), (gr, (c, e)), (gt, (rhs[:, :h], rhs[:, h:]))):
                m = np.sqrt(x * x + y * y).astype(F32)
                g[:, :h] += (k * m) * x
                g[:, h:] += (k * m) * y
        gR = np.zeros_like(R)
        for i in range(B):  # per-key sums in batch order
            gE[batch[i, 0]] += gl[i]
            gE[batch[i, 2]] += gt[i]
            gR[batch[i, 1]] += gr[i]
        self.E = self.oE.step(E.reshape(-1), gE.reshape(-1)).reshape(E.shape)
        self.R = self.oR.step(R.reshape(-1), gR.reshape(-1)).reshape(R.shape)

    def epoch(self, triples, perm):
        t = np.asarray(triples, dtype=np.int64).reshape(-1, 3)[np.asarray(perm, dtype=np.int64)]
        n = len(t)
        bs = min(int(self.hp["batch_size"]), n)
        start = 0
        while start < n:
            self._step(t[start:min(start + bs, n)])
            start += int(self.hp["batch_size"])


class TransETrainer:
    """PairwiseRankingOptimizer.epoch / step_on_batch (src/link_prediction/optimization/
    pairwise_ranking_optimizer.py:102-157) for TransE (models/transe.py:67-75, L2
    regularizers.py), numpy float32 over the whole tables, Adam.  ``epoch`` takes the
    epoch's positive and corrupted rows in order."""

    def __init__(self, E, R, hp: dict, norm=2):
        self.E = np.array(E, dtype=F32)
        self.R = np.array(R, dtype=F32)
        self.hp = hp
        self.norm = int(norm)
        self.oE, self.oR = AdamState(self.E.size, hp["lr"]), AdamState(self.R.size, hp["lr"])

    def _step(self, pos, neg):
        E, R = self.E, self.R
        B, d = len(pos), E.shape[1]
        rows = [E[pos[:, 0]], R[pos[:, 1]], E[pos[:, 2]], E[neg[:, 0]], R[neg[:, 1]], E[neg[:, 2]]]
        a = ((rows[0] + rows[1]) - rows[2]).astype(F32)
        b = ((rows[3] + rows[4]) - rows[5]).astype(F32)
        if self.norm == 1:  # transe.py:72 with p = 1: sum |v|, gradient sgn(v)
            sp, sn = np.abs(a).sum(1).astype(F32), np.abs(b).sum(1).astype(F32)
            hinge = ((sp - sn) + F32(self.hp["margin"])) > 0
            cp = np.where(hinge, F32(1.0 / B), F32(0))[:, None].astype(F32)
            cn = np.where(hinge, -F32(1.0 / B), F32(0))[:, None].astype(F32)
            a, b = np.sign(a).astype(F32), np.sign(b).astype(F32)
        else:
            sp = np.sqrt((a * a).sum(1)).astype(F32)
            sn = np.sqrt((b * b).sum(1)).astype(F32)
            hinge = ((sp - sn) + F32(self.hp["margin"])) > 0
            cp = np.where(hinge, F32(1.0 / B) / sp, F32(0))[:, None].astype(F32)
            cn = np.where(hinge, -F32(1.0 / B) / sn, F32(0))[:, None].astype(F32)
        wl = F32(self.hp.get("regularizer_weight", 0.0)) / (F32(3) * F32(B) * F32(d))
        g = [cp * a + wl * rows[0], cp * a + wl * rows[1], -cp * a + wl * rows[2],
             cn * b + wl * rows[3], cn * b + wl * rows[4], -cn * b + wl * rows[5]]
        gE, gR = np.zeros_like(E), np.zeros_like(R)
        keys = [(pos, 0, gE), (pos, 1, gR), (pos, 2, gE), (neg, 0, gE), (neg, 1, gR), (neg, 2, gE)]
        for i in range(B):
            for role, (src, col, G) in enumerate(keys):
                G[src[i, col]] += g[role][i]
        self.E = self.oE.step(E.reshape(-1), gE.reshape(-1)).reshape(E.shape)
        self.R = self.oR.step(R.reshape(-1), gR.reshape(-1)).reshape(R.shape)

    def epoch(self, pos, neg):
        pos = np.asarray(pos, dtype=np.int64).reshape(-1, 3)
        neg = np.asarray(neg, dtype=np.int64).reshape(-1, 3)
        bs = int(self.hp["batch_size"])
        for start in range(0, len(pos), bs):
            self._step(pos[start:start + bs], neg[start:start + bs])


# =============================================================================
# post-training (one trainable kelpie row; SURVEY App. C gradients)
# =============================================================================
class ConvETrainer:
    """Full-model ConvE training, one BCEOptimizer step at a time (bce_optimizer.py:
    45-150 on conve.py:133-158 in train mode): the reference's layer sequence restated
    with torch.nn.functional on the CPU (autograd for the gradients), the dropout noise
    given (the product draws it on the host in the forward's order), Adam with torch's
    defaults on every parameter, batch norms in eval mode for a one-pair batch."""

    def __init__(self, E, R, conv_w, conv_b, fc_w, fc_b, bn_w, bn_b, bn_m, bn_v):
        d = E.shape[1]
        t = lambda a: torch.tensor(np.asarray(a, np.float32), requires_grad=True)  # noqa: E731
        self.d = d
        self.params = {"E": t(E), "R": t(R), "cw": t(np.asarray(conv_w).reshape(32, 1, 3, 3)), "cb": t(conv_b),
                       "fw": t(fc_w), "fb": t(fc_b)}
        sl = [(0, 1), (1, 33), (33, 33 + d)]
        for i, (a0, a1) in enumerate(sl, 1):
            self.params[f"w{i}"] = t(np.asarray(bn_w)[a0:a1])
            self.params[f"b{i}"] = t(np.asarray(bn_b)[a0:a1])
        self.rm = [torch.tensor(np.asarray(bn_m, np.float32)[a0:a1]) for a0, a1 in sl]
        self.rv = [torch.tensor(np.asarray(bn_v, np.float32)[a0:a1]) for a0, a1 in sl]
        self.opt = torch.optim.Adam(list(self.params.values()), lr=1e-3)

    def step(self, pairs, tail_off, tails, in_noise, fm_noise, hid_noise, lr, label_smoothing, bn_train):
        import torch.nn.functional as F
        P = self.params
        for g in self.opt.param_groups:
            g["lr"] = lr
        d, H = self.d, self.d // 20
        pairs = torch.as_tensor(np.asarray(pairs, np.int64).reshape(-1, 2))
        B = len(pairs)
        lhs = P["E"][pairs[:, 0]].view(-1, 1, 20, H)
        rel = P["R"][pairs[:, 1]].view(-1, 1, 20, H)
        x = torch.cat([lhs, rel], 2)
        x = F.batch_norm(x, self.rm[0], self.rv[0], P["w1"], P["b1"], bool(bn_train), 0.1, 1e-5)
        if in_noise is not None:
            x = x * torch.as_tensor(np.asarray(in_noise, np.float32).reshape(B, 1, 40, H))
        x = F.conv2d(x, P["cw"], P["cb"])
        x = F.batch_norm(x, self.rm[1], self.rv[1], P["w2"], P["b2"], bool(bn_train), 0.1, 1e-5)
        x = torch.relu(x)
        if fm_noise is not None:
            x = x * torch.as_tensor(np.asarray(fm_noise, np.float32).reshape(B, 32, 1, 1))
        x = x.view(B, -1)
        x = F.linear(x, P["fw"], P["fb"])
        if hid_noise is not None:
            x = x * torch.as_tensor(np.asarray(hid_noise, np.float32).reshape(B, d))
        x = F.batch_norm(x, self.rm[2], self.rv[2], P["w3"], P["b3"], bool(bn_train), 0.1, 1e-5)
        x = torch.relu(x)
        p = torch.sigmoid(torch.mm(x, P["E"].transpose(1, 0)))
        N = P["E"].shape[0]
        tgt = torch.zeros(B, N)
        for b in range(B):
            for e in tails[tail_off[b]:tail_off[b + 1]]:
                tgt[b, int(e)] = 1.0
        if label_smoothing:
            tgt = (1.0 - label_smoothing) * tgt
            tgt += 1.0 / N
        self.opt.zero_grad()
        torch.nn.functional.binary_cross_entropy(p, tgt).backward()
        self.opt.step()

    def read(self):
        g = lambda k: self.params[k].detach().numpy().copy()  # noqa: E731
        cat = lambda xs: np.concatenate([np.asarray(v, np.float32) for v in xs])  # noqa: E731
        return {"E": g("E"), "R": g("R"), "conv_w": g("cw").reshape(32, 9), "conv_b": g("cb"), "fc_w": g("fw"),
                "fc_b": g("fb"), "bn_w": cat([g(f"w{i}") for i in (1, 2, 3)]),
                "bn_b": cat([g(f"b{i}") for i in (1, 2, 3)]), "bn_m": cat([m.numpy() for m in self.rm]),
                "bn_v": cat([v.numpy() for v in self.rv])}


def _rows_with_inverses(ds, triples):
    t = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
    return np.vstack([t, ds.invert_triples(t)])


def posttrain_complex(model: OracleModel, ds, triples, x0, hp, rng):
    """KelpieMultiClassNLLOptimizer (multiclass_nll_optimizer.py:57-99,138-164)."""
    k = ds.num_entities
    rows = _rows_with_inverses(ds, triples)
    n = rows.shape[0]
    bs = min(int(hp["batch_size"]), n)
    x = x0.astype(F32).copy()
    D = model.dimension
    name = hp["optimizer_name"]
    if name == "Adagrad":
        opt = AdagradState(D, hp["lr"])
    elif name == "Adam":
        opt = AdamState(D, hp["lr"], (hp["decay1"], hp["decay2"]))
    else:
        opt = SGDState(D, hp["lr"])
    w_reg = float(hp.get("regularizer_weight", 0.0))
    n2 = hp.get("regularizer_name", "N3") == "N2"  # multiclass_nll_optimizer.py:45-48
    for _ in range(int(hp["epochs"])):
        perm = rng.randperm(n)
        prow = rows[perm]
        start = 0
        while start < n:
            batch = prow[start:start + bs]
            E = np.vstack([model.E, x[None]])
            lhs = E[batch[:, 0]]
            rel = model.R[batch[:, 1]]
            q = model.complex_query(lhs, rel)
            logits = (q @ E.T).astype(np.float64)
            logits -= logits.max(1, keepdims=True)
            p = np.exp(logits)
            p /= p.sum(1, keepdims=True)
            b = batch.shape[0]
            G = p.copy()
            G[np.arange(b), batch[:, 2]] -= 1.0
            G /= b
            g = (G[:, k:k + 1] * q).sum(0)  # kelpie as candidate tail
            dq = G @ E.astype(np.float64)  # (b, D)
            hk = batch[:, 0] == k
            if hk.any():
                d = model.dim
                gr, gi = dq[hk, :d], dq[hk, d:]
                c, dd = rel[hk, :d].astype(np.float64), rel[hk, d:].astype(np.float64)
                g[:d] += (gr * c + gi * dd).sum(0)
                g[d:] += (-gr * dd + gi * c).sum(0)
            if w_reg != 0.0:
                d = model.dim
                for side, mask in ((lhs, hk), (E[batch[:, 2]], batch[:, 2] == k)):
                    if mask.any():
                        a_, b_ = side[mask, :d].astype(np.float64), side[mask, d:].astype(np.float64)
                        mod = np.sqrt(a_ ** 2 + b_ ** 2)
                        if n2:  # regularizers.py:25-35: ||f||^3, f = complex moduli of the row
                            mod = np.sqrt((mod ** 2).sum(1, keepdims=True))
                        g[:d] += (3 * w_reg / b * mod * a_).sum(0)
                        g[d:] += (3 * w_reg / b * mod * b_).sum(0)
            x = opt.step(x, g.astype(F32))
            start += int(hp["batch_size"])
    return x


def posttrain_transe(model: OracleModel, ds, triples, x0, hp, rng):
    """KelpiePairwiseRankingOptimizer (pairwise_ranking_optimizer.py:55-98,139-157,160-203)."""
    k = ds.num_entities
    N = ds.num_entities + 1
    rows = _rows_with_inverses(ds, triples)
    n = rows.shape[0]
    ratio = int(hp["negative_triples_ratio"])
    bs = int(hp["batch_size"])
    margin = F32(hp["margin"])
    lam = float(hp["regularizer_weight"])
    x = x0.astype(F32).copy()
    d = model.dimension
    l1 = model.norm == 1
    opt = AdamState(d, hp["lr"])
    for _ in range(int(hp["epochs"])):
        # in-place shuffle (compounding across epochs) + ratio*R negatives
        rows_e, ents, hot = rng.transe_epoch(rows, N, ratio)
        rep = np.repeat(rows_e, ratio, axis=0)[:n]
        ents, hot = ents[:n], hot[:n]
        neg = rep.copy()
        neg[:, 0] = np.where(hot == 1, ents, rep[:, 0])
        neg[:, 2] = np.where(hot == 1, rep[:, 2], ents)
        start = 0
        while start < n:
            end = min(start + bs, n)
            pos, ng = rep[start:end], neg[start:end]
            B = pos.shape[0]
            E = np.vstack([model.E, x[None]])
            g = np.zeros(d, np.float64)
            vs = []
            for tri in (pos, ng):
                v = (E[tri[:, 0]] + model.R[tri[:, 1]] - E[tri[:, 2]]).astype(F32)
                if l1:
                    f = np.abs(v.astype(np.float64)).sum(1)
                else:
                    f = np.sqrt((v.astype(np.float64) ** 2).sum(1))
                vs.append((v, f, tri))
            # clamp_min backward passes the gradient where z >= 0
            act = (vs[0][1] - vs[1][1] + float(margin)) >= 0
            for sign, (v, f, tri) in ((1.0, vs[0]), (-1.0, vs[1])):
                if l1:  # d|v|_1/dv = sgn(v), sgn(0) = 0 (torch's norm backward, p = 1)
                    u = np.sign(v).astype(np.float64)
                else:
                    with np.errstate(invalid="ignore", divide="ignore"):
                        u = np.where(f[:, None] > 0, v / f[:, None], 0.0)
                coef = sign * act / B
                g += ((coef * (tri[:, 0] == k))[:, None] * u).sum(0)
                g -= ((coef * (tri[:, 2] == k))[:, None] * u).sum(0)
            if lam != 0.0:
                cnt = sum(int((tri[:, 0] == k).sum() + (tri[:, 2] == k).sum()) for tri in (pos, ng))
                g += lam / (3.0 * B * d) * cnt * x.astype(np.float64)
            x = opt.step(x, g.astype(F32))
            start += bs
    return x


def posttrain_conve(model: OracleModel, ds, triples, x0, hp, rng):
    """KelpieBCEOptimizer (bce_optimizer.py:45-112,161-208): Adam(lr=1e-3), no shuffle."""
    k = ds.num_entities
    N = ds.num_entities + 1
    rows = _rows_with_inverses(ds, triples)
    er = OrderedDict()
    for h, r, t in rows.tolist():
        er.setdefault((h, r), []).append(t)
    pairs = list(er.keys())
    ls = float(hp["label_smoothing"])
    bs = int(hp["batch_size"])
    x = x0.astype(F32).copy()
    d = model.dimension
    opt = AdamState(d, 1e-3)
    p_hid, p_in, p_fm = model.hidden_dropout, model.input_dropout, model.fmap_dropout
    for _ in range(int(hp["epochs"])):
        start = 0
        while start < len(pairs):
            batch = pairs[start:start + bs]
            b = len(batch)
            hs = np.array([p[0] for p in batch], np.int64)
            rs = np.array([p[1] for p in batch], np.int64)
            y = np.zeros((b, N), F32)
            for i, pr in enumerate(batch):
                y[i, er[pr]] = 1.0
            if ls:
                y = (F32(1.0 - ls) * y).astype(F32)
                y = (y + F32(1.0 / N)).astype(F32)
            # the forward's draw order: input dropout over the (b, 1, 40, eh) image, the
            # feature-map Dropout2d over (b, 32), the hidden dropout over (b, d)
            # (conve.py:142,147,151; nothing drawn at rate 0, ATen _dropout_impl)
            m_in = rng.dropout_mask((b, 2 * d), p_in) if p_in > 0 else None
            m_fm = rng.dropout_mask((b, 32), p_fm) if p_fm > 0 else None
            mask = rng.dropout_mask((b, d), p_hid) if p_hid > 0 else None
            E = np.vstack([model.E, x[None]])
            enc, cache = model.conve_encode(E[hs], model.R[rs], mask, m_in, m_fm)
            s = (enc @ E.T).astype(F32)
            p = (1.0 / (1.0 + np.exp(-s.astype(np.float64)))).astype(F32)
            # BCELoss + sigmoid backward (torch): (p-y)/max(p(1-p),1e-12) * p(1-p) / (b*N)
            w = (p * (F32(1.0) - p)).astype(np.float64)
            G = (p.astype(np.float64) - y) / np.maximum(w, 1e-12) * w / (b * N)
            g = (G[:, k:k + 1] * enc).sum(0)
            hk = hs == k
            if hk.any():
                denc = (G[hk] @ E.astype(np.float64)).astype(F32)
                sub = tuple(None if a is None else a[hk] for a in cache)
                g += model.conve_backward_lhs(denc, sub).sum(0)
            x = opt.step(x, g.astype(F32))
            start += bs
    return x


POSTTRAIN = {"ComplEx": posttrain_complex, "TransE": posttrain_transe, "ConvE": posttrain_conve}


def triple_results(model: OracleModel, x, kelpie_triple, filt):
    """``PostTrainingEngine.get_triple_results`` (post_training_engine.py:101-125)."""
    s, p, o = kelpie_triple
    scores = model.all_scores([kelpie_triple], kelpie_row=x)[0].copy()
    target = float(scores[o])
    F = filter_list(filt, s, p)
    if model.is_minimizer():
        scores[F] = 1e6
        scores[o] = target
        rank = int((scores <= F32(target)).sum())
    else:
        scores[F] = -1e6
        rank = int((scores >= F32(target)).sum())
    return {"target_score": target, "target_rank": rank}


# =============================================================================
# RNG protocol: which generator draws what, in reference order
# =============================================================================
class TorchNumpyRNG:
    """Draws from torch's CPU default generator and numpy's global RandomState,
    exactly as the reference calls them."""

    def rand_init(self, D):
        return torch.rand(1, D).numpy()[0].astype(F32)  # post_training_engine.py:52

    def xavier_row(self, init, d):
        # transe.py:93-95: xavier_normal_ on a (1,d) Parameter: std = sqrt(2/(d+1))
        t = torch.from_numpy(init.reshape(1, -1).copy())
        torch.nn.init.xavier_normal_(t)
        return t.numpy()[0].astype(F32)

    def randperm(self, n):
        return torch.randperm(n).numpy()  # multiclass_nll_optimizer.py:148

    def transe_epoch(self, rows, n_entities, ratio):
        # pairwise_ranking_optimizer.py:166-172: shuffle in place, then
        # randint(N) and randint(2) over the ratio-times repeated rows
        np.random.shuffle(rows)
        n = ratio * rows.shape[0]
        ents = torch.randint(high=n_entities, size=(n,)).numpy()
        hot = torch.randint(high=2, size=(n,)).numpy()
        return rows, ents, hot

    def conve_ctor(self, hidden, dim):
        # KelpieConvE.__init__ builds a fresh ConvE(init_random=False) (conve.py:193-205),
        # whose Conv2d(1,32,3) and Linear(hidden, dim) reset_parameters() draw from the
        # CPU generator (conve.py:46-52) before being replaced by frozen copies.
        torch.nn.Conv2d(1, 32, (3, 3), 1, 0, bias=True)
        torch.nn.Linear(hidden, dim)

    def dropout_mask(self, shape, p):
        # ATen CPU dropout (_dropout_impl): zeros without a draw at p == 1, else
        # empty_like(x).bernoulli_(1-p).div_(1-p)
        if p == 1:
            return np.zeros(shape, F32)
        m = torch.empty(shape).bernoulli_(1 - p)
        m.div_(1 - p)
        return m.numpy().astype(F32)


# =============================================================================
# engines
# =============================================================================
def _sigmoid(x):
    return 1 / (1 + math.exp(-x))  # post_training_engine.py:19-20


class OracleEngine:
    """Post-training relevance engine (post_training_engine.py:17-125)."""

    def __init__(self, model: OracleModel, ds: OracleDataset, hp: dict, rng=None):
        self.model, self.ds, self.hp = model, ds, hp
        self.rng = rng or TorchNumpyRNG()
        self.o_to_training = defaultdict(list)
        for h, r, t in ds.training_triples.tolist():
            self.o_to_training[t].append((h, r, t))
        self.set_cache()

    def set_cache(self):
        self.base_results = {}
        self.views = {}

    def view(self, s):
        if s not in self.views:
            self.views[s] = OracleKelpieView(self.ds, s)
        return self.views[s]

    def _init_row(self, init):
        if self.model.name == "ConvE":
            d = self.model.dimension
            self.rng.conve_ctor(32 * 38 * (d // 20 - 2), d)
        if self.model.name == "ComplEx":
            return (init * F32(self.model.init_scale)).astype(F32)
        if self.model.name == "TransE":
            return self.rng.xavier_row(init, self.model.dimension)
        return init.copy()

    def _post_train(self, rows, x0):
        return POSTTRAIN[self.model.name](self.model, self.ds, rows, x0, self.hp, self.rng)

    def _pair(self, pred, triples, mode):
        """Returns (pt_results, base_results) -- PostTrainingEngine.compute_relevance (:46-62)."""
        s = pred[0]
        v = self.view(s)
        init = self.rng.rand_init(self.model.dimension)
        x_base0 = self._init_row(init)
        kp = v.as_kelpie(pred)
        key = tuple(pred)
        if key not in self.base_results:
            xb = self._post_train(v.base_training, x_base0)
            self.base_results[key] = triple_results(self.model, xb, kp, v.filter)
        base = self.base_results[key]
        x_pt0 = self._init_row(init)
        rows, filt = (v.removed(triples) if mode == "necessary" else v.added(triples))
        xp = self._post_train(rows, x_pt0)
        pt = triple_results(self.model, xp, kp, filt)
        return pt, base

    def necessary_relevance(self, pred, triples):
        pt, base = self._pair(pred, triples, "necessary")
        rank_d = pt["target_rank"] - base["target_rank"]
        if self.model.is_minimizer():
            sd = pt["target_score"] - base["target_score"]
        else:
            sd = base["target_score"] - pt["target_score"]
        return float(F32(F32(rank_d) + F32(_sigmoid(sd)))), pt, base  # float32 tensor add (App. A-Q5)

    def individual_sufficient_relevance(self, pred, triples):
        pt, base = self._pair(pred, triples, "sufficient")
        rank_i = base["target_rank"] - pt["target_rank"]
        if self.model.is_minimizer():
            si = base["target_score"] - pt["target_score"]
        else:
            si = pt["target_score"] - base["target_score"]
        rel = float(F32(F32(rank_i) + F32(_sigmoid(si))))
        rel /= float(base["target_rank"])
        return rel, pt, base

    def sufficient_relevance(self, pred, rule, entities):
        s = pred[0]
        rels, details = [], []
        for e in entities:
            crule = [replace_entity(tuple(t), s, e) for t in rule]
            cpred = replace_entity(tuple(pred), s, e)
            r, pt, base = self.individual_sufficient_relevance(cpred, crule)
            rels.append(r)
            details.append((pt, base))
        return sum(rels) / len(rels), details

    def select_entities_to_convert(self, pred, k, degree_cap=None, criage=False):
        """engine.py:22-126."""
        ds = self.ds
        s, p, o = pred
        ents = []
        for e in range(ds.num_entities):
            if e == s:
                continue
            deg = ds.entity_to_degree.get(e, 0)
            if deg < 1:
                continue
            if degree_cap and deg > degree_cap:
                continue
            if criage and e not in self.o_to_training:
                continue
            if (e, p) in ds.to_filter:
                if ds.relation_to_type[p] in (ONE_TO_ONE, MANY_TO_ONE):
                    continue
                if o in ds.to_filter[(e, p)]:
                    continue
            ents.append(e)
        if not ents:
            return []
        out = []
        for i0 in range(0, len(ents), 4):
            chunk = ents[i0:i0 + 4]
            sc = self.model.all_scores([(e, p, o) for e in chunk])
            for j, e in enumerate(chunk):
                row = sc[j].copy()
                F = ds.to_filter.get((e, p), [])
                t = row[o]
                if self.model.is_minimizer():
                    row[F] = 1e6
                    if 1e6 > t > row.min():
                        out.append(e)
                else:
                    row[F] = -1e6
                    if -1e6 < t < row.max():
                        out.append(e)
        return random.sample(out, k=min(k, len(out)))


# =============================================================================
# builder
# =============================================================================
def build_explanations(relevance_fn, pred, candidates, xsi, k=10, length_cap=4, window=10):
    """StochasticBuilder.build_explanations (stochastic_builder.py:33-107, 110-192),
    without summarisation; returns (rule_to_relevance top-k, #relevances)."""
    t2r = {}
    for t in candidates:
        t2r[t] = relevance_fn(pred, [t])
    srt = sorted(t2r.items(), key=lambda x: x[1], reverse=True)
    rule_to_rel = [((t,), r) for t, r in srt]
    n = len(t2r)
    nrel = n
    best = rule_to_rel[0][1]
    if not best > xsi:
        for L in range(2, min(n, length_cap) + 1):
            rules = list(combinations(candidates, L))
            rules = [(r, sum(t2r[t] for t in r)) for r in rules]
            rules = sorted(rules, key=lambda x: x[1], reverse=True)
            terminate = False
            cbest = -1e6
            win = [None] * window
            cur = {}
            cnt = 0
            for i, (rule, _) in enumerate(rules):
                if terminate:
                    break
                rel = relevance_fn(pred, list(rule))
                cur[rule] = rel
                cnt += 1
                win[i % window] = rel
                if rel > xsi:
                    break
                elif rel >= cbest:
                    cbest = rel
                elif i >= window:
                    avg = sum(win) / window
                    thr = avg / cbest
                    terminate = random.random() > thr
            nrel += cnt
            cs = sorted(cur.items(), key=lambda x: x[1], reverse=True)
            rule_to_rel += cs
            if cs[0][1] > best:
                best = cs[0][1]
            if best > xsi:
                break
    rule_to_rel = sorted(rule_to_rel, key=lambda x: (x[1], 1 / len(x[0])), reverse=True)
    return rule_to_rel[:k], nrel


def topology_prefilter(ds: OracleDataset, pred, k):
    """TopologyPreFilter.select_triples (topology_prefilter.py:18-37): BFS hop
    distance from the other endpoint to the pred's object over the undirected
    training multigraph; stable sort; first k."""
    s, _, o = pred
    adj = defaultdict(set)
    for h, _, t in ds.training_triples.tolist():
        adj[h].add(t)
        adj[t].add(h)

    def dist(a):
        if a == o:
            return 0
        seen = {a}
        frontier = [a]
        d = 0
        while frontier:
            d += 1
            nxt = []
            for u in frontier:
                for w in adj[u]:
                    if w == o:
                        return d
                    if w not in seen:
                        seen.add(w)
                        nxt.append(w)
            frontier = nxt
        return 1e6

    triples = sorted(ds.entity_to_training_triples[s])
    res = {t: dist(t[2] if t[0] == s else t[0]) for t in triples}
    res = sorted(res.items(), key=lambda x: x[1])
    return [t for t, _ in res][:k]


# ---------------------------------------------------------------------------- baseline engines (§8(f) f4)
def complex_score_rows(om: OracleModel, lhs, rel, rhs):
    """``ComplEx.score_embeddings`` (complex.py:48-57): sum over d of
    (l0 r0 - l1 r1) rh0 + (l0 r1 + l1 r0) rh1, float32."""
    d = om.dim
    l0, l1 = lhs[..., :d], lhs[..., d:]
    r0, r1 = rel[..., :d], rel[..., d:]
    h0, h1 = rhs[..., :d], rhs[..., d:]
    real = ((l0 * r0 - l1 * r1) * h0).astype(F32)
    im = ((l0 * r1 + l1 * r0) * h1).astype(F32)
    return (real + im).astype(F32).sum(-1, dtype=F32)


def complex_score_grad(om: OracleModel, triple, entity):
    """``DPEngine.get_gradient`` (data_poisoning_engine.py:21-49): d score / d (lhs if
    entity == s else rhs), as torch's autograd forms it element by element."""
    s, p, o = triple
    d = om.dim
    lhs, rel, rhs = om.E[s], om.R[p], om.E[o]
    l0, l1, r0, r1, h0, h1 = lhs[:d], lhs[d:], rel[:d], rel[d:], rhs[:d], rhs[d:]
    if entity == s:
        return np.concatenate([h0 * r0 + h1 * r1, -(h0 * r1) + h1 * r0]).astype(F32)
    return np.concatenate([l0 * r0 - l1 * r1, l0 * r1 + l1 * r0]).astype(F32)


def dp_individual(om: OracleModel, pred, perspective, triple, epsilon, lambd, mode):
    """``NecessaryDPEngine.compute_relevance`` / ``SufficientDPEngine.compute_individual_relevance``
    (data_poisoning_engine.py:52-94, 97-137).  ComplEx only: the other models have no
    ``score_embeddings`` (AttributeError in the reference)."""
    if om.name != "ComplEx":
        raise AttributeError(f"'{om.name}' object has no attribute 'score_embeddings'")
    pred_s, _, pred_o = pred
    s = triple[0]
    entity = pred_s if perspective == "head" else pred_o
    g = complex_score_grad(om, pred, entity)
    e = om.E[entity]
    step = (F32(epsilon) * g).astype(F32)
    toward = (mode == "necessary") == om.is_minimizer()  # minimizer/necessary: + eps g
    pert = (e + step if toward else e - step).astype(F32)
    t = np.asarray([triple, triple])
    lhs, rel, rhs = om.E[t[:, 0]].copy(), om.R[t[:, 1]], om.E[t[:, 2]].copy()
    if s == entity:
        lhs[1] = pert
    else:
        rhs[1] = pert
    orig, per = complex_score_rows(om, lhs, rel, rhs)
    diff = F32(orig - F32(lambd * per))
    if mode == "necessary":
        return F32(-diff) if om.is_minimizer() else diff
    return diff if om.is_minimizer() else F32(-diff)


def dp_relevance(om: OracleModel, pred, perspective, triple, epsilon, mode, entities=None, lambd=1):
    if mode == "necessary":
        return dp_individual(om, pred, perspective, triple, epsilon, lambd, mode)
    pred_s = pred[0]
    rels = []
    for ent in entities:
        # the reference rebinds triple and pred inside its loop (data_poisoning_engine.py:144-146),
        # so every conversion after the first reuses the first conversion's triple and pred
        triple = replace_entity(tuple(triple), pred_s, ent)
        pred = replace_entity(tuple(pred), pred_s, ent)
        rels.append(dp_individual(om, pred, perspective, triple, epsilon, lambd, mode))
    acc = 0
    for r in rels:
        acc = acc + r
    return acc / len(rels)


def criage_z(om: OracleModel, triple):
    """``criage_first_step`` of (s, p): ComplEx query (complex.py:131-132), ConvE encoder output
    (conve.py:102-124, eval mode)."""
    s, p = triple[0], triple[1]
    lhs, rel = om.E[s][None], om.R[p][None]
    if om.name == "ComplEx":
        return om.complex_query(lhs, rel)
    if om.name == "ConvE":
        return om.conve_encode(lhs, rel)[0]
    raise Exception("Criage does not support this model.")


def _np_sigmoid(x):
    return 1 / (1 + np.exp(-x))


def criage_hessian(om: OracleModel, entity, tail_triples):
    """``CriageEngine.compute_hessian`` (criage_engine.py:74-104): float32 terms
    sig' * x^T x (x = lhs * rel elementwise) accumulated in float64, in triple order."""
    e = om.E[entity]
    D = om.E.shape[1]
    H = np.zeros((D, D))
    for s, p, _ in tail_triples:
        x = (om.E[s] * om.R[p]).astype(F32).reshape(1, -1)
        x2 = np.dot(e, x.T)
        sig = _np_sigmoid(x2)
        sig = sig * (1 - sig)
        H += sig * np.dot(x.T, x)
    return H


def criage_variation(om: OracleModel, z_pred, z_triple, entity, H, mode):
    """``estimate_score_variation`` (criage_engine.py:107-134, 158-177), float64 solve."""
    e = om.E[entity]
    x2 = np.dot(e, z_triple.T)
    sig = _np_sigmoid(x2)
    A = H + sig * (1 - sig) * np.dot(z_triple.T, z_triple)
    m = np.linalg.inv(A)
    rel = np.dot(z_pred, ((1 - sig) * np.dot(z_triple, m)).T)
    return -rel[0][0] if mode == "necessary" else rel[0][0]


def criage_relevance(om: OracleModel, ds: OracleDataset, pred, triple, perspective, mode, entities=None,
                     tails=None):
    """``Necessary/SufficientCriageEngine.compute_relevance`` (criage_engine.py:30-52, 140-155)."""
    if tails is None:
        tails = defaultdict(list)
        for h, r, t in ds.training_triples.tolist():
            tails[t].append((h, r, t))

    def one(pred, triple):
        ps, pp, po = pred
        ent = po if perspective == "tail" else ps
        if perspective == "head":
            pred = (po, pp, ps)
        H = criage_hessian(om, ent, tails.get(ent, []))
        return criage_variation(om, criage_z(om, pred), criage_z(om, triple), ent, H, mode)

    if mode == "necessary":
        return one(tuple(pred), tuple(triple))
    ps, pp, po = pred
    s, p, _ = triple
    rels = []
    for ent in entities:
        t2 = (s, p, ent)
        p2 = (ent, pp, po) if perspective == "head" else (ps, pp, ent)
        rels.append(one(p2, t2))
    return sum(rels) / len(rels)


def criage_prefilter(ds: OracleDataset, pred, k=50):
    """``CriagePreFilter.select_triples`` (criage_prefilter.py:14-27)."""
    tails = defaultdict(list)
    for h, r, t in ds.training_triples.tolist():
        tails[t].append((h, r, t))
    s, _, o = pred
    oo = sorted(tails.get(o, []))
    so = sorted(tails.get(s, []))
    if k == -1:
        return oo + so
    return oo[:k] + so[:k]

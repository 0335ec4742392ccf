"""CPU stand-in for the HIP context, built on the oracle (TEST INFRASTRUCTURE).

It lets the CPU test tier exercise the product's host layer -- slot assembly,
the RNG protocol, filters, relevance formulas, the builder's speculative
windows -- against the reference golden vectors without a GPU.  It consumes
exactly the arrays the product ships across the C ABI (x0, rows, draws, pred,
filter) and computes each slot with the oracle's post-training code driven by
those replayed draws.  It is never used by the product: kelpie_amd has no CPU
fallback and raises when libkelpie_hip.so is unavailable.
"""
from __future__ import annotations

from collections import Counter

import numpy as np

from oracle import kelpie_oracle as ko


class _DS:
    def __init__(self, n_ent, n_rel):
        self.num_entities = n_ent
        self.num_relations = n_rel

    def invert_triples(self, t):
        t = np.asarray(t, dtype=np.int64).reshape(-1, 3)
        out = t.copy()
        out[:, 0] = t[:, 2]
        out[:, 2] = t[:, 0]
        out[:, 1] += self.num_relations
        return out


class ReplayRNG:
    """Feeds one slot's shipped draws back to the oracle's post-training code."""

    def __init__(self, model_name, blob, R, epochs, dim=None, p_drop=0.0):
        self.model_name = model_name
        self.blob = np.asarray(blob, dtype=np.int32)
        self.R = R
        self.epochs = epochs
        self.e = 0
        self.dim = dim
        self.p_drop = p_drop
        self.off = 0

    def randperm(self, n):
        if self.blob.size >= self.epochs * n and n > 0:
            p = self.blob[self.e * n:(self.e + 1) * n].astype(np.int64)
        else:
            p = np.arange(n)
        self.e += 1
        return p

    def transe_epoch(self, rows, n_entities, ratio):
        R = self.R
        blk = self.blob.reshape(self.epochs, 3, R)[self.e] if R else np.zeros((3, 0), np.int32)
        self.e += 1
        return rows[blk[0].astype(np.int64)], blk[1].astype(np.int64), blk[2].astype(np.int64)

    def dropout_mask(self, shape, p):
        # the shipped layout: per step, one word-aligned run of keep bits per dropout
        # (input, feature map, hidden: the forward's draw order)
        n = int(np.prod(shape))
        words = (n + 31) // 32
        w = self.blob[self.off:self.off + words].view(np.uint32)
        self.off += words
        bits = np.unpackbits(w.view(np.uint8), bitorder="little")[:n].astype(np.float32)
        if p == 1:  # zeros (the library ships zero words and draws nothing)
            return np.zeros(shape, np.float32)
        scale = np.float32(1.0) / np.float32(1.0 - p)
        return (bits * scale).astype(np.float32).reshape(shape)


class OracleBackedContext:
    def __init__(self, model):
        """``model``: a kelpie_amd FrozenModel (weights are read from it)."""
        self.model = model
        name = model.name
        w = {"entity_embeddings": model.entity_embeddings, "relation_embeddings": model.relation_embeddings}
        params = {}
        if name == "ComplEx":
            dim = model.real_dimension
            params["init_scale"] = model.init_scale
        elif name == "ConvE":
            dim = model.dimension
            w.update({"conv_weight": model.conv_weight.reshape(32, 1, 3, 3), "conv_bias": model.conv_bias,
                      "fc_weight": model.fc_weight, "fc_bias": model.fc_bias})
            # the oracle rebuilds alpha/beta from BN stats; give it identity stats and
            # pre-folded weights/bias so alpha = bn_alpha, beta = bn_beta exactly
            off = 0
            for i, c in ((1, 1), (2, 32), (3, model.dimension)):
                a, b = model.bn_alpha[off:off + c], model.bn_beta[off:off + c]
                off += c
                w[f"bn{i}_weight"], w[f"bn{i}_bias"] = a, b
                w[f"bn{i}_mean"], w[f"bn{i}_var"] = np.zeros(c, np.float32), np.ones(c, np.float32)
            params["hidden_dropout_rate"] = model.hidden_dropout_rate
            params["input_dropout_rate"] = model.input_dropout_rate
            params["feature_map_dropout_rate"] = model.feature_map_dropout_rate
        else:
            dim = model.dimension
            params["norm"] = model.norm
        self.om = ko.OracleModel(name, w, dim, params)
        if name == "ConvE":
            off = 0
            for i, c in ((1, 1), (2, 32), (3, model.dimension)):
                self.om.bn[i] = (model.bn_alpha[off:off + c], model.bn_beta[off:off + c])
                off += c
        self.ds = _DS(model.dataset.num_entities, model.dataset.num_relations)
        self.n_ent = model.dataset.num_entities
        self.dim = model.dimension
        self.calls = []

    def _hp(self, hp):
        if self.model.name == "ComplEx":
            names = {0: "Adagrad", 1: "Adam", 2: "SGD"}
            return {"optimizer_name": names[hp.optimizer], "batch_size": hp.batch_size, "epochs": hp.epochs,
                    "lr": hp.lr, "decay1": hp.beta1, "decay2": hp.beta2, "regularizer_weight": hp.reg_weight,
                    "regularizer_name": {0: "N3", 1: "N2"}[hp.reg_kind]}
        if self.model.name == "TransE":
            return {"batch_size": hp.batch_size, "epochs": hp.epochs, "lr": hp.lr, "margin": hp.margin,
                    "negative_triples_ratio": hp.neg_ratio, "regularizer_weight": hp.reg_weight}
        return {"batch_size": hp.batch_size, "epochs": hp.epochs, "label_smoothing": hp.label_smoothing}

    def posttrain_rank(self, hp, x0, row_off, rows, rng_off, rng, pred, filt_off, filt, want_x=False):
        n = len(row_off) - 1
        hpd = self._hp(hp)
        out_s = np.zeros(n, np.float32)
        out_r = np.zeros(n, np.int64)
        out_x = np.zeros((n, self.dim), np.float32)
        self.calls.append(n)
        for i in range(n):
            r = rows[row_off[i]:row_off[i + 1]]
            R = len(r)
            trip = r[:R // 2]
            blob = rng[rng_off[i]:rng_off[i + 1]]
            rr = ReplayRNG(self.model.name, blob, R, int(hp.epochs), self.dim, getattr(hp, "hidden_dropout", 0.0))
            x = ko.POSTTRAIN[self.model.name](self.om, self.ds, trip, x0[i], hpd, rr)
            kp = tuple(int(v) for v in pred[i])
            F = Counter(int(e) for e in filt[filt_off[i]:filt_off[i + 1]])
            res = ko.triple_results(self.om, x, kp, {(kp[0], kp[1]): F})
            out_s[i] = res["target_score"]
            out_r[i] = res["target_rank"]
            out_x[i] = x
        return out_s, out_r, (out_x if want_x else None)

    def all_scores(self, heads, rels):
        t = np.stack([heads, rels, np.zeros_like(heads)], 1)
        return self.om.all_scores(t)

    def convertible(self, heads, rel, obj, filt_off, filt):
        keep = np.zeros(len(heads), np.uint8)
        sc = self.all_scores(np.asarray(heads), np.full(len(heads), rel))
        for i in range(len(heads)):
            row = sc[i].copy()
            F = filt[filt_off[i]:filt_off[i + 1]]
            t = row[obj]
            if self.model.is_minimizer():
                row[F] = 1e6
                keep[i] = 1 if (1e6 > t > row.min()) else 0
            else:
                row[F] = -1e6
                keep[i] = 1 if (-1e6 < t < row.max()) else 0
        return keep

    def predict_tails(self, triples, filt_off, filt):
        sc, rk = ko.predict_tails(self.om, self.model.dataset, triples)
        return np.array(sc, np.float32), np.array(rk, np.int64)

    def last_timing(self):
        return {"device_s": 0.0, "hot_s": 0.0, "hot_launches": 0}

    def train_epoch(self, hp, triples, perm, epoch):
        """Stand-in for kp_train_epoch: the oracle's trainer on this context's tables."""
        if epoch == 0 or getattr(self, "_trainer", None) is None:
            hpd = self._hp(hp)
            if self.model.name == "TransE":
                self._trainer = ko.TransETrainer(self.om.E, self.om.R, hpd, norm=self.om.norm)
            else:
                hpd["optimizer_name"] = {0: "Adagrad", 1: "Adam", 2: "SGD"}[hp.optimizer]
                self._trainer = ko.ComplExTrainer(self.om.E, self.om.R, hpd)
        self._trainer.epoch(triples, perm)
        self.om.E, self.om.R = self._trainer.E, self._trainer.R

    def read_tables(self, n_rel2):
        if getattr(self, "_cvtrainer", None) is not None:
            r = self._cvtrainer.read()
            return r["E"], r["R"]
        return self.om.E.copy(), self.om.R.copy()

    # stand-ins for kp_conve_train_* (the oracle's ConvE trainer on this context's weights)
    def conve_train_begin(self, bn_w, bn_b, bn_m, bn_v):
        m = self.model
        self._cvtrainer = ko.ConvETrainer(m.entity_embeddings, m.relation_embeddings, m.conv_weight, m.conv_bias,
                                          m.fc_weight, m.fc_bias, bn_w, bn_b, bn_m, bn_v)

    def conve_train_step(self, pairs, tail_off, tails, in_noise, fm_noise, hid_noise, lr, label_smoothing, bn_train):
        self._cvtrainer.step(pairs, tail_off, tails, in_noise, fm_noise, hid_noise, lr, label_smoothing, bn_train)

    def conve_train_read(self):
        r = self._cvtrainer.read()
        return {k: r[k] for k in ("conv_w", "conv_b", "fc_w", "fc_b", "bn_w", "bn_b", "bn_m", "bn_v")}


def _dp_relevance(self, items, epsilon, lambd, step_sign, rel_sign):
    """Stand-in for kp_dp_relevance (oracle arithmetic on the shipped items)."""
    om = self.om
    out = []
    for s, p, o, e, h, r, t in np.asarray(items).reshape(-1, 7).tolist():
        g = ko.complex_score_grad(om, (s, p, o), e)
        step = (np.float32(epsilon) * g).astype(np.float32)
        pert = (om.E[e] + step if step_sign > 0 else om.E[e] - step).astype(np.float32)
        lhs, rel, rhs = om.E[[h, h]].copy(), om.R[[r, r]], om.E[[t, t]].copy()
        if h == e:
            lhs[1] = pert
        else:
            rhs[1] = pert
        a, b = ko.complex_score_rows(om, lhs, rel, rhs)
        out.append(np.float32(rel_sign) * np.float32(a - np.float32(lambd * b)))
    return np.asarray(out, np.float32)


def _criage_relevance(self, items, ent_ids, tails_off, tails):
    """Stand-in for kp_criage_relevance."""
    om = self.om
    H = {}
    out, status = [], []
    for zs, zp, ts, tp, slot in np.asarray(items).reshape(-1, 5).tolist():
        ent = int(ent_ids[slot])
        if ent not in H:
            tl = [(h, r, ent) for h, r in np.asarray(tails).reshape(-1, 2)[tails_off[slot]:tails_off[slot + 1]].tolist()]
            H[ent] = ko.criage_hessian(om, ent, tl)
        try:
            v = ko.criage_variation(om, ko.criage_z(om, (zs, zp, 0)), ko.criage_z(om, (ts, tp, 0)), ent, H[ent],
                                    "sufficient")
            out.append(float(v))
            status.append(0)
        except np.linalg.LinAlgError:
            out.append(float("nan"))
            status.append(1)
    return np.asarray(out), np.asarray(status, np.int32)


OracleBackedContext.dp_relevance = _dp_relevance
OracleBackedContext.criage_relevance = _criage_relevance

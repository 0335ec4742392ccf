"""Baseline relevance engines of the reference, on the GPU.

Drop-in for ``src/relevance_engines/data_poisoning_engine.py`` and
``src/relevance_engines/criage_engine.py`` plus ``src/prefilters/criage_prefilter.py``:
same class names, constructors, ``compute_relevance`` argument orders and
errors.  Each call is one batched HIP launch (``kp_dp_relevance`` /
``kp_criage_relevance``); ``compute_relevance_batch`` evaluates many
candidate triples of one prediction in one launch.

Reference behaviour kept on purpose:

* the DP engine scores with ``model.score_embeddings``, which only ComplEx has
  (TransE and ConvE raise ``AttributeError``, data_poisoning_engine.py:44);
* ``SufficientDPEngine.compute_relevance`` rebinds ``triple`` and ``pred``
  inside its loop (data_poisoning_engine.py:144-146), so every conversion after
  the first reuses the first one's triple and prediction;
* DP relevances are float32 (numpy scores), sufficient means are accumulated in
  float32; CRIAGE values are float64;
* ``NecessaryCriageEngine`` returns ``None`` when the system is singular
  (``numpy.linalg.inv`` raises inside its ``try``, criage_engine.py:117-133);
  ``SufficientCriageEngine`` lets ``numpy.linalg.LinAlgError`` propagate.
* The reference's ``DataPoisoningBuilder`` / ``CriageBuilder`` call an engine
  method ``compute_rule_relevance`` that no engine defines (dp_builder.py:20,
  criage_builder.py:22); the engines here do not define it either.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np

from .data import Dataset
from .engine import RelevanceEngine


class DPEngine(RelevanceEngine):
    """data_poisoning_engine.py:9-49."""

    def __init__(self, model, dataset, epsilon: float):
        RelevanceEngine.__init__(self, model=model, dataset=dataset)
        self.epsilon = epsilon
        self.lambd = 1
        self.entities_to_convert = []

    def _check_model(self):
        if self.model.name != "ComplEx":
            raise AttributeError(f"'{self.model.name}' object has no attribute 'score_embeddings'")

    def _items(self, pred, perspective, triples):
        pred_s, _, pred_o = (int(v) for v in pred)
        entity = pred_s if perspective == "head" else pred_o
        return [[int(pred[0]), int(pred[1]), int(pred[2]), entity, int(t[0]), int(t[1]), int(t[2])] for t in triples]

    def _run(self, items, mode):
        self._check_model()
        if not items:
            return np.zeros(0, np.float32)
        toward = (mode == "necessary") == self.model.is_minimizer()
        # necessary, maximizer: e - eps g, rel = orig - lambd pert; sufficient: e + eps g, rel = -(orig - lambd pert)
        rel_sign = 1 if (mode == "necessary") != self.model.is_minimizer() else -1
        return self.model.ctx.dp_relevance(np.asarray(items), self.epsilon, self.lambd, 1 if toward else -1, rel_sign)

    def compute_relevance(self, pred, perspective: str, triple):
        raise NotImplementedError


class NecessaryDPEngine(DPEngine):
    """data_poisoning_engine.py:51-94."""

    def compute_relevance(self, pred, perspective: str, triple):
        return self.compute_relevance_batch(pred, perspective, [triple])[0]

    def compute_relevance_batch(self, pred, perspective: str, triples):
        return [np.float32(v) for v in self._run(self._items(pred, perspective, triples), "necessary")]

    def compute_relevance_multi(self, jobs, perspective: str):
        """[(pred, triples), ...] in one launch -> [[relevance per triple], ...]."""
        items = [it for pred, triples in jobs for it in self._items(pred, perspective, triples)]
        vals = self._run(items, "necessary")
        out, k = [], 0
        for _, triples in jobs:
            out.append([np.float32(v) for v in vals[k:k + len(triples)]])
            k += len(triples)
        return out


class SufficientDPEngine(DPEngine):
    """data_poisoning_engine.py:97-152."""

    def compute_relevance(self, pred, perspective: str, triple):
        return self.compute_relevance_batch(pred, perspective, [triple])[0]

    def compute_relevance_batch(self, pred, perspective: str, triples):
        self._check_model()
        if not self.entities_to_convert:
            raise ZeroDivisionError("division by zero")  # sum([]) / len([])
        pred_s = int(pred[0])
        items, counts = [], []
        for triple in triples:
            p, t = tuple(int(v) for v in pred), tuple(int(v) for v in triple)
            n = 0
            for entity in self.entities_to_convert:
                t = Dataset.replace_entity_in_triple(t, pred_s, int(entity))
                p = Dataset.replace_entity_in_triple(p, pred_s, int(entity))
                items += self._items(p, perspective, [t])
                n += 1
            counts.append(n)
        vals = self._run(items, "sufficient")
        out, k = [], 0
        for n in counts:
            acc = np.float32(0)
            for v in vals[k:k + n]:
                acc = np.float32(acc + v)
            out.append(np.float32(acc / np.float32(n)))
            k += n
        return out


class CriageEngine(RelevanceEngine):
    """criage_engine.py:11-104."""

    def __init__(self, model, dataset):
        RelevanceEngine.__init__(self, model=model, dataset=dataset)
        if model.name not in ("ComplEx", "ConvE", "DistMult"):
            raise Exception("Criage does not support this model.")
        self.entity_dimension = self.model.dimension
        self.tail_to_training_triples = defaultdict(list)
        for h, r, t in dataset.training_triples.tolist():
            self.tail_to_training_triples[t].append((h, r, t))
        self.entities_to_convert = []

    def _items(self, pairs, perspective):
        """pairs: [(pred, triple)] -> (values float64, status) per pair (criage_engine.py:30-52)."""
        ent_slot, ent_ids, off, tails, items = {}, [], [0], [], []
        for pred, triple in pairs:
            ps, pp, po = (int(v) for v in pred)
            ent = po if perspective == "tail" else ps
            if perspective == "head":
                ps, po = po, ps  # z of the swapped prediction (criage_engine.py:36-37)
            if ent not in ent_slot:
                ent_slot[ent] = len(ent_ids)
                ent_ids.append(ent)
                for h, r, _ in self.tail_to_training_triples.get(ent, []):
                    tails.append((h, r))
                off.append(len(tails))
            items.append([ps, pp, int(triple[0]), int(triple[1]), ent_slot[ent]])
        if not items:
            return np.zeros(0), np.zeros(0, np.int32)
        return self.model.ctx.criage_relevance(np.asarray(items), np.asarray(ent_ids), np.asarray(off),
                                               np.asarray(tails, dtype=np.int32).reshape(-1, 2))

    def compute_relevance(self, pred, triple, perspective: str):
        raise NotImplementedError


class NecessaryCriageEngine(CriageEngine):
    """criage_engine.py:107-134."""

    def compute_relevance(self, pred, triple, perspective: str):
        return self.compute_relevance_batch(pred, [triple], perspective)[0]

    def compute_relevance_batch(self, pred, triples, perspective: str):
        vals, status = self._items([(pred, t) for t in triples], perspective)
        return [None if st else -float(v) for v, st in zip(vals, status)]

    def compute_relevance_multi(self, jobs, perspective: str):
        """[(pred, triples), ...] in one launch (one Hessian per distinct entity)."""
        vals, status = self._items([(pred, t) for pred, triples in jobs for t in triples], perspective)
        out, k = [], 0
        for _, triples in jobs:
            out.append([None if st else -float(v) for v, st in zip(vals[k:k + len(triples)], status[k:k + len(triples)])])
            k += len(triples)
        return out


class SufficientCriageEngine(CriageEngine):
    """criage_engine.py:137-177."""

    def compute_relevance(self, pred, triple, perspective: str):
        return self.compute_relevance_batch(pred, [triple], perspective)[0]

    def compute_relevance_batch(self, pred, triples, perspective: str):
        if not self.entities_to_convert:
            raise ZeroDivisionError("division by zero")
        pred_s, pred_p, pred_o = (int(v) for v in pred)
        pairs = []
        for triple in triples:
            s, p = int(triple[0]), int(triple[1])
            for entity in self.entities_to_convert:
                t2 = (s, p, int(entity))
                p2 = (int(entity), pred_p, pred_o) if perspective == "head" else (pred_s, pred_p, int(entity))
                pairs.append((p2, t2))
        vals, status = self._items(pairs, perspective)
        if status.any():
            raise np.linalg.LinAlgError("Singular matrix")
        n = len(self.entities_to_convert)
        return [float(sum(float(v) for v in vals[i * n:(i + 1) * n]) / n) for i in range(len(triples))]


class CriagePreFilter:
    """criage_prefilter.py:7-27."""

    def __init__(self, dataset):
        self.dataset = dataset
        self.o_to_training_triples = defaultdict(list)
        for h, r, t in dataset.training_triples.tolist():
            self.o_to_training_triples[t].append((h, r, t))

    def select_triples(self, pred, k=50):
        pred_s, _, pred_o = pred
        oo = sorted(self.o_to_training_triples.get(int(pred_o), []))
        so = sorted(self.o_to_training_triples.get(int(pred_s), []))
        if k == -1:
            return oo + so
        return oo[:k] + so[:k]

"""Candidate prefilters upstream of the relevance engine.

Same classes, constructor arguments and ``select_triples(pred, k)`` results as
the reference's ``src/prefilters``; the graph searches run in the library's host
C++ (``kp_graph_*`` in ``include/kelpie_hip.h``, ``kelpie_amd/csrc/kp_graph.cpp``).

* ``TopologyPreFilter`` (topology_prefilter.py:9-37): hop distance from each
  candidate's other endpoint to the prediction's object; ONE breadth-first
  search from the object serves every candidate (the reference runs networkx
  once per candidate; hop distances are symmetric).
* ``WeightedTopologyPreFilter`` (weighted_topology_prefilter.py:13-56): edge
  cost ``1 - jaccard(classes(u), classes(v))``; one Dijkstra per distinct
  candidate endpoint replaying networkx's search order, so float sums and ties
  match.  An entity without a classes row counts as an empty class set (the
  reference raises ``KeyError`` when a search reaches it).
* ``NoPreFilter`` (no_prefilter.py).

``TypeBasedPreFilter`` is not provided: the reference's relation vectors are
``(num_entities, 2|R|)`` matrices per entity whose cosine is a matrix, and its
sort then fails (out of scope).
"""
from __future__ import annotations

import ast
import csv
import math

from . import _lib

TOPOLOGY_PREFILTER = "topology_based"
WEIGHTED_TOPOLOGY_PREFILTER = "weighted_topology_based"
TYPE_PREFILTER = "type_based"
NO_PREFILTER = "none"

NO_PATH = 1e6  # topology_prefilter.py:36-37


def _key(x):  # prefilter.py:8
    return x[1]


class PreFilter:
    def __init__(self, dataset):
        self.dataset = dataset


class NoPreFilter(PreFilter):
    """no_prefilter.py: every training triple of the subject, unsorted."""

    def __init__(self, dataset):
        super().__init__(dataset)
        self.entity_to_training_triples = self.dataset.entity_to_training_triples

    def select_triples(self, pred, k=-1):
        s, _, _ = pred
        return self.entity_to_training_triples[s]


class TopologyPreFilter(PreFilter):
    def __init__(self, dataset):
        super().__init__(dataset)
        self.graph = _lib.Graph(dataset.num_entities, dataset.training_triples)
        self.entity_to_training_triples = self.dataset.entity_to_training_triples

    def _distances(self, objects):
        return self.graph.bfs(objects)

    def select_triples(self, pred, k=50):
        return self.select_triples_batch([pred], k)[0]

    def select_triples_batch(self, preds, k=50):
        """select_triples for many predictions: one search per distinct object."""
        objs = sorted({int(p[2]) for p in preds})
        dist = dict(zip(objs, self._distances(objs)))
        out = []
        for pred in preds:
            s, _, o = (int(v) for v in pred)
            d = dist[o]
            triples = sorted(self.entity_to_training_triples[s])
            results = {}
            for t in triples:
                e = t[2] if t[0] == s else t[0]
                v = int(d[e])
                results[t] = NO_PATH if v < 0 else v
            ranked = sorted(results.items(), key=_key)
            out.append([x[0] for x in ranked][:k])
        return out


def load_entity_classes(path, entity_to_id):
    """``{entity id: set of class labels}`` from a reasoned ``entities.csv``
    (columns entity, classes; classes a Python set literal), the table the
    reference loads as ``entities_semantic_impl`` (src/data/dataset.py:78-83).
    Parsed with ``ast.literal_eval`` (no code execution)."""
    out = {}
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            eid = entity_to_id.get(row["entity"])
            if eid is None:
                continue
            out[int(eid)] = set(ast.literal_eval(row["classes"]))
    return out


class WeightedTopologyPreFilter(PreFilter):
    def __init__(self, dataset, entity_classes=None):
        """``entity_classes``: {entity id: iterable of class labels}; defaults to
        ``dataset.entity_classes`` (see :func:`load_entity_classes`)."""
        super().__init__(dataset)
        classes = entity_classes if entity_classes is not None else getattr(dataset, "entity_classes", None)
        if classes is None:
            raise ValueError("WeightedTopologyPreFilter needs entity classes (load_entity_classes)")
        self.graph = _lib.Graph(dataset.num_entities, dataset.training_triples)
        label_id, off, ids = {}, [0], []
        for e in range(dataset.num_entities):
            for c in classes.get(e, ()):
                ids.append(label_id.setdefault(c, len(label_id)))
            off.append(len(ids))
        self.graph.set_classes(off, ids)
        self.entity_to_training_triples = self.dataset.entity_to_training_triples

    def select_triples(self, pred, k=50):
        s, _, o = (int(v) for v in pred)
        triples = sorted(self.entity_to_training_triples[s])
        ends = [t[2] if t[0] == s else t[0] for t in triples]
        uniq = list(dict.fromkeys(ends))
        d = dict(zip(uniq, self.graph.dijkstra_pairs(uniq, [o] * len(uniq)))) if uniq else {}
        results = {t: (NO_PATH if math.isinf(d[e]) else float(d[e])) for t, e in zip(triples, ends)}
        ranked = sorted(results.items(), key=_key)
        return [x[0] for x in ranked][:k]


PREFILTERS = {TOPOLOGY_PREFILTER: TopologyPreFilter, NO_PREFILTER: NoPreFilter,
              WEIGHTED_TOPOLOGY_PREFILTER: WeightedTopologyPreFilter}

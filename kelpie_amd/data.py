"""Host-side data layer: the reference's dataset indices and per-entity kelpie views.

``Dataset`` keeps the attribute names and semantics of the reference
``src/data/dataset.py:17-352`` that the relevance path reads
(``entity_to_training_triples`` in ``list(set(...))`` order, ``to_filter`` /
``train_to_filter`` over direct and inverse keys, ``entity_to_degree``,
``relation_to_type``, ``invert_triples``, ``replace_entity_in_triple(s)``).
It is built from id triples (the PyKEEN download path, ``dataset.py:97``, is
replaced by :func:`Dataset.from_directory` over local TSV files with
PyKEEN-style sorted-label ids).

``KelpieView`` replaces ``KelpieDataset`` (``src/data/kelpie_dataset.py``):
instead of deep-copying the whole filter dictionaries per subject
(``kelpie_dataset.py:13-14``, seconds per prediction) it keeps only the
kelpie entity's own triples and the filter multisets of keys that start at
the kelpie entity, which is everything the post-training rank reads.
"""
from __future__ import annotations

import csv
import itertools
import os
from collections import Counter, defaultdict

import numpy as np

ONE_TO_ONE = "1-1"
ONE_TO_MANY = "1-N"
MANY_TO_ONE = "N-1"
MANY_TO_MANY = "N-N"


class Dataset:
    def __init__(self, num_entities, num_relations, train, valid, test, name="synthetic",
                 entity_to_id=None, relation_to_id=None):
        self.name = name
        self._num_entities = int(num_entities)
        self._num_relations = int(num_relations)
        self._train = np.ascontiguousarray(np.asarray(train, dtype=np.int64).reshape(-1, 3))
        self._valid = np.ascontiguousarray(np.asarray(valid, dtype=np.int64).reshape(-1, 3))
        self._test = np.ascontiguousarray(np.asarray(test, dtype=np.int64).reshape(-1, 3))
        self.entity_to_id = entity_to_id or {f"e{i:06d}": i for i in range(self._num_entities)}
        self.relation_to_id = relation_to_id or {f"r{i:04d}": i for i in range(self._num_relations)}
        self.id_to_entity = {v: k for k, v in self.entity_to_id.items()}
        self.id_to_relation = {v: k for k, v in self.relation_to_id.items()}
        self._build_indices()

    # ------------------------------------------------------------------ loading
    @classmethod
    def from_directory(cls, path, name=None):
        """Load ``train.txt`` / ``valid.txt`` / ``test.txt`` (tab-separated labels).

        Ids follow PyKEEN's ``TriplesFactory.from_path``: sorted unique labels of
        the training file; valid/test triples with unseen labels are dropped."""

        def read(fn):
            out = []
            fp = os.path.join(path, fn)
            if not os.path.exists(fp):
                return out
            with open(fp, newline="") as f:
                for row in csv.reader(f, delimiter="\t"):
                    if len(row) >= 3:
                        out.append((row[0].strip(), row[1].strip(), row[2].strip()))
            return out

        tr, va, te = read("train.txt"), read("valid.txt"), read("test.txt")
        ents = sorted({h for h, _, _ in tr} | {t for _, _, t in tr})
        rels = sorted({r for _, r, _ in tr})
        e2i = {e: i for i, e in enumerate(ents)}
        r2i = {r: i for i, r in enumerate(rels)}

        def ids(trip):
            keep = [(e2i[h], r2i[r], e2i[t]) for h, r, t in trip if h in e2i and t in e2i and r in r2i]
            return np.array(keep, dtype=np.int64).reshape(-1, 3)

        return cls(len(ents), len(rels), ids(tr), ids(va), ids(te), name=name or os.path.basename(path),
                   entity_to_id=e2i, relation_to_id=r2i)

    # ------------------------------------------------------------------ indices
    def _build_indices(self):
        # dataset.py:104-125
        e2tr, e2va, e2te = defaultdict(list), defaultdict(list), defaultdict(list)
        for dst, arr in ((e2tr, self._train), (e2va, self._valid), (e2te, self._test)):
            for s, p, o in arr.tolist():
                dst[s].append((s, p, o))
                dst[o].append((s, p, o))
        for e in list(e2tr):
            e2tr[e] = list(set(e2tr[e]))
        # the reference's validation / test dedup loops rewrite the TRAINING lists
        # of those entities (dataset.py:118-125); keep the order effect
        for e in list(e2va):
            e2tr[e] = list(set(e2tr[e]))
        for e in list(e2te):
            e2tr[e] = list(set(e2tr[e]))
        self.entity_to_training_triples = e2tr
        self.entity_to_validation_triples = e2va
        self.entity_to_testing_triples = e2te
        self.entity_to_degree = {e: len(t) for e, t in e2tr.items()}
        R = self._num_relations
        self.train_to_filter = defaultdict(list)
        for s, p, o in self._train.tolist():
            self.train_to_filter[(s, p)].append(o)
            self.train_to_filter[(o, p + R)].append(s)
        self.to_filter = defaultdict(list)
        for arr in (self._train, self._valid, self._test):
            for s, p, o in arr.tolist():
                self.to_filter[(s, p)].append(o)
                self.to_filter[(o, p + R)].append(s)
        self._compute_relation_to_type()

    def _compute_relation_to_type(self):
        # dataset.py:282-317
        s_num, o_num = defaultdict(list), defaultdict(list)
        for (e, r) in self.train_to_filter:
            n = len(self.to_filter[(e, r)])
            if r >= self._num_relations:
                s_num[r - self._num_relations].append(n)
            else:
                o_num[r].append(n)
        self.relation_to_type = {}
        for r in s_num:
            a_s, a_o = np.average(s_num[r]), np.average(o_num[r])
            if a_s > 1.2 and a_o > 1.2:
                t = MANY_TO_MANY
            elif a_s > 1.2 and a_o <= 1.2:
                t = MANY_TO_ONE
            elif a_s <= 1.2 and a_o > 1.2:
                t = ONE_TO_MANY
            else:
                t = ONE_TO_ONE
            self.relation_to_type[r] = t

    # ------------------------------------------------------------------ reference API
    @property
    def num_entities(self):
        return self._num_entities

    @property
    def num_relations(self):
        return self._num_relations

    @property
    def training_triples(self):
        return self._train

    @property
    def validation_triples(self):
        return self._valid

    @property
    def testing_triples(self):
        return self._test

    @property
    def all_triples(self):
        return np.vstack([self._train, self._valid, self._test])

    def invert_triples(self, triples):
        t = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
        out = t.copy()
        out[:, 0] = t[:, 2]
        out[:, 2] = t[:, 0]
        out[:, 1] += self._num_relations
        return out

    @staticmethod
    def replace_entity_in_triple(triple, old_entity, new_entity):
        s, p, o = triple
        return (new_entity if s == old_entity else s, p, new_entity if o == old_entity else o)

    @staticmethod
    def replace_entity_in_triples(triples, old_entity, new_entity):
        return [Dataset.replace_entity_in_triple(t, old_entity, new_entity) for t in triples]

    # ------------------------------------------------------------------ edits (verification)
    # dataset.py:242-280, the edits verify_explanations.py makes on a deep copy: the
    # training rows are filtered / appended, and the DIRECT (s, p) filter keys and the
    # training-triple index follow; the inverse keys are left as they are, as there.
    def copy(self):
        import copy
        return copy.deepcopy(self)

    def add_training_triple(self, triple):
        s, p, o = (int(v) for v in triple)
        self._train = np.vstack([self._train, np.array([[s, p, o]], dtype=np.int64)])
        self.entity_to_training_triples[s].append((s, p, o))
        self.entity_to_training_triples[o].append((s, p, o))
        self.entity_to_degree[s] = self.entity_to_degree.get(s, 0) + 1
        self.entity_to_degree[o] = self.entity_to_degree.get(o, 0) + 1
        self.to_filter[(s, p)].append(o)
        self.train_to_filter[(s, p)].append(o)

    def add_training_triples(self, triples):
        for t in triples:
            self.add_training_triple(t)

    def remove_training_triple(self, triple):
        s, p, o = (int(v) for v in triple)
        t = self._train
        self._train = np.ascontiguousarray(t[~((t[:, 0] == s) & (t[:, 1] == p) & (t[:, 2] == o))])
        self.entity_to_training_triples[s].remove((s, p, o))  # ValueError when absent, as there
        if s != o:
            self.entity_to_training_triples[o].remove((s, p, o))
        self.entity_to_degree[s] -= 1
        if s != o:
            self.entity_to_degree[o] -= 1
        self.to_filter[(s, p)].remove(o)
        self.train_to_filter[(s, p)].remove(o)

    def remove_training_triples(self, triples):
        for t in set(tuple(int(v) for v in x) for x in triples):  # set(triples) order, as there
            self.remove_training_triple(t)

    def labels_triple(self, t):
        s, p, o = t
        return (self.id_to_entity[s], self.id_to_relation[p], self.id_to_entity[o])

    def labels_triples(self, ts):
        return [self.labels_triple(t) for t in ts]

    def ids_triple(self, t):
        s, p, o = t
        return (self.entity_to_id[s], self.relation_to_id[p], self.entity_to_id[o])

    def ids_triples(self, ts):
        return [self.ids_triple(t) for t in ts]

    def printable_triple(self, t):
        s, p, o = self.labels_triple(t)
        return f"<{s}, {p}, {o}>"


class KelpieView:
    """Training rows and rank filter of one subject's kelpie mimic.

    ``kelpie_entity`` = ``num_entities`` (kelpie_dataset.py:20-25).  Filters are
    multisets, exactly like the reference's ``to_filter`` lists where
    ``list.remove`` drops one occurrence (kelpie_dataset.py:145-149)."""

    def __init__(self, dataset: Dataset, entity: int):
        self.dataset = dataset
        self.original_entity = int(entity)
        self.kelpie_entity = dataset.num_entities
        self.num_entities = dataset.num_entities + 1
        k, s = self.kelpie_entity, self.original_entity
        # the entity's training triples as they are now (a snapshot: the dataset may be
        # edited later), as an int32 array with the original entity replaced; the list of
        # tuples (base_triples) is built on first use -- the TransE scheduler never needs it
        self._src = list(dataset.entity_to_training_triples.get(s, []))
        arr = np.fromiter(itertools.chain.from_iterable(self._src), dtype=np.int32,
                          count=3 * len(self._src)).reshape(-1, 3)
        arr[arr[:, 0] == s, 0] = k
        arr[arr[:, 2] == s, 2] = k
        self.base_arr = arr
        self.n_base_rows = 2 * len(self._src)
        self._base_triples = None
        self._filter = self._index = self._base_rows = self._native = None
        self._filter_lists = {}  # rel -> filter_for(rel) without a delta (shared: callers copy or only read)

    @property
    def base_triples(self):
        """The kelpie entity's training triples (tuples, the dataset's order)."""
        if self._base_triples is None:
            k, s = self.kelpie_entity, self.original_entity
            rep = Dataset.replace_entity_in_triple
            self._base_triples = [rep(t, s, k) for t in self._src]
        return self._base_triples

    def _other_triples(self):
        """The kelpie entity's validation and test triples (they only enter the filters)."""
        k, s = self.kelpie_entity, self.original_entity
        rep = Dataset.replace_entity_in_triple
        ds = self.dataset
        return ([rep(t, s, k) for t in ds.entity_to_validation_triples.get(s, [])]
                + [rep(t, s, k) for t in ds.entity_to_testing_triples.get(s, [])])

    @property
    def filter(self):
        """rank key (kelpie, p) -> Counter of filtered objects (train + valid + test)."""
        if self._filter is None:
            k, R = self.kelpie_entity, self.dataset.num_relations
            # only keys whose head is the kelpie entity can be ranked
            f = defaultdict(Counter)
            for a, p, b in self.base_triples + self._other_triples():
                if a == k:
                    f[p][b] += 1
                if b == k:
                    f[p + R][a] += 1
            self._filter = f
        return self._filter

    @property
    def index(self):
        if self._index is None:
            self._index = {t: i for i, t in enumerate(self.base_triples)}
        return self._index

    @property
    def base_rows(self):
        if self._base_rows is None:
            self._base_rows = self._rows(self.base_arr)
        return self._base_rows

    @property
    def native(self):
        """This view in the library's host scheduler (kp_view_create, csrc/kp_sched.cpp)."""
        if self._native is None:
            from . import _lib
            # _other_triples() as an array: the replacement done on the array (same triples,
            # same order) instead of one Python tuple per triple
            ds, k, s = self.dataset, self.kelpie_entity, self.original_entity
            oth = ds.entity_to_validation_triples.get(s, []) + ds.entity_to_testing_triples.get(s, [])
            extra = np.array(oth, dtype=np.int32).reshape(-1, 3)
            extra[extra[:, 0] == s, 0] = k
            extra[extra[:, 2] == s, 2] = k
            self._native = _lib.NativeView(k, ds.num_relations, s, self.base_arr, extra)
        return self._native

    def _rows(self, t):
        """Kelpie rows followed by their inverses (o, p + |R|, s), the optimizers' order
        (pairwise_ranking_optimizer.py:64-65, multiclass_nll_optimizer.py:66-67)."""
        n = len(t)
        out = np.empty((2 * n, 3), np.int32)
        out[:n] = t
        out[n:, 0] = t[:, 2]
        out[n:, 1] = t[:, 1] + self.dataset.num_relations
        out[n:, 2] = t[:, 0]
        return out

    def as_kelpie_triple(self, triple):
        if self.original_entity not in tuple(triple):
            raise Exception(f"Could not find the original entity {self.original_entity} "
                            f"in the passed triple {tuple(triple)}")
        return Dataset.replace_entity_in_triple(tuple(triple), self.original_entity, self.kelpie_entity)

    def filter_for(self, rel, delta=None):
        """Filtered-out entities of key (kelpie, rel), after an optional multiset delta
        (the multiset's insertion order: base entities first, then the delta's new ones)."""
        base = self.filter.get(rel)
        if not delta:
            if base is None:
                return []
            cached = self._filter_lists.get(rel)
            if cached is None:
                cached = self._filter_lists[rel] = [e for e, n in base.items() if n > 0]
            return cached
        base = base or {}
        out = [e for e, n in base.items() if n + delta.get(e, 0) > 0]
        out += [e for e, n in delta.items() if e not in base and n > 0]
        return out

    def _delta(self, conv, sign):
        k = self.kelpie_entity
        R = self.dataset.num_relations
        d = {}
        for a, p, b in conv:
            if a == k:
                dp = d.setdefault(p, {})
                dp[b] = dp.get(b, 0) + sign
            if b == k:
                dp = d.setdefault(p + R, {})
                dp[a] = dp.get(a, 0) + sign
        return d

    def removed(self, triples, rows=True):
        """Rows and filter delta after ``remove_training_triples`` (kelpie_dataset.py:130-158).
        ``rows=False``: the row COUNT instead of the rows (same checks and errors), for
        a slot another rank post-trains (kelpie_amd.distributed)."""
        for s, _, o in triples:
            assert self.original_entity == s or self.original_entity == o
        conv = [Dataset.replace_entity_in_triple(tuple(t), self.original_entity, self.kelpie_entity)
                for t in triples]
        idx = [self.index[x] for x in conv]  # KeyError for a foreign triple, like the reference
        delta = self._delta(conv, -1)
        for rel, cnt in delta.items():
            cur = self.filter.get(rel, {})
            for e, n in cnt.items():
                if cur.get(e, 0) + n < 0:
                    raise ValueError("list.remove(x): x not in list")
        if not rows:
            return 2 * (len(self.base_triples) - len(set(idx))), delta
        keep = np.ones(len(self.base_triples), dtype=bool)
        keep[idx] = False
        return self._rows(self.base_arr[keep]), delta

    def added(self, triples, rows=True):
        """Rows and filter delta after ``add_training_triples`` (kelpie_dataset.py:92-128)
        (``rows=False``: the row count, as :meth:`removed`)."""
        for s, _, o in triples:
            assert self.original_entity == s or self.original_entity == o
        conv = [Dataset.replace_entity_in_triple(tuple(t), self.original_entity, self.kelpie_entity)
                for t in triples]
        if not rows:
            return 2 * (len(self.base_triples) + len(conv)), None  # additions cannot fail
        rows = np.concatenate([self.base_arr, np.asarray(conv, dtype=np.int32).reshape(-1, 3)])
        return self._rows(rows), self._delta(conv, +1)

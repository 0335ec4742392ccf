"""Seeded synthetic knowledge graphs and model weights shaped like the reference datasets.

The reference's large training files (FB15k-237, YAGO3-10, DB100K) are absent
from the image and its trained checkpoints are a figshare download
(SURVEY.md §0 finding 2), so benchmarks and parity fixtures run on graphs drawn
from published dataset statistics (SURVEY.md §8(d) "Synthetic inputs"):
Zipf-like entity popularity ``p_i ∝ i^-0.8``, uniform relations, deduplicated,
then split train / valid / test.  Weights follow the reference initialisers
(TransE / ConvE ``xavier_normal_``: ``transe.py:30-35``, ``conve.py:54-59``;
ComplEx ``U[0,1)·init_scale``: ``complex.py:27-35``).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

# (entities, relations, train, valid, test) -- published dataset statistics
SHAPES = {
    "FB15k-237": (14541, 237, 272115, 17535, 20466),
    "DB100K": (99604, 470, 597572, 50000, 50000),
    "YAGO3-10": (123182, 37, 1079040, 5000, 5000),
    "tiny": (300, 12, 2400, 120, 120),
    "small": (2000, 40, 20000, 600, 600),
}


@dataclass
class SynthGraph:
    name: str
    num_entities: int
    num_relations: int
    train: np.ndarray  # int64 [n,3]
    valid: np.ndarray
    test: np.ndarray


def make_graph(shape: str = "FB15k-237", seed: int = 0, n_ent=None, n_rel=None,
               n_train=None, n_valid=None, n_test=None, zipf: float = 0.8) -> SynthGraph:
    base = SHAPES[shape]
    n_ent = n_ent or base[0]
    n_rel = n_rel or base[1]
    n_train = n_train or base[2]
    n_valid = n_valid if n_valid is not None else base[3]
    n_test = n_test if n_test is not None else base[4]
    rng = np.random.default_rng(seed)
    pop = np.arange(1, n_ent + 1, dtype=np.float64) ** (-zipf)
    pop /= pop.sum()
    # popularity rank -> entity id is a random permutation
    perm = rng.permutation(n_ent)
    want = n_train + n_valid + n_test
    chunks = []
    have = 0
    seen = set()
    while have < want:
        m = int((want - have) * 1.3) + 64
        h = perm[rng.choice(n_ent, size=m, p=pop)]
        t = perm[rng.choice(n_ent, size=m, p=pop)]
        r = rng.integers(0, n_rel, size=m)
        keep = h != t
        trip = np.stack([h, r, t], axis=1)[keep]
        keys = trip[:, 0] * (n_rel * n_ent) + trip[:, 1] * n_ent + trip[:, 2]
        _, first = np.unique(keys, return_index=True)
        first.sort()
        out = []
        for i in first:
            k = int(keys[i])
            if k in seen:
                continue
            seen.add(k)
            out.append(i)
            if have + len(out) >= want:
                break
        chunks.append(trip[out])
        have += len(out)
    allt = np.concatenate(chunks)[:want].astype(np.int64)
    rng.shuffle(allt, axis=0)
    train = allt[:n_train]
    rest = allt[n_train:]
    # like PyKEEN, drop valid/test triples whose entities never occur in train
    seen_e = np.zeros(n_ent, dtype=bool)
    seen_e[train[:, 0]] = True
    seen_e[train[:, 2]] = True
    rest = rest[seen_e[rest[:, 0]] & seen_e[rest[:, 2]]]
    valid = rest[:n_valid]
    test = rest[n_valid:n_valid + n_test]
    return SynthGraph(shape, n_ent, n_rel, train, valid, test)


def xavier_normal(rng: np.random.Generator, rows: int, cols: int) -> np.ndarray:
    std = np.sqrt(2.0 / (rows + cols))
    return (rng.standard_normal((rows, cols)) * std).astype(np.float32)


def make_weights(model: str, n_ent: int, n_rel: int, dim: int, seed: int = 0,
                 init_scale: float = 1e-3, conve_random_bn: bool = False, trained_scale=None):
    """Random-init weights of the reference architectures.

    Returns a dict with ``entity_embeddings`` [n_ent, D] and
    ``relation_embeddings`` [2*n_rel, D] (inverse relations live at p+|R|,
    ``transe.py:23``), plus the frozen ConvE layers when ``model == "ConvE"``.
    ``trained_scale`` replaces the initialiser by N(0, trained_scale) tables,
    which look more like trained embeddings (scores of order 1) than the raw
    initialisers do; the parity fixtures use it.
    """
    rng = np.random.default_rng(seed)
    R2 = 2 * n_rel
    if model == "TransE":
        return {"entity_embeddings": xavier_normal(rng, n_ent, dim),
                "relation_embeddings": xavier_normal(rng, R2, dim)}
    if model == "ComplEx" and trained_scale:
        D = 2 * dim
        return {"entity_embeddings": (rng.standard_normal((n_ent, D)) * trained_scale).astype(np.float32),
                "relation_embeddings": (rng.standard_normal((R2, D)) * trained_scale).astype(np.float32)}
    if model == "ComplEx":
        D = 2 * dim
        return {"entity_embeddings": (rng.random((n_ent, D)) * init_scale).astype(np.float32),
                "relation_embeddings": (rng.random((R2, D)) * init_scale).astype(np.float32)}
    if model == "ConvE":
        if trained_scale:
            w = {"entity_embeddings": (rng.standard_normal((n_ent, dim)) * trained_scale).astype(np.float32),
                 "relation_embeddings": (rng.standard_normal((R2, dim)) * trained_scale).astype(np.float32)}
        else:
            w = {"entity_embeddings": xavier_normal(rng, n_ent, dim),
                 "relation_embeddings": xavier_normal(rng, R2, dim)}
        h = dim // 20
        hid = 32 * (2 * 20 - 2) * (h - 2)
        # torch default init for Conv2d(1,32,3) / Linear(hid, dim): U(-1/sqrt(fan_in), ..)
        bc = 1.0 / np.sqrt(9.0)
        w["conv_weight"] = rng.uniform(-bc, bc, size=(32, 1, 3, 3)).astype(np.float32)
        w["conv_bias"] = rng.uniform(-bc, bc, size=(32,)).astype(np.float32)
        bf = 1.0 / np.sqrt(hid)
        w["fc_weight"] = rng.uniform(-bf, bf, size=(dim, hid)).astype(np.float32)
        w["fc_bias"] = rng.uniform(-bf, bf, size=(dim,)).astype(np.float32)
        for name, c in (("bn1", 1), ("bn2", 32), ("bn3", dim)):
            if conve_random_bn:
                w[f"{name}_weight"] = rng.uniform(0.5, 1.5, size=(c,)).astype(np.float32)
                w[f"{name}_bias"] = rng.uniform(-0.2, 0.2, size=(c,)).astype(np.float32)
                w[f"{name}_mean"] = rng.uniform(-0.1, 0.1, size=(c,)).astype(np.float32)
                w[f"{name}_var"] = rng.uniform(0.5, 1.5, size=(c,)).astype(np.float32)
            else:
                w[f"{name}_weight"] = np.ones(c, np.float32)
                w[f"{name}_bias"] = np.zeros(c, np.float32)
                w[f"{name}_mean"] = np.zeros(c, np.float32)
                w[f"{name}_var"] = np.ones(c, np.float32)
        return w
    raise ValueError(model)

"""Link-prediction evaluation: the reference's ``Evaluator``
(``src/link_prediction/evaluation.py:11-89``) over the device's filtered ranks
(``FrozenModel.predict_triples`` -> ``kp_predict_tails``).  Same metrics (MRR,
Hits@1, Hits@10, MR over tail and head ranks) and the same ``ranks.csv`` output.
"""
from __future__ import annotations

import csv
import html

import numpy as np


class Evaluator:
    def __init__(self, model):
        self.model = model
        self.dataset = model.dataset

    def evaluate(self, triples, write_output: bool = False, output_path: str = "ranks.csv"):
        triples = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
        results = self.model.predict_triples(triples)  # one device pass (the reference batches by 256)
        ranks = [r["rank"] for r in results]
        if write_output:
            self.write_output(triples, ranks, output_path)
        all_ranks = []
        for i in range(triples.shape[0]):
            all_ranks.append(results[i]["rank"]["tail"])
            all_ranks.append(results[i]["rank"]["head"])
        return {"mrr": self.mrr(all_ranks), "h1": self.hits_at(all_ranks, 1), "h10": self.hits_at(all_ranks, 10),
                "mr": self.mr(all_ranks)}

    def write_output(self, triples, ranks, path="ranks.csv"):
        """evaluation.py:50-72: ``;``-separated head, relation, tail, head_rank, tail_rank."""
        with open(path, "w", newline="") as f:
            w = csv.writer(f, delimiter=";")
            w.writerow(["head", "relation", "tail", "head_rank", "tail_rank"])
            for (s, p, o), r in zip(triples.tolist(), ranks):
                w.writerow([html.unescape(self.dataset.id_to_entity[s]), html.unescape(self.dataset.id_to_relation[p]),
                            html.unescape(self.dataset.id_to_entity[o]), r["head"], r["tail"]])

    @staticmethod
    def mrr(values):
        mrr = 0.0
        for value in values:
            mrr += 1.0 / float(value)
        return mrr / float(len(values))

    @staticmethod
    def mr(values):
        return np.average(values)

    @staticmethod
    def hits_at(values, k: int):
        hits = 0
        for value in values:
            if value <= k:
                hits += 1
        return float(hits) / float(len(values))

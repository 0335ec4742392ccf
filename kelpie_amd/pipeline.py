"""Explanation pipelines and the on-disk formats around them.

Mirrors the reference's callers of the relevance engine:

* ``NecessaryPipeline`` / ``SufficientPipeline`` (src/pipeline.py:4-47) and
  ``build_pipeline`` (src/explain.py:49-89, the post-training branch): prefilter
  -> ``StochasticBuilder`` over the MI355X engine;
* ``read_preds`` (explain.py:159-163): one tab-separated label triple per line;
* ``explain_preds`` / ``write_explanations`` (explain.py:190-203): the
  ``output.json`` list of ``{"triple", "rule_to_relevance", "#relevances",
  "execution_time"[, "entities_to_convert"]}`` records, rewritten after every
  prediction as the reference does.

The DP / CRIAGE baselines and summarisation are out of scope.
"""
from __future__ import annotations

import json

from .builder import StochasticBuilder
from .engine import NecessaryPostTrainingEngine, PostTrainingEngine, SufficientPostTrainingEngine
from .prefilters import PREFILTERS, TOPOLOGY_PREFILTER, TYPE_PREFILTER, TopologyPreFilter


class Pipeline:
    def __init__(self, dataset, prefilter, builder):
        self.dataset = dataset
        self.prefilter = prefilter
        self.builder = builder
        self.engine = self.builder.engine
        self.model = self.engine.model

    def explain(self, pred, prefilter_k=-1):
        if isinstance(self.engine, PostTrainingEngine):
            self.engine.set_cache()
        return self.prefilter.select_triples(pred=pred, k=prefilter_k)


class NecessaryPipeline(Pipeline):
    def explain(self, pred, prefilter_k=-1):
        filtered_triples = super().explain(pred=pred, prefilter_k=prefilter_k)
        return self.builder.build_explanations(pred, filtered_triples)


class SufficientPipeline(Pipeline):
    def explain(self, pred, prefilter_k=50, to_convert_k=10):
        filtered_triples = super().explain(pred, prefilter_k)
        self.engine.select_entities_to_convert(pred, to_convert_k, 200)
        result = self.builder.build_explanations(pred, filtered_triples)
        result["entities_to_convert"] = [self.dataset.id_to_entity[x] for x in self.engine.entities_to_convert]
        return result


def build_pipeline(model, dataset, hp, mode, prefilter=None, xsi=None, window=32, entity_classes=None):
    """explain.py:49-89 for the post-training engines (baseline=None, no summarisation)."""
    if prefilter == TYPE_PREFILTER:
        raise NotImplementedError("type_based prefilter: out of scope (kelpie_amd/prefilters.py)")
    cls = PREFILTERS.get(prefilter, TopologyPreFilter) if prefilter else PREFILTERS[TOPOLOGY_PREFILTER]
    pf = cls(dataset, entity_classes) if entity_classes is not None and "Weighted" in cls.__name__ else cls(dataset)
    if mode == "necessary":
        xsi = 5 if xsi is None else xsi
        engine = NecessaryPostTrainingEngine(model, dataset, hp)
        return NecessaryPipeline(dataset, pf, StochasticBuilder(xsi, engine, window=window))
    if mode == "sufficient":
        xsi = 0.9 if xsi is None else xsi
        engine = SufficientPostTrainingEngine(model, dataset, hp)
        return SufficientPipeline(dataset, pf, StochasticBuilder(xsi, engine, window=window))
    raise ValueError(f"unknown mode {mode!r}")


def read_preds(path):
    """explain.py:162-163: ``[x.strip().split("\\t") for x in lines]``."""
    with open(path, "r") as f:
        return [x.strip().split("\t") for x in f.readlines()]


def write_explanations(path, explanations):
    with open(path, "w") as f:
        json.dump(explanations, f)


def explain_preds(pipeline, dataset, preds, prefilter_k, skip=-1, output_path=None):
    """The loop of explain.py:190-203: label triples -> ids -> pipeline.explain;
    predictions with index <= skip are skipped; ``output.json`` is rewritten after
    each prediction when ``output_path`` is given."""
    explanations = []
    for i, pred in enumerate(preds):
        if i <= skip:
            continue
        ids = dataset.ids_triple(pred)
        explanations.append(pipeline.explain(pred=ids, prefilter_k=prefilter_k))
        if output_path is not None:
            write_explanations(output_path, explanations)
    return explanations

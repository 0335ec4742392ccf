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


def build_pipeline(model, dataset, hp, mode, prefilter=None, xsi=None, window="auto", entity_classes=None,
                   pipelined=False):
    """explain.py:49-89 for the post-training engines (baseline=None, no summarisation)."""
    if prefilter == TYPE_PREFILTER:
        raise NotImplementedError("type_based prefilter: out of scope (kelpie_amd/prefilters.py)")
    cls = PREFILTERS.get(prefilter, TopologyPreFilter) if prefilter else PREFILTERS[TOPOLOGY_PREFILTER]
    pf = cls(dataset, entity_classes) if entity_classes is not None and "Weighted" in cls.__name__ else cls(dataset)
    if mode == "necessary":
        xsi = 5 if xsi is None else xsi
        engine = NecessaryPostTrainingEngine(model, dataset, hp)
        return NecessaryPipeline(dataset, pf, StochasticBuilder(xsi, engine, window=window, pipelined=pipelined))
    if mode == "sufficient":
        xsi = 0.9 if xsi is None else xsi
        engine = SufficientPostTrainingEngine(model, dataset, hp)
        return SufficientPipeline(dataset, pf, StochasticBuilder(xsi, engine, window=window, pipelined=pipelined))
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


def reference_construction_draws(model_name, num_entities, num_relations, model_params):
    """Consume the process-global torch CPU generator exactly as the reference's
    ``model_class(dataset=..., hp=..., init_random=True)`` does in explain.py:171-172,
    before ``load_state_dict`` overwrites the tables (the reference run on CPU: ``.cuda()``
    copies, so the xavier draws come from the CPU generator as well):

    * TransE (transe.py:27-32): ``torch.rand(|E|, d)``, ``torch.rand(2|R|, d)``, then
      ``xavier_normal_`` on both;
    * ComplEx (complex.py:27-31): ``torch.rand(|E|, 2d)``, ``torch.rand(2|R|, 2d)``;
    * ConvE (conve.py:44-61): the ``Conv2d(1, 32, 3x3)`` and ``Linear(hidden, d)``
      ``reset_parameters`` draws, then as TransE.

    The values are discarded; only the generator state matters (every later draw of the
    run -- kelpie inits, permutations, negatives, dropout masks -- follows it)."""
    import torch
    n_rel2 = 2 * int(num_relations)
    if model_name == "ComplEx":
        d = 2 * int(model_params["dimension"])
        torch.rand(int(num_entities), d)
        torch.rand(n_rel2, d)
        return
    d = int(model_params["dimension"])
    if model_name == "ConvE":
        torch.nn.Conv2d(1, 32, (3, 3), 1, 0, bias=True)
        torch.nn.Linear(int(model_params["hidden_layer_size"]), d)
    elif model_name != "TransE":
        raise ValueError(model_name)
    e = torch.rand(int(num_entities), d)
    r = torch.rand(n_rel2, d)
    torch.nn.init.xavier_normal_(e)
    torch.nn.init.xavier_normal_(r)


def run_explain(model_name, dataset, state, model_params, hp, mode, preds, prefilter=None, prefilter_k=20,
                xsi=None, skip=-1, output_path=None, device=0):
    """explain.py main() (explain.py:143-203) without the CLI: seeds 42 (explain.py:144),
    the reference model construction's random draws (:171-172), the checkpoint state dict
    (``torch.load(path, weights_only=True)``, :174) as a frozen model on the MI355X, the
    pipeline (:177-186) and the loop over ``preds`` writing ``output.json``."""
    import random

    import numpy as np
    import torch

    from .models import from_state_dict
    random.seed(42)
    np.random.seed(42)
    torch.manual_seed(42)
    reference_construction_draws(model_name, dataset.num_entities, dataset.num_relations, model_params)
    model = from_state_dict(model_name, dataset, state, model_params, device=device)
    pipe = build_pipeline(model, dataset, hp, mode, prefilter=prefilter, xsi=xsi)
    return explain_preds(pipe, dataset, preds, prefilter_k=prefilter_k, skip=skip, output_path=output_path)

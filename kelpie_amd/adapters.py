"""Adapters from the reference's in-memory objects to kelpie_amd (drop-in glue).

A maintainer of the reference swaps its engines for ours in
``src/explain.py:build_pipeline`` (``explain.py:70,85``) with

    from kelpie_amd.adapters import necessary_engine, sufficient_engine
    engine = necessary_engine(model, dataset, hp)      # was NecessaryPostTrainingEngine(...)

The adapters read only public attributes (duck typing): the reference
``Dataset``'s id triples, label maps and ``num_*`` counts
(``src/data/dataset.py:143-186``) and the model's tensors
(``entity_embeddings``, ``relation_embeddings``, the ConvE layers and
hyper-parameters, ``src/link_prediction/models/*.py``).  Nothing from the
reference is imported.
"""
from __future__ import annotations

import numpy as np

from .data import Dataset
from .engine import NecessaryPostTrainingEngine, SufficientPostTrainingEngine
from .models import ComplEx, ConvE, TransE


def _np(t):
    return t.detach().cpu().numpy() if hasattr(t, "detach") else np.asarray(t)


def dataset_from_reference(ref_dataset) -> Dataset:
    return Dataset(ref_dataset.num_entities, ref_dataset.num_relations, _np(ref_dataset.training_triples),
                   _np(ref_dataset.validation_triples), _np(ref_dataset.testing_triples),
                   name=getattr(ref_dataset, "name", "reference"),
                   entity_to_id=dict(ref_dataset.entity_to_id), relation_to_id=dict(ref_dataset.relation_to_id))


def model_from_reference(ref_model, dataset: Dataset, device=0):
    name = ref_model.name
    E, R = _np(ref_model.entity_embeddings), _np(ref_model.relation_embeddings)
    if name == "ComplEx":
        return ComplEx(dataset, E, R, init_scale=ref_model.init_scale, device=device)
    if name == "TransE":
        return TransE(dataset, E, R, norm=ref_model.norm, device=device)
    if name == "ConvE":
        bn = {}
        for i in (1, 2, 3):
            m = getattr(ref_model, f"batch_norm_{i}")
            bn[i] = {"weight": _np(m.weight), "bias": _np(m.bias), "running_mean": _np(m.running_mean),
                     "running_var": _np(m.running_var)}
        return ConvE(dataset, E, R, _np(ref_model.convolutional_layer.weight).reshape(32, 3, 3),
                     _np(ref_model.convolutional_layer.bias), _np(ref_model.hidden_layer.weight),
                     _np(ref_model.hidden_layer.bias), bn=bn, input_dropout_rate=ref_model.input_dropout_rate,
                     feature_map_dropout_rate=ref_model.feature_map_dropout_rate,
                     hidden_dropout_rate=ref_model.hidden_dropout_rate, device=device)
    raise ValueError(f"unsupported model {name}")


def necessary_engine(ref_model, ref_dataset, hp, device=0):
    ds = dataset_from_reference(ref_dataset)
    return NecessaryPostTrainingEngine(model_from_reference(ref_model, ds, device), ds, hp)


def sufficient_engine(ref_model, ref_dataset, hp, device=0):
    ds = dataset_from_reference(ref_dataset)
    return SufficientPostTrainingEngine(model_from_reference(ref_model, ds, device), ds, hp)

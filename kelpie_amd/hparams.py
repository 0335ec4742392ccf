"""Hyper-parameter records with the reference's fields, types and errors.

The reference turns its hp dicts into Pydantic models before it uses them:

* optimizer hp, per post-training (``post_training_engine.py:71``:
  ``optimizer_class.get_hyperparams_class()(**self.hp)``):
  ``MultiClassNLLOptimizerHyperParams`` (``multiclass_nll_optimizer.py:16-24``, ComplEx),
  ``PairwiseRankingOptimizerHyperParams`` (``pairwise_ranking_optimizer.py:19-25``, TransE),
  ``BCEOptimizerHyperParams`` (``bce_optimizer.py:17-22``, ConvE);
* model params, when the model is built (``explain.py:169-172``):
  ``TransEHyperParams`` (``transe.py:12-14``), ``ComplExHyperParams`` (``complex.py:12-14``),
  ``ConvEHyperParams`` (``conve.py:15-20``).

The same classes here give the same behaviour: a missing field or a value of the wrong
type raises ``pydantic.ValidationError`` (a ``ValueError``) naming the field, values are
coerced as Pydantic's default (lax) mode coerces them (``"43"`` -> 43), and keys the class
does not declare are ignored.  The engine validates its hp when it is constructed, so a
malformed config fails before any device work instead of as a ``KeyError`` deep inside
the slot assembly.
"""
from __future__ import annotations

from pydantic import BaseModel


class MultiClassNLLOptimizerHyperParams(BaseModel):
    optimizer_name: str
    batch_size: int
    epochs: int
    lr: float
    decay1: float
    decay2: float
    regularizer_name: str
    regularizer_weight: float


class PairwiseRankingOptimizerHyperParams(BaseModel):
    batch_size: int
    epochs: int
    lr: float
    margin: float
    negative_triples_ratio: int
    regularizer_weight: float


class BCEOptimizerHyperParams(BaseModel):
    batch_size: int
    label_smoothing: float
    lr: float
    decay: float
    epochs: int


class TransEHyperParams(BaseModel):
    dimension: int
    norm: int


class ComplExHyperParams(BaseModel):
    dimension: int
    init_scale: float


class ConvEHyperParams(BaseModel):
    dimension: int
    input_dropout_rate: float
    feature_map_dropout_rate: float
    hidden_dropout_rate: float
    hidden_layer_size: int


# MODEL_REGISTRY[name]["optimizer"].get_hyperparams_class() (link_prediction/__init__.py)
OPTIMIZER_HP = {"ComplEx": MultiClassNLLOptimizerHyperParams, "TransE": PairwiseRankingOptimizerHyperParams,
                "ConvE": BCEOptimizerHyperParams}
MODEL_HP = {"ComplEx": ComplExHyperParams, "TransE": TransEHyperParams, "ConvE": ConvEHyperParams}


def optimizer_hp(model_name: str, hp: dict) -> dict:
    """``hp`` validated against the model's optimizer hp class: the declared fields,
    coerced to their types, plus any other keys unchanged (the reference passes the
    same dict on)."""
    cls = OPTIMIZER_HP[model_name]
    return {**dict(hp), **cls(**hp).model_dump()}


def model_params(model_name: str, params: dict) -> dict:
    """``params`` validated against the model's hp class (explain.py:169-170)."""
    cls = MODEL_HP[model_name]
    return {**dict(params), **cls(**params).model_dump()}

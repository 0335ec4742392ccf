"""kelpie_amd -- MI355X-native relevance engine for Kelpie explanations.

Drop-in for the reference's post-training relevance path
(src/relevance_engines/post_training_engine.py and the explanation builder's
inner loop); the arithmetic runs in the gfx950 HIP library libkelpie_hip.so
(C ABI in include/kelpie_hip.h).
"""
from .data import Dataset, KelpieView  # noqa: F401
from .engine import NecessaryPostTrainingEngine, PostTrainingEngine, SufficientPostTrainingEngine  # noqa: F401
from .models import MODEL_REGISTRY, ComplEx, ConvE, TransE, from_state_dict  # noqa: F401
from .builder import StochasticBuilder  # noqa: F401
from .prefilters import NoPreFilter, TopologyPreFilter, WeightedTopologyPreFilter  # noqa: F401
from .baselines import (CriagePreFilter, NecessaryCriageEngine, NecessaryDPEngine, SufficientCriageEngine,  # noqa: F401
                        SufficientDPEngine)
from .pipeline import NecessaryPipeline, SufficientPipeline, build_pipeline, explain_preds, read_preds  # noqa: F401

__version__ = "0.1.0"

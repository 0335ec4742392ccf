"""Import harness for the read-only Python reference (fixture generation only).

This file is TEST INFRASTRUCTURE.  It is used by ``make_golden.py`` in the
development container to run the reference relevance engine on CPU and capture
golden vectors.  Nothing in ``kelpie_amd`` imports it, and it is never executed
on the GPU box (``/root/reference`` does not exist there).

What it does (no reference source is copied):

* registers placeholder modules for three imports the reference makes at module
  load time but that are absent from this image and are not on the relevance
  path: ``pykeen`` (only ``get_dataset`` is used, by ``src/data/dataset.py:97``;
  our stub serves an in-memory triple set), ``optuna`` (only
  ``optuna.exceptions.TrialPruned`` is referenced by the optimizers' ``train``
  early-stopping branches) and ``bispy`` (bisimulation summarisation, not used);
* redirects the reference's hard-coded ``.cuda()`` / ``device="cuda"`` sites
  to CPU.  ``Tensor.cuda`` becomes ``clone()`` (the GPU path copies, and
  ``transe.py:93-95`` / ``complex.py:155-157`` mutate that copy in place);
* seeds torch / numpy / random directly (``utils/utils.py:16-21`` would touch
  ``torch.cuda``).
"""
from __future__ import annotations

import os
import random
import sys
import types

import numpy as np
import torch
from torch.overrides import TorchFunctionMode

REF_ROOT = os.environ.get("KELPIE_REFERENCE", "/root/reference")


# --------------------------------------------------------------------------
# in-memory dataset served through the pykeen.get_dataset placeholder
# --------------------------------------------------------------------------
class _Split:
    def __init__(self, triples: np.ndarray):
        self.mapped_triples = torch.as_tensor(np.asarray(triples, dtype=np.int64).reshape(-1, 3))


class _MemDataset:
    def __init__(self, n_ent, n_rel, train, valid, test, entity_to_id=None, relation_to_id=None):
        self.num_entities = int(n_ent)
        self.num_relations = int(n_rel)
        self.entity_to_id = entity_to_id or {f"e{i:06d}": i for i in range(n_ent)}
        self.relation_to_id = relation_to_id or {f"r{i:04d}": i for i in range(n_rel)}
        self.training = _Split(train)
        self.validation = _Split(valid)
        self.testing = _Split(test)


_REGISTRY: dict[str, _MemDataset] = {}


def register_dataset(name, n_ent, n_rel, train, valid, test, entity_to_id=None, relation_to_id=None):
    _REGISTRY[name] = _MemDataset(n_ent, n_rel, train, valid, test, entity_to_id, relation_to_id)


def _get_dataset(dataset=None, **kwargs):
    return _REGISTRY[dataset]


def _install_stubs():
    pk = types.ModuleType("pykeen")
    pkd = types.ModuleType("pykeen.datasets")
    pkd.get_dataset = _get_dataset
    pk.datasets = pkd
    sys.modules.setdefault("pykeen", pk)
    sys.modules.setdefault("pykeen.datasets", pkd)

    op = types.ModuleType("optuna")
    ope = types.ModuleType("optuna.exceptions")

    class TrialPruned(Exception):
        pass

    ope.TrialPruned = TrialPruned
    op.exceptions = ope
    sys.modules.setdefault("optuna", op)
    sys.modules.setdefault("optuna.exceptions", ope)

    bp = types.ModuleType("bispy")
    bp.compute_maximum_bisimulation = lambda *a, **k: []
    sys.modules.setdefault("bispy", bp)


class _CpuDeviceMode(TorchFunctionMode):
    """Rewrites device='cuda' keyword arguments to CPU (bce_optimizer.py:102,112)."""

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        dev = kwargs.get("device", None)
        if dev is not None and "cuda" in str(dev):
            kwargs = dict(kwargs)
            kwargs["device"] = "cpu"
        return func(*args, **kwargs)


_MODE = None


def _install_cpu_redirect():
    global _MODE
    torch.Tensor.cuda = lambda self, *a, **k: self.clone()
    torch.nn.Module.cuda = lambda self, *a, **k: self
    _orig_to = torch.nn.Module.to

    def _to(self, *args, **kwargs):
        if args and isinstance(args[0], (str, torch.device)) and "cuda" in str(args[0]):
            return self
        return _orig_to(self, *args, **kwargs)

    torch.nn.Module.to = _to
    _MODE = _CpuDeviceMode()
    _MODE.__enter__()


def load_reference():
    """Return the imported reference ``src`` package (CPU-redirected)."""
    if not os.path.isdir(os.path.join(REF_ROOT, "src")):
        raise RuntimeError(f"reference not found at {REF_ROOT}")
    sys.dont_write_bytecode = True
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    _install_stubs()
    _install_cpu_redirect()
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    import src  # noqa: F401
    import src.data  # noqa: F401
    import src.link_prediction  # noqa: F401
    import src.relevance_engines  # noqa: F401
    import src.explanation_builders  # noqa: F401
    return sys.modules["src"]


def seed_all(seed: int = 42):
    """Same three seeds as ``explain.py:144`` (without the torch.cuda touch)."""
    np.random.seed(seed)
    torch.manual_seed(seed)
    random.seed(seed)

"""Relevances of a few ConvE YAGO3-10-shape (d = 200) predictions, saved for a bitwise
comparison between two library builds (GPU box):

    KELPIE_HIP_LIB=<lib> python tools/conve_bitwise.py <out.npy>
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import bench  # noqa: E402


def main():
    import random

    import torch
    from kelpie_amd import NecessaryPostTrainingEngine
    wl = bench.WORKLOADS["conve-yago310-necessary"]
    ds, model, _ = bench.build(wl, 0, 0)
    eng = NecessaryPostTrainingEngine(model, ds, wl["hp"])
    preds = bench.pick_preds(ds, 2, seed=1234)
    random.seed(42)
    np.random.seed(42)
    torch.manual_seed(42)
    items = [(p, [[c] for c in bench.candidates_of(ds, p, 8)]) for p in preds]
    out = eng.compute_relevance_multi(items)
    vals = np.array([float(v) for r in out for v in r], dtype=np.float64)
    np.save(sys.argv[1], vals)
    print("relevances", vals.size, vals[:4])


if __name__ == "__main__":
    main()

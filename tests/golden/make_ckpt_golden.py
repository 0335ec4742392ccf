"""Reference checkpoints for the f1 ``.pt`` loader (development container only).

For three golden cases the reference model is built exactly as make_golden.py builds
it (same seeded weights), saved with ``torch.save(model.state_dict())`` (the format of
the reference's ``models/*.pt``, loaded at explain.py:169-176), and its ``all_scores``
on the first test triples is recorded.  Output: tests/golden/ckpt_<name>.pt and
tests/golden/ckpt_golden.json.  The .pt files are plain tensors (the test loads them
with ``torch.load(..., weights_only=True)``).

    python tests/golden/make_ckpt_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import ref_harness  # noqa: E402
from make_golden import CASES, build_case  # noqa: E402

NAMES = ["complex_tiny", "transe_tiny", "conve60_tiny"]


def main():
    src = ref_harness.load_reference()
    out = {}
    for name in NAMES:
        g, _, dataset, model = build_case(src, name, CASES[name])
        path = os.path.join(HERE, f"ckpt_{name}.pt")
        torch.save(model.state_dict(), path)
        trip = np.asarray(g.test[:6], dtype=np.int64)
        with torch.no_grad():
            sc = model.all_scores(trip).detach().cpu().numpy()
        out[name] = {"keys": sorted(model.state_dict().keys()), "triples": trip.tolist(),
                     "all_scores": sc.astype(np.float64).tolist()}
        print(name, out[name]["keys"], sc.shape, flush=True)
    with open(os.path.join(HERE, "ckpt_golden.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()

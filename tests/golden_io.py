"""Loader for the golden fixtures under tests/golden (data only)."""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["transe_tiny", "complex_tiny", "complex_adam_tiny", "conve_tiny", "conve60_tiny", "complex200_small",
         "transe200_small", "conve_drop_tiny", "conve60_drop_tiny", "complex_n3_tiny", "complex_n2_tiny",
         "transe_l1_tiny", "complex200_n3_small"]


def load_case(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        rec = json.load(f)
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    arrays = {k: z[k] for k in z.files}
    if rec.get("regenerated"):
        from kelpie_amd import synth
        a = rec["weights_args"]
        w = synth.make_weights(rec["model"], rec["num_entities"], rec["num_relations"], a["dim"],
                               seed=rec["weights_seed"], conve_random_bn=a["conve_random_bn"],
                               trained_scale=a["trained_scale"])
        for k, digest in rec["regenerated"].items():
            v = np.ascontiguousarray(w[k])
            assert hashlib.sha256(v.tobytes()).hexdigest() == digest, f"regenerated {k} differs"
            arrays[k] = v
    weights = {k: v for k, v in arrays.items() if k not in ("train", "valid", "test")}
    return rec, arrays, weights


def seed_all(seed=42):
    import random
    import torch
    np.random.seed(seed)
    torch.manual_seed(seed)
    random.seed(seed)

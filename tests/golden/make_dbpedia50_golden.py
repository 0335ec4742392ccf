"""Golden run of BASELINE.json configs[0] on REAL data: TransE on DBpedia50, necessary
mode, the first 10 predictions of ``preds/TransE_DBpedia50.csv``, the reference's own
explanation config ``configs/TransE_DBpedia50_explanation.json`` (d = 256, 65 epochs),
through the reference's whole pipeline (``explain.py:159-203``: topology prefilter,
k = 20, StochasticBuilder, xsi 5).

TEST INFRASTRUCTURE, development container only (reads /root/reference).  The label ->
id maps come from ``kelpie_amd.Dataset.from_directory`` (sorted training labels, the
PyKEEN ``TriplesFactory.from_path`` rule) and are served to the reference through the
``get_dataset`` placeholder of ``ref_harness``, so both sides index the same triples.
Trained checkpoints are not available offline (figshare download): the weights are
seeded random (``kelpie_amd.synth.make_weights``, TransE xavier init), regenerated at
test time from the seed and checked by sha256.  The preds file is copied as data.

    python tests/golden/make_dbpedia50_golden.py
writes tests/golden/dbpedia50_transe.json (+ dbpedia50_preds.tsv)

    python tests/golden/make_dbpedia50_golden.py --fp64
runs the same pipeline with the reference model in float64 (``tools/conditioning.py``'s
patches: the random draws made in float32 as the fp32 run makes them, then widened) and
writes tests/golden/dbpedia50_transe_fp64.json: the second reference variant of the
element-wise rule (tests/test_dbpedia50.py).
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import ref_harness  # noqa: E402
from kelpie_amd import Dataset, synth  # noqa: E402

N_PREDS = 10
SEED = 2024


def main():
    fp64 = "--fp64" in sys.argv[1:]
    src = ref_harness.load_reference()
    ref = ref_harness.REF_ROOT
    ds = Dataset.from_directory(os.path.join(ref, "data", "DBpedia50"))
    with open(os.path.join(ref, "configs", "TransE_DBpedia50_explanation.json")) as f:
        cfg = json.load(f)
    preds_src = os.path.join(ref, "preds", "TransE_DBpedia50.csv")
    with open(preds_src) as f:
        lines = [x.strip().split("\t") for x in f.readlines()][:N_PREDS]
    with open(os.path.join(HERE, "dbpedia50_preds.tsv"), "w") as f:
        f.write("".join("\t".join(t) + "\n" for t in lines))
    d = cfg["model_params"]["dimension"]
    w = synth.make_weights("TransE", ds.num_entities, ds.num_relations, d, seed=SEED)
    sha = {k: hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() for k, v in w.items()}

    ref_harness.register_dataset("DBpedia50_real", ds.num_entities, ds.num_relations, ds.training_triples,
                                 ds.validation_triples, ds.testing_triples, ds.entity_to_id, ds.relation_to_id)
    from src.data import Dataset as RefDataset
    from src.explain import build_pipeline
    from src.link_prediction import MODEL_REGISTRY
    torch.set_num_threads(8)
    patches = None
    if fp64:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from conditioning import _Patches, to_double
        patches = _Patches(fp64=True, dim=cfg["model_params"]["dimension"]).__enter__()
    ref_harness.seed_all(42)  # explain.py:144
    dataset = RefDataset("DBpedia50_real")
    assert dataset.num_entities == ds.num_entities and len(dataset.training_triples) == len(ds.training_triples)
    cls = MODEL_REGISTRY["TransE"]["class"]
    model = cls(dataset=dataset, hp=cls.get_hyperparams_class()(**cfg["model_params"]), init_random=True)
    with torch.no_grad():
        model.entity_embeddings.data = torch.from_numpy(w["entity_embeddings"].copy())
        model.relation_embeddings.data = torch.from_numpy(w["relation_embeddings"].copy())
    model.eval()
    if fp64:
        to_double(model)
    pipeline = build_pipeline(model, dataset, cfg["training"], "necessary", None, None, None, None)
    out, per_pred = [], []
    t_all = time.time()
    for pred in lines:
        t0 = time.time()
        ex = pipeline.explain(pred=dataset.ids_triple(pred), prefilter_k=20)
        per_pred.append(time.time() - t0)
        out.append(json.loads(json.dumps(ex, default=lambda x: x.item() if hasattr(x, "item") else list(x))))
        print(pred, ex["#relevances"], f"{per_pred[-1]:.1f}s", flush=True)
    if fp64:
        patches.__exit__(None, None, None)
        with open(os.path.join(HERE, "dbpedia50_transe_fp64.json"), "w") as f:
            json.dump({"variant": "reference in float64 (tools/conditioning.py patches)", "weights_seed": SEED,
                       "weights_sha256": sha, "explanations": out, "reference_seconds": time.time() - t_all}, f)
        return
    rec = {"config": "BASELINE.json configs[0]: TransE DBpedia50 necessary-mode, 10 predictions",
           "dataset": "reference data/DBpedia50 (train/valid/test.txt), ids: sorted training labels",
           "num_entities": ds.num_entities, "num_relations": ds.num_relations,
           "n_train": int(len(ds.training_triples)), "model_params": cfg["model_params"], "hp": cfg["training"],
           "weights_seed": SEED, "weights_sha256": sha, "preds_file": "dbpedia50_preds.tsv", "prefilter_k": 20,
           "xsi": 5.0, "seed": 42, "explanations": out, "reference_seconds_per_pred": per_pred,
           "reference_seconds": time.time() - t_all, "reference_threads": 8}
    with open(os.path.join(HERE, "dbpedia50_transe.json"), "w") as f:
        json.dump(rec, f)


if __name__ == "__main__":
    main()

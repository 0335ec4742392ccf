"""Conditioning of the reference's post-training at the bench's random init
(development container only; TEST INFRASTRUCTURE, never runs on the GPU box).

The bench workloads use the reference's own random initialisers (ComplEx
U[0,1)*1e-3, ConvE xavier / torch default layers).  At that init the
post-training target is dense and the adaptive optimizers (Adagrad's
g/sqrt(g^2) first step, Adam) turn last-bit gradient differences into whole
+-lr steps, so the final rank of the target can move by a place or two under a
perturbation that is mathematically a no-op.  This script measures that on the
bench's own sample, by running the *reference itself* (imported through
``tests/golden/ref_harness.py``) under three variants that compute the same
mathematical function:

* ``fp32``      - the reference as it is;
* ``fp32_perm`` - the same run with the tables' reduction order permuted:
  ComplEx: the d complex coordinates are permuted (the same permutation in the
  Re and Im halves of every entity row, relation row and the kelpie init), so
  every dot product q.E_e sums its 400 terms in another order; ConvE: the 32
  conv filters are permuted (conv weight / bias, BN2 and the matching blocks of
  FC columns), so the 9,728-term FC reduction runs in another order;
* ``fp64``      - every table, layer and optimizer state in float64, with the
  random draws taken in float32 exactly as the fp32 run takes them (torch.rand,
  the construction-time uniform_/normal_ draws and the dropout masks are drawn
  into float32 tensors and cast), so both runs consume the generators alike.

If the GPU's distance from the reference is no larger than these variants'
distances from each other, the difference is the problem's conditioning, not a
precision deficit of the GPU path.  Writes ``profiles/conditioning_<workload>.json``
(relevances, rank deltas, per post-training target score / rank of every run,
plus the GPU run of ``profiles/noise_floor_<workload>.json`` on the same sample).

    python tools/conditioning.py --workload complex-db100k-necessary
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import bench  # noqa: E402
import noise_floor  # noqa: E402
import ref_harness  # noqa: E402
from kelpie_amd import synth  # noqa: E402


def permuted_weights(wl, w, seed=7):
    """Weights whose forward/backward compute the same function with other reduction orders."""
    rng = np.random.default_rng(seed)
    w = dict(w)
    if wl["model"] == "ComplEx":
        d = wl["dim"]
        p = rng.permutation(d)
        cols = np.concatenate([p, p + d])
        w["entity_embeddings"] = np.ascontiguousarray(w["entity_embeddings"][:, cols])
        w["relation_embeddings"] = np.ascontiguousarray(w["relation_embeddings"][:, cols])
        return w, cols
    if wl["model"] == "ConvE":
        f = rng.permutation(32)
        w["conv_weight"] = np.ascontiguousarray(w["conv_weight"].reshape(32, 1, 3, 3)[f])
        w["conv_bias"] = np.ascontiguousarray(w["conv_bias"][f])
        for k in ("bn2_weight", "bn2_bias", "bn2_mean", "bn2_var"):
            w[k] = np.ascontiguousarray(w[k][f])
        fc = w["fc_weight"].reshape(wl["dim"], 32, -1)  # FC columns are channel-major (32 x 38 x 8)
        w["fc_weight"] = np.ascontiguousarray(fc[:, f, :].reshape(wl["dim"], -1))
        return w, None
    raise ValueError("no reduction-order permutation for " + wl["model"])


class _Patches:
    """Monkeypatches for one variant, undone on exit."""

    def __init__(self, init_cols=None, fp64=False, dim=None):
        self.init_cols, self.fp64, self.dim = init_cols, fp64, dim
        self.saved = []

    def _set(self, obj, name, val):
        self.saved.append((obj, name, getattr(obj, name)))
        setattr(obj, name, val)

    def __enter__(self):
        orig_rand = torch.rand
        cols, fp64, dim = self.init_cols, self.fp64, self.dim

        def rand(*size, **kw):
            if fp64 and "dtype" not in kw:
                out = orig_rand(*size, dtype=torch.float32, **kw).to(torch.float64)
            else:
                out = orig_rand(*size, **kw)
            if cols is not None and out.dim() == 2 and out.shape[0] == 1 and out.shape[1] == dim:
                out = out[:, torch.as_tensor(cols)].contiguous()  # the kelpie init (post_training_engine.py:52)
            return out

        self._set(torch, "rand", rand)
        if fp64:
            torch.set_default_dtype(torch.float64)
            ou, on = torch.Tensor.uniform_, torch.Tensor.normal_

            def uniform_(t, *a, **k):
                if t.dtype == torch.float64:
                    tmp = torch.empty(t.shape, dtype=torch.float32)
                    ou(tmp, *a, **k)
                    with torch.no_grad():
                        t.copy_(tmp)
                    return t
                return ou(t, *a, **k)

            def normal_(t, *a, **k):
                if t.dtype == torch.float64:
                    tmp = torch.empty(t.shape, dtype=torch.float32)
                    on(tmp, *a, **k)
                    with torch.no_grad():
                        t.copy_(tmp)
                    return t
                return on(t, *a, **k)

            self._set(torch.Tensor, "uniform_", uniform_)
            self._set(torch.Tensor, "normal_", normal_)
            odrop = torch.nn.functional.dropout

            def dropout(x, p=0.5, training=True, inplace=False):
                # at::native dropout on CPU: noise = empty_like(x).bernoulli_(1 - p) / (1 - p); x * noise
                if not training or p == 0 or x.dtype != torch.float64:
                    return odrop(x, p, training, inplace)
                noise = torch.empty(x.shape, dtype=torch.float32).bernoulli_(1 - p)
                noise.div_(1 - p)
                return x * noise.to(torch.float64)

            self._set(torch.nn.functional, "dropout", dropout)
        return self

    def __exit__(self, *exc):
        for obj, name, val in reversed(self.saved):
            setattr(obj, name, val)
        torch.set_default_dtype(torch.float32)


def to_double(model):
    with torch.no_grad():
        for name in ("entity_embeddings", "relation_embeddings"):
            t = getattr(model, name)
            t.data = t.data.double()
    for mod in model.modules():
        if isinstance(mod, torch.nn.Module) and mod is not model:
            mod.double()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="complex-db100k-necessary", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--variants", nargs="+", default=["fp32", "fp32_perm", "fp64"])
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--fixture-only", action="store_true", help="rewrite the fixture from the profiles record")
    ap.add_argument("--pred-index", type=int, default=None,
                    help="a further sample: prediction k of bench.pick_preds (fixture <workload>__p<k>.json)")
    ap.add_argument("--candidates", type=int, default=3, help="candidates of that prediction (with --pred-index)")
    args = ap.parse_args()
    name = args.workload if args.pred_index is None else f"{args.workload}__p{args.pred_index}"
    if args.fixture_only:
        with open(os.path.join(ROOT, "profiles", f"conditioning_{name}.json")) as f:
            write_fixture(json.load(f))
        return
    torch.set_num_threads(args.threads)
    wl = bench.WORKLOADS[args.workload]
    src = ref_harness.load_reference()
    nf_path = os.path.join(ROOT, "profiles", f"noise_floor_{args.workload}.json")
    g = synth.make_graph(wl["shape"], seed=0)
    w0 = synth.make_weights(wl["model"], g.num_entities, g.num_relations, wl["dim"], seed=0)
    if args.pred_index is not None:
        # a further sample of the bench's own predictions: pick_preds' k-th prediction and
        # its first candidates (bench.candidates_of), conversion entities as the reference
        # selects them (engine.py:22-126, seeds 42)
        from kelpie_amd import Dataset
        ds = Dataset(g.num_entities, g.num_relations, g.train, g.valid, g.test, name=wl["shape"])
        pk = bench.pick_preds(ds, args.pred_index + 1, seed=1234)[args.pred_index]
        nf = {"pred": list(pk), "candidates": [list(c) for c in bench.candidates_of(ds, pk, wl["candidates"])
                                                [:args.candidates]], "entities_to_convert": None, "runs": {}}
        if wl["mode"] == "sufficient":
            from src.relevance_engines import SufficientPostTrainingEngine
            dataset, model = noise_floor.reference_model(src, wl, g, w0)
            # the synthetic DB100K shape has entities with no training triple, which the
            # reference's degree lookup (engine.py:73, a plain dict) raises on; real datasets
            # index every entity from the training file.  Degree 0 there means "skip", as the
            # engine's own `< 1` test does (kelpie_amd/engine.py uses .get(e, 0)).
            import collections
            dataset.entity_to_degree = collections.defaultdict(int, dataset.entity_to_degree)
            ref_harness.seed_all(42)
            se = SufficientPostTrainingEngine(model, dataset, wl["hp"])
            se.select_entities_to_convert(tuple(pk), wl["convert"], 200)
            nf["entities_to_convert"] = [int(e) for e in se.entities_to_convert]
    elif os.path.exists(nf_path):
        with open(nf_path) as f:
            nf = json.load(f)  # the sample (pred, candidates, conversion entities) and its GPU run
    else:
        # the same sample noise_floor.py takes: the bench's first prediction, its first candidates
        from kelpie_amd import Dataset
        ds = Dataset(g.num_entities, g.num_relations, g.train, g.valid, g.test, name=wl["shape"])
        p0 = bench.pick_preds(ds, 1, seed=1234)[0]
        nf = {"pred": list(p0), "candidates": [list(c) for c in bench.candidates_of(ds, p0, wl["candidates"])[:3]],
              "entities_to_convert": None, "runs": {}}
        if wl["mode"] == "sufficient":
            from src.relevance_engines import SufficientPostTrainingEngine
            dataset, model = noise_floor.reference_model(src, wl, g, w0)
            ref_harness.seed_all(42)
            se = SufficientPostTrainingEngine(model, dataset, wl["hp"])
            se.select_entities_to_convert(tuple(p0), wl["convert"], 200)  # engine.py:125
            nf["entities_to_convert"] = [int(e) for e in se.entities_to_convert]
    pred = tuple(nf["pred"])
    cands = [tuple(c) for c in nf["candidates"]]
    ents = nf.get("entities_to_convert")
    D = wl["dim"] * (2 if wl["model"] == "ComplEx" else 1)
    out_path = os.path.join(ROOT, "profiles", f"conditioning_{name}.json")
    out = {"workload": args.workload, "name": name, "pred": list(pred), "candidates": [list(c) for c in cands],
           "entities_to_convert": ents, "threads": args.threads, "runs": {}}
    if os.path.exists(out_path):
        with open(out_path) as f:
            out["runs"] = json.load(f).get("runs", {})
    for v in args.variants:
        # no permuted variant for TransE (nothing to permute) or under feature-map dropout:
        # its per-channel masks (conve.py:147) would land on other filters, another model
        if v in out["runs"] or (v == "fp32_perm" and (wl["model"] == "TransE"
                                                      or wl.get("fmap_dropout", 0) > 0)):
            continue
        w, cols = (permuted_weights(wl, w0) if v == "fp32_perm" else (w0, None))
        dataset, model = noise_floor.reference_model(src, wl, g, w)
        with _Patches(init_cols=cols, fp64=(v == "fp64"), dim=D):
            if v == "fp64":
                to_double(model)
            t0 = time.time()
            rels, log = noise_floor.run_reference(src, wl, dataset, model, pred, cands, ents)
        deltas = noise_floor.deltas_of(log, wl["mode"])
        out["runs"][v] = {"relevances": rels, "results": log, "rank_deltas": deltas, "seconds": time.time() - t0,
                          "cand_seconds": noise_floor.run_reference.cand_seconds}
        print(f"{v}: rels {rels} deltas {deltas} ({time.time() - t0:.0f}s)", flush=True)
        with open(out_path, "w") as f:
            json.dump(out, f, indent=1)
    if "gpu" in nf["runs"]:
        out["runs"]["gpu"] = {k: nf["runs"]["gpu"][k] for k in ("relevances", "rank_deltas")}
    names = list(out["runs"])
    rates, diffs = {}, {}
    for i, a in enumerate(names):
        for b in names[i + 1:]:
            da, db = out["runs"][a]["rank_deltas"], out["runs"][b]["rank_deltas"]
            rates[f"{a} vs {b}"] = float(np.mean([x == y for x, y in zip(da, db)]))
            diffs[f"{a} vs {b}"] = int(max(abs(x - y) for x, y in zip(da, db)))
    out["rank_delta_match_rates"], out["rank_delta_max_abs_diff"] = rates, diffs
    print(json.dumps(diffs, indent=1))
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    write_fixture(out)


def write_fixture(rec):
    """tests/golden/fullsize/<workload>.json: the sample and the reference runs on it (data
    only), read by the full-size GPU parity test and by bench.py's match rate."""
    fx = {k: rec[k] for k in ("workload", "pred", "candidates", "entities_to_convert", "threads")}
    fx["generator"] = "tools/conditioning.py (reference imported through tests/golden/ref_harness.py, CPU)"
    fx["runs"] = {}
    for name, run in rec["runs"].items():
        if name.startswith("gpu"):
            continue
        res = [[{"rank": r["target_rank"], "score": r["target_score"]} for r in call] for call in run["results"]]
        fx["runs"][name] = {"relevances": run["relevances"], "rank_deltas": run["rank_deltas"], "results": res,
                            "seconds": run.get("seconds"), "cand_seconds": run.get("cand_seconds")}
    d = os.path.join(ROOT, "tests", "golden", "fullsize")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, rec.get("name", rec["workload"]) + ".json"), "w") as f:
        json.dump(fx, f, indent=1)


if __name__ == "__main__":
    main()

"""Per-post-training probe of the full-size parity sample (development container only;
TEST INFRASTRUCTURE, imports the reference through tests/golden/ref_harness.py).

``--side ref``: runs the reference on a fixture's sample (tools/conditioning.py
variants fp32 / fp64) and records, for every get_triple_results call, the kelpie row
and the full score vector -> ``gpurun_out/probe_<workload>_<variant>.npz``.

``--side gpu`` (on the GPU box): runs the engine on the same sample and records every
slot's post-trained kelpie row, target score and rank -> ``gpurun_out/probe_<workload>_gpu<tag>.npz``.

``--side compare``: for every post-training, the relative error of the kelpie rows
against fp64, the target score errors, and for rank mismatches the number of
entities whose fp64 score lies within the GPU's target-score error of the target.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "gpurun_out")


def _fixture(name):
    import json
    with open(os.path.join(ROOT, "tests", "golden", "fullsize", name + ".json")) as f:
        return json.load(f)


def ref_side(workload, variant, threads, name):
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import bench
    import conditioning
    import noise_floor
    import ref_harness
    from kelpie_amd import synth
    torch.set_num_threads(threads)
    wl = bench.WORKLOADS[workload]
    fx = _fixture(name)
    src = ref_harness.load_reference()
    g = synth.make_graph(wl["shape"], seed=0)
    w0 = synth.make_weights(wl["model"], g.num_entities, g.num_relations, wl["dim"], seed=0)
    D = wl["dim"] * (2 if wl["model"] == "ComplEx" else 1)
    dataset, model = noise_floor.reference_model(src, wl, g, w0)
    rows, scores, meta = [], [], []
    from src.relevance_engines import post_training_engine as pte
    orig = pte.PostTrainingEngine.get_triple_results

    def wrapped(self, m, triple):
        r = orig(self, m, triple)
        with torch.no_grad():
            k = m.entity_embeddings[-1].detach().double().cpu().numpy().copy()
            s = m.all_scores(np.array([triple]))[0].detach().double().cpu().numpy().copy()
        rows.append(k)
        scores.append(s)
        meta.append((int(r["target_rank"]), float(r["target_score"])))
        return r

    pte.PostTrainingEngine.get_triple_results = wrapped
    with conditioning._Patches(init_cols=None, fp64=(variant == "fp64"), dim=D):
        if variant == "fp64":
            conditioning.to_double(model)
        rels, log = noise_floor.run_reference(src, wl, dataset, model, tuple(fx["pred"]),
                                              [tuple(c) for c in fx["candidates"]], fx.get("entities_to_convert"))
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, f"probe_{name}_{variant}.npz"), rows=np.array(rows),
                        scores=np.array(scores), rank=np.array([m[0] for m in meta]),
                        score=np.array([m[1] for m in meta]))
    print(variant, rels, noise_floor.deltas_of(log))


def gpu_side(workload, tag, name):
    import bench
    from kelpie_amd import NecessaryPostTrainingEngine, SufficientPostTrainingEngine
    from kelpie_amd import engine as keng
    wl = bench.WORKLOADS[workload]
    fx = _fixture(name)
    ds, model, _ = bench.build(wl, 0, 0)
    cls = SufficientPostTrainingEngine if wl["mode"] == "sufficient" else NecessaryPostTrainingEngine
    eng = cls(model, ds, wl["hp"])
    captured = []
    orig = model.ctx.posttrain_rank

    def pr(*a, **k):
        k["want_x"] = True
        s, r, x = orig(*a, **k)
        captured.append((np.array(s), np.array(r), np.array(x)))
        return s, r, x

    model.ctx.posttrain_rank = pr
    _, _, _, par = bench.parity_sample(eng, wl, fx, None)
    s = np.concatenate([c[0] for c in captured])
    r = np.concatenate([c[1] for c in captured])
    x = np.concatenate([c[2] for c in captured])
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, f"probe_{name}_gpu{tag}.npz"), rows=x, score=s, rank=r)
    print(json.dumps(par))


def compare(workload, tags):
    ref = {v: np.load(os.path.join(OUT, f"probe_{workload}_{v}.npz")) for v in ("fp32", "fp64")}
    # (workload here is the fixture name)
    e64 = ref["fp64"]
    print(f"{'i':>3} {'rank64':>7} {'r32':>6} " + " ".join(f"{'r' + t:>6}" for t in tags) +
          "  xerr32   " + " ".join(f"xerr{t:<6}" for t in tags) + "  serr32    " +
          " ".join(f"serr{t:<6}" for t in tags) + "  gap64(rel)")
    gpus = {t: np.load(os.path.join(OUT, f"probe_{workload}_gpu{t}.npz")) for t in tags}
    n = len(e64["rank"])
    for i in range(n):
        x64 = e64["rows"][i]
        s64 = e64["scores"][i]
        tgt = e64["score"][i]
        # distance from the fp64 target to the nearest other fp64 score
        d = np.abs(s64 - tgt)
        d = d[d > 0]
        gap = d.min() / abs(tgt) if len(d) else float("nan")
        cols = [f"{i:>3} {e64['rank'][i]:>7} {ref['fp32']['rank'][i]:>6} "]
        cols += [f"{gpus[t]['rank'][i]:>6} " for t in tags]
        xe = lambda x: np.abs(x - x64).max() / np.abs(x64).max()  # noqa: E731
        se = lambda s: abs(s - tgt) / abs(tgt)  # noqa: E731
        cols.append(f" {xe(ref['fp32']['rows'][i]):.2e} ")
        cols += [f"{xe(gpus[t]['rows'][i]):.2e}   " for t in tags]
        cols.append(f" {se(ref['fp32']['score'][i]):.2e} ")
        cols += [f"{se(gpus[t]['score'][i]):.2e}   " for t in tags]
        cols.append(f" {gap:.1e}")
        mark = " *" if any(gpus[t]["rank"][i] != e64["rank"][i] for t in tags) else ""
        print("".join(cols) + mark)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", choices=["ref", "gpu", "compare"], required=True)
    ap.add_argument("--workload", default="complex-fb15k237-sufficient")
    ap.add_argument("--variant", default="fp32")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--tag", default="")
    ap.add_argument("--tags", nargs="+", default=[""])
    ap.add_argument("--fixture", default=None, help="tests/golden/fullsize/<name>.json (default: the workload's)")
    a = ap.parse_args()
    name = a.fixture or a.workload
    if a.fixture:
        a.workload = _fixture(name)["workload"]
    if a.side == "ref":
        ref_side(a.workload, a.variant, a.threads, name)
    elif a.side == "gpu":
        gpu_side(a.workload, a.tag, name)
    else:
        compare(name, a.tags)


if __name__ == "__main__":
    main()

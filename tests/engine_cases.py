"""Shared checks of the product engine against the reference golden vectors.

Used by test_engine_cpu.py (oracle-backed context: host protocol only) and
test_gpu_parity.py (the HIP library on an MI355X)."""
from __future__ import annotations

import numpy as np

from golden_io import load_case, seed_all

import kelpie_amd as ka

TOL = 1e-4


def build_product(name, backend):
    rec, arrays, w = load_case(name)
    ds = ka.Dataset(rec["num_entities"], rec["num_relations"], arrays["train"], arrays["valid"], arrays["test"])
    mp = rec["model_params"]
    if rec["model"] == "ComplEx":
        model = ka.ComplEx(ds, w["entity_embeddings"], w["relation_embeddings"], init_scale=mp["init_scale"])
    elif rec["model"] == "TransE":
        model = ka.TransE(ds, w["entity_embeddings"], w["relation_embeddings"], norm=mp["norm"])
    else:
        bn = {i: {"weight": w[f"bn{i}_weight"], "bias": w[f"bn{i}_bias"], "running_mean": w[f"bn{i}_mean"],
                  "running_var": w[f"bn{i}_var"]} for i in (1, 2, 3)}
        model = ka.ConvE(ds, w["entity_embeddings"], w["relation_embeddings"], w["conv_weight"].reshape(32, 3, 3),
                         w["conv_bias"], w["fc_weight"], w["fc_bias"], bn=bn,
                         input_dropout_rate=mp["input_dropout_rate"],
                         feature_map_dropout_rate=mp["feature_map_dropout_rate"],
                         hidden_dropout_rate=mp["hidden_dropout_rate"])
    if backend == "cpu":
        from cpu_backend import OracleBackedContext
        model._ctx = OracleBackedContext(model)
    return rec, ds, model


def _close(a, b, tol=TOL):
    return abs(a - b) <= tol * max(1.0, abs(b))


def check_necessary(name, backend, batched):
    """Every recorded compute_relevance call; batched=True evaluates all rules of
    a prediction in one engine batch (must equal the sequential reference)."""
    rec, ds, model = build_product(name, backend)
    seed_all(rec["seed"])
    eng = ka.NecessaryPostTrainingEngine(model, ds, rec["hp"])
    stats = {"rank_match": 0, "n": 0, "max_rel_err": 0.0, "max_score_err": 0.0}
    for block in rec["necessary"]:
        eng.set_cache()
        pred = tuple(block["pred"])
        rules = [[tuple(t) for t in c["rule"]] for c in block["calls"]]
        if batched:
            rels = eng.compute_relevance_batch(pred, rules)
            results = list(eng.last_results)
        else:
            rels, results = [], []
            for r in rules:
                rels.append(eng.compute_relevance(pred, r))
                results.append(eng.last_results[0])
        for ci, (call, rel, (pt, base)) in enumerate(zip(block["calls"], rels, results)):
            exp_pt = call["results"][-1]
            stats["n"] += 1
            stats["rank_match"] += int(pt["target_rank"] == exp_pt["target_rank"])
            stats["max_rel_err"] = max(stats["max_rel_err"], abs(rel - call["relevance"]))
            stats["max_score_err"] = max(stats["max_score_err"], abs(pt["target_score"] - exp_pt["target_score"]))
            if ci == 0:
                eb = call["results"][0]
                assert base["target_rank"] == eb["target_rank"], (name, pred, "base rank")
                assert _close(base["target_score"], eb["target_score"]), (name, pred, "base score")
            assert pt["target_rank"] == exp_pt["target_rank"], (name, pred, call["rule"], pt, exp_pt)
            assert _close(pt["target_score"], exp_pt["target_score"]), (name, pred, call["rule"], pt, exp_pt)
            assert abs(rel - call["relevance"]) <= TOL, (name, pred, call["rule"], rel, call["relevance"])
    return stats


def check_sufficient(name, backend, batched):
    rec, ds, model = build_product(name, backend)
    seed_all(rec["seed"])
    eng = ka.SufficientPostTrainingEngine(model, ds, rec["hp"])
    for block in rec["sufficient"]:
        eng.set_cache()
        pred = tuple(block["pred"])
        ents = eng.select_entities_to_convert(pred, block["k"], block["degree_cap"])
        assert ents == block["entities_to_convert"], (ents, block["entities_to_convert"])
        rules = [[tuple(t) for t in c["rule"]] for c in block["calls"]]
        rels = eng.compute_relevance_batch(pred, rules) if batched else [eng.compute_relevance(pred, r) for r in rules]
        for call, rel in zip(block["calls"], rels):
            assert abs(rel - call["relevance"]) <= TOL, (name, call["rule"], rel, call["relevance"])


def check_builder(name, backend, window=32, pipelined=False):
    """The builder's explanations equal the reference's; returns the library calls made
    and the builder's stats per recorded builder case."""
    rec, ds, model = build_product(name, backend)
    calls = [0]
    seen = set()
    for ctx in model.contexts(2):
        if id(ctx) in seen:
            continue
        seen.add(id(ctx))
        orig = ctx.posttrain_rank

        def counted(*a, _orig=orig, **k):
            calls[0] += 1
            return _orig(*a, **k)

        ctx.posttrain_rank = counted
    out_stats = []
    for key in ("builder", "builder_window"):
        b = rec.get(key)
        if not b:
            continue
        seed_all(rec["seed"])
        eng = ka.NecessaryPostTrainingEngine(model, ds, rec["hp"])
        builder = ka.StochasticBuilder(b["xsi"], eng, window=window, pipelined=pipelined)
        eng.set_cache()
        out = builder.build_explanations(tuple(b["pred"]), [tuple(t) for t in b["candidates"]])
        assert out["#relevances"] == b["n_relevances"], (key, out["#relevances"], b["n_relevances"])
        assert len(out["rule_to_relevance"]) == len(b["rule_to_relevance"])
        for (rule, rel), (erule, erel) in zip(out["rule_to_relevance"], b["rule_to_relevance"]):
            assert [list(t) for t in rule] == [list(t) for t in erule]
            assert abs(rel - erel) <= TOL
        out_stats.append((calls[0], dict(builder.stats)))
        calls[0] = 0
    return out_stats


def _two_stand_in_contexts(model):
    """CPU tier: give the pipeline a second (stand-in) context, so two batches are in
    flight on two contexts as on the GPU (FrozenModel.contexts)."""
    from cpu_backend import OracleBackedContext
    extra = OracleBackedContext(model)
    model.contexts = lambda n: [model.ctx, extra][:max(1, min(n, 2))]


def check_pipeline(name, backend, two_contexts=False):
    """compute_relevance_pipeline (host schedules batch k+1 while batch k runs)
    over every recorded prediction equals the reference's sequential calls."""
    rec, ds, model = build_product(name, backend)
    if two_contexts and backend == "cpu":
        _two_stand_in_contexts(model)
    seed_all(rec["seed"])
    eng = ka.NecessaryPostTrainingEngine(model, ds, rec["hp"])
    batches = [[(tuple(b["pred"]), [[tuple(t) for t in c["rule"]] for c in b["calls"]])] for b in rec["necessary"]]
    outs = eng.compute_relevance_pipeline(batches)
    assert len(eng.last_batch_stats) == len(batches)
    for block, out in zip(rec["necessary"], outs):
        for call, rel in zip(block["calls"], out[0]):
            assert abs(rel - call["relevance"]) <= TOL, (name, call["rule"], rel, call["relevance"])
    if not rec.get("sufficient"):
        return
    rec, ds, model = build_product(name, backend)
    if two_contexts and backend == "cpu":
        _two_stand_in_contexts(model)
    seed_all(rec["seed"])
    eng = ka.SufficientPostTrainingEngine(model, ds, rec["hp"])
    batches = []
    for block in rec["sufficient"]:
        eng.set_cache()
        pred = tuple(block["pred"])
        ents = eng.select_entities_to_convert(pred, block["k"], block["degree_cap"])
        batches.append([(pred, [[tuple(t) for t in c["rule"]] for c in block["calls"]], ents)])
    for block, out in zip(rec["sufficient"], eng.compute_relevance_pipeline(batches)):
        for call, rel in zip(block["calls"], out[0]):
            assert abs(rel - call["relevance"]) <= TOL, (name, call["rule"], rel, call["relevance"])


def check_pipeline_explain(name, backend, tmpdir):
    """NecessaryPipeline (prefilter -> builder, src/pipeline.py:21-29) over read_preds /
    explain_preds / output.json equals the reference's recorded builder run."""
    import json
    import os
    from kelpie_amd.pipeline import build_pipeline, explain_preds, read_preds
    rec, ds, model = build_product(name, backend)
    b = rec["builder"]
    pred = tuple(b["pred"])
    preds_path = os.path.join(tmpdir, "preds.csv")
    with open(preds_path, "w") as f:
        f.write("\t".join(ds.labels_triple(pred)) + "\n")
    seed_all(rec["seed"])
    pipe = build_pipeline(model, ds, rec["hp"], "necessary", xsi=b["xsi"])
    out_path = os.path.join(tmpdir, "output.json")
    res = explain_preds(pipe, ds, read_preds(preds_path), prefilter_k=len(b["candidates"]), output_path=out_path)
    with open(out_path) as f:
        on_disk = json.load(f)
    assert len(res) == len(on_disk) == 1
    out = on_disk[0]
    assert set(out) == {"triple", "rule_to_relevance", "#relevances", "execution_time"}
    assert out["triple"] == list(b["triple"])
    assert out["#relevances"] == b["n_relevances"]
    assert len(out["rule_to_relevance"]) == len(b["rule_to_relevance"])
    for (rule, rel), (erule, erel) in zip(out["rule_to_relevance"], b["rule_to_relevance"]):
        assert [list(t) for t in rule] == [list(t) for t in erule]  # label triples
        assert abs(rel - erel) <= TOL

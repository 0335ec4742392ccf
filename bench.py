#!/usr/bin/env python
"""Throughput of the MI355X relevance engine on the reference's headline path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

Metric (BASELINE.json): candidate explanations evaluated per second,
including post-training, plus the rank-delta match rate.  A unit is one
``compute_relevance`` call (one increment of the reference's ``#relevances``,
stochastic_builder.py:50,61).  A *step* is one prediction's singleton
candidates (the builder's hot loop A) evaluated as one engine batch, with the
per-prediction caches reset first (so the base post-trainings are included,
as in the reference's ``execution_time``).

Default workload (north star: ComplEx on FB15k-237, sufficient mode with
conversion entities): synthetic FB15k-237-shaped graph (14,541 entities, 237
relations, 272,115 train triples; kelpie_amd.synth), ComplEx d=200 with the
reference's random init, the ComplEx DBpedia50 explanation hp (Adagrad 0.043,
43 epochs, batch 512), 20 candidates per prediction, 10 conversion entities
(pipeline.py:36-39, degree cap 200).

For N > 1 the driver launches one rank per GPU with torchrun; a plain
``python bench.py --gpus N`` starts the N local ranks itself (torchrun as a child
process), and a WORLD_SIZE other than N is refused.  A step then holds
N times the predictions (weak scaling: the per-GPU work is fixed); every rank walks
every batch's draws -- the reference's one global random stream, in the same order on
every rank -- but schedules in full and post-trains only the slots it claims (for the
others it only advances the generators), with one all-gather of the (slot, score,
rank) records per batch (kelpie_amd.distributed.SlotSharding), so the results equal
the 1-rank run.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "candidate explanations evaluated/sec (incl. post-train) + rank-delta match rate"

COMPLEX_HP = {"optimizer_name": "Adagrad", "batch_size": 512, "epochs": 43, "lr": 0.043, "decay1": 0.9,
              "decay2": 0.999, "regularizer_name": "N3", "regularizer_weight": 0}  # ComplEx_DBpedia50_explanation.json
TRANSE_HP = {"batch_size": 2048, "epochs": 65, "lr": 0.01, "margin": 5, "negative_triples_ratio": 5,
             "regularizer_weight": 1.0}  # TransE_DBpedia50_explanation.json
COMPLEX_DB100K_HP = {"optimizer_name": "Adagrad", "batch_size": 512, "epochs": 83, "lr": 0.0814, "decay1": 0.9,
                     "decay2": 0.999, "regularizer_name": "N3",
                     "regularizer_weight": 0}  # ComplEx_DB100K_explanation.json
CONVE_HP = {"batch_size": 512, "label_smoothing": 0.1, "lr": 0.0432, "decay": 0.995,
            "epochs": 109}  # ConvE_DB100K_explanation.json (hidden dropout 0.2)

WORKLOADS = {
    # BASELINE.json configs[2]: the north-star target (>= 50x, ComplEx on FB15k-237)
    "complex-fb15k237-sufficient": dict(model="ComplEx", shape="FB15k-237", dim=200, mode="sufficient",
                                        hp=COMPLEX_HP, candidates=20, convert=10, preds_per_step=1, depth=3,
                                        cpu_conversions=2),
    # the same with "many conversion entities" (K = 10 / 50 / 100; engine.py:125
    # samples min(K, convertible) of them)
    "complex-fb15k237-sufficient-k50": dict(model="ComplEx", shape="FB15k-237", dim=200, mode="sufficient",
                                            hp=COMPLEX_HP, candidates=20, convert=50, preds_per_step=1, depth=3,
                                            cpu_conversions=2),
    "complex-fb15k237-sufficient-k100": dict(model="ComplEx", shape="FB15k-237", dim=200, mode="sufficient",
                                             hp=COMPLEX_HP, candidates=20, convert=100, preds_per_step=1, depth=3,
                                             cpu_conversions=2),
    # three batches in flight (round 5: 3,412 / 3,545 vs 3,225 / 3,347 cand/s at two, alternating
    # on one box, profiles/r05/necessary_depth_ab.txt: at two the device idled 11 % of the time
    # in 15-26 ms gaps at batch boundaries, profiles/r05/timeline_complex-fb15k237-necessary.txt)
    "complex-fb15k237-necessary": dict(model="ComplEx", shape="FB15k-237", dim=200, mode="necessary",
                                       hp=COMPLEX_HP, candidates=20, preds_per_step=16, depth=3),
    # BASELINE.json configs[1]
    "transe-fb15k237-necessary": dict(model="TransE", shape="FB15k-237", dim=200, mode="necessary",
                                      hp=TRANSE_HP, candidates=20, preds_per_step=16),
    # BASELINE.json configs[3] (necessary + sufficient; the 8-GPU sharding is bench.py --gpus N)
    "complex-db100k-necessary": dict(model="ComplEx", shape="DB100K", dim=200, mode="necessary",
                                     hp=COMPLEX_DB100K_HP, candidates=20, preds_per_step=16),
    "complex-db100k-sufficient": dict(model="ComplEx", shape="DB100K", dim=200, mode="sufficient",
                                      hp=COMPLEX_DB100K_HP, candidates=20, convert=10, preds_per_step=1,
                                      cpu_conversions=2, depth=3),
    # BASELINE.json configs[4]
    # eight predictions per step.  (Round 6 measured six against eight: 498.6 / 518.6 / 510.8
    # against 486.5 / 485.0 / 487.6 cand/s, profiles/r06/r06z6/ -- but at a fixed step count
    # the two time different predictions, and eight's are 7.5 % heavier per candidate (65.7
    # against 61.1 training rows): per row eight is as fast, 32.0k against 31.2k rows/s.)
    "conve-yago310-necessary": dict(model="ConvE", shape="YAGO3-10", dim=200, mode="necessary", hp=CONVE_HP,
                                    candidates=20, preds_per_step=8, hidden_dropout=0.2, depth=3),
    # the same with all three ConvE dropouts in post-training at the rates of the reference's
    # ConvE YAGO4-20 config (configs/ConvE_YAGO4-20_training.json: input 0.2, feature map 0.3,
    # hidden 0.1; conve.py:142,147,151): the frozen-head pairs are re-encoded every step
    "conve-yago310-necessary-drop": dict(model="ConvE", shape="YAGO3-10", dim=200, mode="necessary", hp=CONVE_HP,
                                         candidates=20, preds_per_step=8, hidden_dropout=0.1, input_dropout=0.2,
                                         fmap_dropout=0.3, depth=3),
}


def committed_counters(workload, kernel):
    """HBM bytes (FETCH_SIZE + WRITE_SIZE) and SQ counters per launch of ``kernel`` from the
    newest committed rocprofv3 pass of this workload (profiles/rNN_<workload>_pmc.json,
    tools/prof_summary.py) -- only a pass stamped with the library sources this run
    executes (``library_source_sha16``): a pass of an older kernel is never cited, the
    line then says traffic null.  PMC counters cannot be read inside the timed run."""
    import glob
    import json
    import re
    from kelpie_amd._lib import source_sha16
    here = os.path.dirname(os.path.abspath(__file__))
    m = re.match(r"(kp_attn3?)<(\d+),(\w+)>", kernel)
    want = f"{m.group(1)}<{m.group(2)}, {ATT_MODES[m.group(3)]}>" if m else kernel
    sha = source_sha16()
    for path in sorted(glob.glob(os.path.join(here, "profiles", f"r*_{workload}_pmc.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("library_source_sha16") != sha:
            continue
        fetch = d.get("fetch_bytes_per_launch") or {}
        for name, v in fetch.items():
            if want in name and v.get("hbm_bytes"):
                w = next((x["hbm_bytes"] for n2, x in (d.get("write_bytes_per_launch") or {}).items() if n2 == name),
                         None)
                sq = next((x for n2, x in (d.get("sq_per_launch") or {}).items() if want in n2), None)
                return {"read": v["hbm_bytes"], "write": w, "sq": sq, "source": os.path.relpath(path, here)}
    return {"read": None, "write": None, "sq": None, "source": None,
            "note": f"no committed counter pass of library sources {sha}"}


ATT_MODES = {"ATT_SOFTMAX_O": 0, "ATT_SOFTMAX": 1, "ATT_BCE_O": 2}
# dense bf16 MFMA peak of MI355X: 256 CUs x 4 SIMDs x 1024 FLOP/clk (16x16x32 bf16 in 16
# cycles) x 2.4 GHz (MI355X_MICROARCH.md: ~2.5 PF dense)
BF16_DENSE_TFLOPS = 2516.6


def union_seconds(iv):
    """Total length of the union of [start, end] intervals (seconds)."""
    iv = np.asarray(iv, dtype=np.float64).reshape(-1, 2)
    if len(iv) == 0:
        return 0.0
    iv = iv[np.argsort(iv[:, 0])]
    total, (s0, e0) = 0.0, iv[0]
    for s1, e1 in iv[1:]:
        if s1 > e0:
            total += e0 - s0
            s0, e0 = s1, e1
        else:
            e0 = max(e0, e1)
    return total + (e0 - s0)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _heartbeat(every_s=30.0):
    """A line on stderr every ``every_s`` seconds from a daemon thread, so a long silent
    phase (graph building, the CPU-baseline leg at YAGO3-10 size) shows progress."""
    import threading
    import time

    t0 = time.time()

    def beat():
        while True:
            time.sleep(every_s)
            log(f"[bench] alive {time.time() - t0:.0f}s")

    threading.Thread(target=beat, daemon=True).start()


def build(wl, device, rank):
    from kelpie_amd import ComplEx, ConvE, Dataset, TransE, synth
    t0 = time.time()
    g = synth.make_graph(wl["shape"], seed=0)
    ds = Dataset(g.num_entities, g.num_relations, g.train, g.valid, g.test, name=wl["shape"])
    w = synth.make_weights(wl["model"], g.num_entities, g.num_relations, wl["dim"], seed=0)
    if wl["model"] == "ComplEx":
        model = ComplEx(ds, w["entity_embeddings"], w["relation_embeddings"], init_scale=1e-3, device=device)
    elif wl["model"] == "TransE":
        model = TransE(ds, w["entity_embeddings"], w["relation_embeddings"], device=device)
    else:
        model = ConvE(ds, w["entity_embeddings"], w["relation_embeddings"], w["conv_weight"].reshape(32, 3, 3),
                      w["conv_bias"], w["fc_weight"], w["fc_bias"], hidden_dropout_rate=wl["hidden_dropout"],
                      input_dropout_rate=wl.get("input_dropout", 0.0),
                      feature_map_dropout_rate=wl.get("fmap_dropout", 0.0), device=device)
    log(f"[rank {rank}] graph+indices {time.time() - t0:.1f}s  |E|={g.num_entities} train={len(g.train)}")
    return ds, model, w


def pick_preds(ds, n, seed, lo=5, hi=200):
    rng = np.random.default_rng(seed)
    test = ds.testing_triples
    order = rng.permutation(len(test))
    out = []
    for i in order:
        s, p, o = (int(v) for v in test[i])
        if lo <= ds.entity_to_degree.get(s, 0) <= hi:
            out.append((s, p, o))
        if len(out) >= n:
            break
    return out


def candidates_of(ds, pred, k):
    return sorted(ds.entity_to_training_triples[pred[0]])[:k]


def seed_all(seed=42):
    import random
    import torch
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def load_fixture(workload):
    """tests/golden/fullsize/<workload>.json (else its first other prediction, __p0): the
    reference itself (fp32 as it runs, and fp64 / permuted-reduction-order variants) on one
    prediction of this workload (tools/conditioning.py, development container).  Data only."""
    for name in (workload, workload + "__p0"):
        path = os.path.join(ROOT, "tests", "golden", "fullsize", name + ".json")
        if os.path.exists(path):
            with open(path) as f:
                fx = json.load(f)
            fx["_file"] = os.path.relpath(path, ROOT)
            return fx
    return None


def _cores():
    import psutil
    return {"cores_physical": psutil.cpu_count(logical=False), "cores_logical": psutil.cpu_count(),
            "affinity": len(os.sched_getaffinity(0))}


def cpu_baseline(wl, ds, weights, pred, cands, ents=None, fixture=None):
    """Time the oracle (numpy restatement, tests-only module) on a bounded sample of the
    same workload: the first candidate of a prediction (which carries the prediction's
    base post-trainings) reported apart, then the steady state over the next candidates
    (SURVEY 8(d)).  Beside it, the reference's own CPU rate measured in the development
    container on the fixture's candidates (tools/conditioning.py)."""
    from threadpoolctl import threadpool_info
    from oracle import kelpie_oracle as ko
    om = ko.OracleModel(wl["model"], weights, wl["dim"],
                        {"init_scale": 1e-3, "hidden_dropout_rate": wl.get("hidden_dropout", 0.0),
                         "input_dropout_rate": wl.get("input_dropout", 0.0),
                         "feature_map_dropout_rate": wl.get("fmap_dropout", 0.0)})
    ods = ko.OracleDataset(ds.num_entities, ds.num_relations, ds.training_triples, ds.validation_triples,
                           ds.testing_triples)
    seed_all(42)
    eng = ko.OracleEngine(om, ods, wl["hp"])
    frac, part = 1.0, ""
    if wl["mode"] == "sufficient":
        # a bounded sample: the first cpu_conversions conversion entities of each candidate
        # (they consume the same draws as the GPU's first ones), counted as that fraction
        # of a candidate
        nconv = min(len(ents), wl.get("cpu_conversions", len(ents)))
        frac = nconv / len(ents)
        part = f", {nconv} of {len(ents)} conversion entities each (counted as {frac:g} candidate)"
    times = []
    for c in cands:
        t0 = time.time()
        if wl["mode"] == "sufficient":
            eng.sufficient_relevance(pred, [c], ents[:nconv])
        else:
            eng.necessary_relevance(pred, [c])
        times.append(time.time() - t0)
    threads = max([t.get("num_threads", 1) for t in threadpool_info()] or [1])
    steady = times[1:]
    out = {"value": (frac * len(steady) / sum(steady)) if steady else None, "unit": "candidates/s",
           "cores": int(threads), "kind": "port", **_cores(),
           # the box gives one GPU's job a fixed CPU share (OMP_NUM_THREADS / MAX_JOBS are set
           # to it and are not to be raised): the oracle's BLAS runs on all of that share
           "cpu_share_of_this_gpu": int(os.environ.get("OMP_NUM_THREADS", threads)),
           "first_candidate_s": times[0] / frac, "steady_candidates": len(steady),
           "steady_s_per_candidate": (sum(steady) / len(steady) / frac) if steady else None,
           "sample": f"1 prediction of the workload: its first candidate (with the prediction's base post-training) "
                     f"timed apart, then {len(steady)} more as the steady state{part}; oracle numpy float32 "
                     f"full-table restatement, {int(threads)} BLAS threads, {sum(times):.1f}s"}
    if fixture is not None:
        run = fixture["runs"].get("fp32", {})
        cs = run.get("cand_seconds")
        if cs and len(cs) > 1:
            out["reference_container_rate"] = (len(cs) - 1) / sum(cs[1:])
            out["reference_container_first_candidate_s"] = cs[0]
            how = f"steady state over {len(cs) - 1} candidates, first candidate {cs[0]:.1f}s apart"
        elif run.get("seconds"):
            out["reference_container_rate"] = len(fixture["candidates"]) / run["seconds"]
            how = f"{len(fixture['candidates'])} candidates incl. the first (base post-training) in {run['seconds']:.0f}s"
        else:
            how = None
        if how:
            out["reference_container"] = (f"the reference itself (torch CPU, {fixture.get('threads')} threads of the "
                                          f"8-core development container, tools/conditioning.py): {how}")
    return out


def parity_sample(eng, wl, fixture, fallback):
    """GPU results on the fixture's prediction and candidates (fresh caches, seeds 42 as
    explain.py:144) and their rank deltas against the reference runs in the fixture."""
    import random
    import torch
    if fixture is not None:
        pred = tuple(fixture["pred"])
        cands = [tuple(c) for c in fixture["candidates"]]
        ents = fixture.get("entities_to_convert")
    else:
        pred, cands, ents = fallback
        cands = cands[:3]
    random.seed(42)
    np.random.seed(42)
    torch.manual_seed(42)
    eng.set_cache()
    if ents is not None:
        eng.entities_to_convert = list(ents)
    rels = eng.compute_relevance_batch(pred, [[c] for c in cands])
    if wl["mode"] == "sufficient":
        deltas = [pt["target_rank"] - b["target_rank"] for rj in eng.last_results for pt, b in rj]
    else:
        deltas = [pt["target_rank"] - b["target_rank"] for pt, b in eng.last_results]
    out = {"gpu_rank_deltas": deltas, "gpu_relevances": rels}
    if fixture is not None:
        for name, run in fixture["runs"].items():
            ref = run["rank_deltas"]
            out[name] = {"match_rate": float(np.mean([a == b for a, b in zip(deltas, ref)])),
                         "max_abs_diff": int(max(abs(a - b) for a, b in zip(deltas, ref)))}
        r32, r64 = fixture["runs"].get("fp32"), fixture["runs"].get("fp64")
        if r32 and r64:
            out["reference_fp32_vs_fp64_max_abs_diff"] = int(max(abs(a - b) for a, b in
                                                                 zip(r32["rank_deltas"], r64["rank_deltas"])))
    return pred, cands, ents, out


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_local_ranks(n):
    """``--gpus N`` without a launcher: run this same script under torchrun with N local
    ranks (127.0.0.1 rendezvous, the driver's own command shape) as a child process --
    never an exec, and nothing here has touched the GPU -- and return its exit status.
    Rank 0 of the child prints the JSON line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(sys.argv[0])]
    cmd += sys.argv[1:]
    log(f"[bench] launching {n} local ranks: {' '.join(cmd)}")
    return subprocess.call(cmd)


def load_builder_fixture(workload):
    """tests/golden/builder/<workload>__{fp32,fp64}.json: the reference's own pipeline
    (prefilter k = 20, StochasticBuilder at the default xsi) on the bench's predictions,
    seeds 42 once (tools/builder_fixture.py, development container).  Data only."""
    out = {}
    for v in ("fp32", "fp64"):
        path = os.path.join(ROOT, "tests", "golden", "builder", f"{workload}__{v}.json")
        if os.path.exists(path):
            with open(path) as f:
                rec = json.load(f)
            out[v] = rec["runs"][v]["explanations"]
            out["_file"] = os.path.relpath(path, ROOT).replace(f"__{v}.json", "__<variant>.json")
    return out


def builder_leg(model, ds, wl, n_preds, sharding=None):
    """The whole explanation builder (the reference's own recorded metric, #relevances /
    execution_time over StochasticBuilder.build_explanations, stochastic_builder.py:33-107;
    explain.py:196): topology prefilter k = 20, singleton rules in one batch, compound
    rules in speculative windows of 32 with generator rewinds -- the evaluations past a
    window's stop are device work the metric does not count (``wasted``).  Seeds 42 once,
    then the bench's first ``n_preds`` predictions in order, so the first one is the
    prediction of the reference's builder fixture."""
    import random
    import torch
    from kelpie_amd.pipeline import build_pipeline
    random.seed(42)
    np.random.seed(42)
    torch.manual_seed(42)
    # speculative windows: "auto" (kelpie_amd.builder) or a fixed size (KELPIE_BUILDER_WINDOW, A/B)
    win = os.environ.get("KELPIE_BUILDER_WINDOW", "auto")
    pipelined = os.environ.get("KELPIE_BUILDER_PIPELINED", "0") == "1"  # A/B: 1 = look-ahead windows
    pipe = build_pipeline(model, ds, wl["hp"], wl["mode"], window=win if win == "auto" else int(win),
                          pipelined=pipelined)
    pipe.engine.sharding = sharding
    preds = pick_preds(ds, n_preds, seed=1234)
    exs = []
    for pred in preds:
        exs.append(pipe.explain(pred=pred, prefilter_k=20))
    st = pipe.builder.stats
    n_rel = sum(ex["#relevances"] for ex in exs)
    t = sum(ex["execution_time"] for ex in exs)
    out = {"metric": "#relevances / execution_time (the reference's recorded builder metric)",
           "value": n_rel / t if t > 0 else None, "unit": "relevances/s", "predictions": len(exs),
           "relevances": n_rel, "execution_time_s": t, "evaluated": st["evaluated"], "wasted": st["wasted"],
           "engine_batches": st["batches"], "xsi": pipe.builder.xsi, "prefilter_k": 20,
           "speculative_window": "auto" if pipe.builder.auto else pipe.builder.spec_window,
           "windows_pipelined": pipe.builder.pipelined,
           # where the builder's time goes: engine batches (wall), and inside them the host
           # schedule (reference-order draws, slot assembly), packing and the library call
           "time_split_s": {k: round(st[k], 4) for k in ("batch_s", "schedule_s", "pack_s", "lib_s")},
           "per_prediction": [{"#relevances": ex["#relevances"], "execution_time_s": ex["execution_time"]}
                              for ex in exs]}
    fx = load_builder_fixture(wl["_name"])
    if fx and exs:
        got = exs[0]
        top = [[list(t) for t in rule] for rule, _ in got["rule_to_relevance"]]
        m = {"fixture": fx["_file"]}
        for v in ("fp32", "fp64"):
            if v in fx:
                ref = fx[v][0]
                m[v] = {"#relevances_equal": got["#relevances"] == ref["#relevances"],
                        "top10_rules_equal": top == [[list(t) for t in rule] for rule, _ in ref["rule_to_relevance"]],
                        "max_abs_relevance_diff_top10": max(
                            [abs(a[1] - b[1]) for a, b in zip(got["rule_to_relevance"], ref["rule_to_relevance"])]
                            or [0.0])}
        out["reference_match_first_prediction"] = m
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="complex-fb15k237-sufficient", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--preds-per-step", type=int, default=None, help="override the workload's predictions per step")
    ap.add_argument("--builder-preds", type=int, default=4,
                    help="predictions explained end to end by the builder leg after the timed region (0: none)")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # a plain `python bench.py --gpus N`: start the N local ranks ourselves, before
        # anything touches the GPU, and exit with their status
        sys.exit(launch_local_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        log(f"[bench] WORLD_SIZE={env_world} but --gpus {args.gpus}: launch one rank per GPU with --gpus N")
        sys.exit(2)
    _heartbeat()

    import torch
    from kelpie_amd import distributed as kd
    from kelpie_amd import NecessaryPostTrainingEngine, SufficientPostTrainingEngine
    rank, world, local = kd.init_from_env()
    wl = dict(WORKLOADS[args.workload], _name=args.workload)
    # one GPU per rank; on a box with fewer GPUs than ranks (gloo rehearsal) they share
    device = local % max(1, torch.cuda.device_count()) if torch.cuda.is_available() else 0
    ds, model, weights = build(wl, device, rank)
    engine_cls = SufficientPostTrainingEngine if wl["mode"] == "sufficient" else NecessaryPostTrainingEngine
    eng = engine_cls(model, ds, wl["hp"])

    if world > 1:
        eng.sharding = kd.SlotSharding()
    n_steps = args.warmup + args.steps
    # --preds-per-step, or KELPIE_PREDS_PER_STEP (A/B through tools/gpu_session.sh), overrides the workload's
    pps = args.preds_per_step or int(os.environ.get("KELPIE_PREDS_PER_STEP", "0") or 0) or None
    per_step = (pps or wl.get("preds_per_step", 1)) * world  # weak scaling
    my_preds = pick_preds(ds, n_steps * per_step, seed=1234)  # every rank schedules every batch
    import random
    random.seed(42)
    np.random.seed(42)
    torch.manual_seed(42)

    # per-prediction setup outside the timed region (prefilter / conversion entities
    # are excluded from the reference's execution_time as well)
    jobs = []
    t_setup = time.time()
    for i in range(n_steps):
        preds = my_preds[i * per_step:(i + 1) * per_step]
        step = []
        for pred in preds:
            cands = candidates_of(ds, pred, wl["candidates"])
            ents = None
            if wl["mode"] == "sufficient":
                ents = eng.select_entities_to_convert(pred, wl["convert"], 200)
            step.append((pred, cands, ents))
        jobs.append(step)
    log(f"[rank {rank}] setup (conversion entities) {time.time() - t_setup:.1f}s")

    breakdown = {"schedule_s": 0.0, "pack_s": 0.0, "lib_s": 0.0, "device_s": 0.0}

    def items_of(step):
        """One engine batch: every singleton candidate of the step's predictions."""
        if wl["mode"] == "sufficient":
            return [(pred, [[c] for c in cands], ents) for pred, cands, ents in step if ents]
        return [(pred, [[c] for c in cands]) for pred, cands, _ in step]

    # Each step is one batch started from cleared per-prediction caches (the base
    # post-trainings are part of the work).  compute_relevance_pipeline schedules
    # step k+1's reference-order draws on the host while step k runs on the GPU.
    # batches in flight (one device context each): 3 for the sufficient workloads, whose
    # small batches leave the device idle during a batch's planning and download
    # (default 588 -> 649 cand/s, profiles/r02v_depth.txt), and for ConvE, whose batch
    # boundaries (host planning of ~100 steps x 3,456 pair records, uploads) left the
    # device idle ~70 ms with two (433 / 436 -> 450 / 448 cand/s, profiles/r04x/); 2 for
    # the others (a third context costs the ComplEx necessary workload 10 %)
    depth = int(os.environ.get("KELPIE_PIPELINE_DEPTH", wl.get("depth", 2)))
    if args.warmup:
        eng.compute_relevance_pipeline([items_of(jobs[i]) for i in range(args.warmup)], depth=depth)
        # the pipeline's other device contexts (engine.compute_relevance_pipeline) run
        # the first warm-up batch too; no random draws are consumed
        eng.warm_contexts(items_of(jobs[0]), depth=depth)
    kd.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = eng.compute_relevance_pipeline([items_of(jobs[i]) for i in range(args.warmup, n_steps)], depth=depth)
    t_call = time.perf_counter() - t0
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    kd.barrier()
    elapsed = time.perf_counter() - t0
    log(f"[rank {rank}] timed region {elapsed * 1e3:.1f} ms, of which the pipeline call {t_call * 1e3:.1f} ms")
    recs = [[r, 0, 0, 0, 0] for o in outs for out in o for r in out]
    hot = [0.0, 0.0, 0]
    ivs = []
    for st in eng.last_batch_stats:
        hot = [hot[0] + st.get("hot_s", 0.0), hot[1] + st.get("hot_work", 0.0), hot[2] + st.get("hot_launches", 0)]
        if st.get("hot_iv") is not None:
            ivs.append(st["hot_iv"])
        for k in breakdown:
            breakdown[k] += st.get(k, 0.0)
    # Batches in flight on two device contexts can run their dominant kernels at the
    # same time, and then a launch's own duration includes the time it waited for the
    # other's workgroups.  The roofline divides the work by the time the device spent
    # in the kernel: the union of all launch intervals (shared time base,
    # kp_hot_intervals); with nothing overlapping it is the plain sum of durations.
    hot_union = union_seconds(np.concatenate(ivs)) if ivs else hot[0]
    elapsed_max = kd.max_over_ranks(elapsed)
    total_units = len(recs)  # every rank holds every result (counted once)

    # roofline of the dominant kernel, from its HIP-event launch durations inside the library
    if wl["model"] == "TransE":
        # algorithmic bytes: one fresh negative entity row per stepped pair,
        # plus every positive-side row once per slot (= once per epoch's pairs / epochs)
        d = model.dimension
        nbytes = 4.0 * d * hot[1] * (1.0 + 1.0 / wl["hp"]["epochs"])
        achieved = nbytes / hot_union / 1e9 if hot_union > 0 else None
        peak = 8000.0
        roof = {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                "frac": (achieved / peak) if achieved else None, "traffic": None, "kernel": "kp_te_posttrain",
                "actual_limit": ("VALU issue on the CUs of the longest slots (R = 200-400 rows, one workgroup "
                                 "per slot, ~1.9k SIMD cycles per stepped item, DESIGN.md section 6); the "
                                 "frozen table (11.6 MB) is L2/MALL-resident, so HBM is not the limit")}
    else:
        # 4 * D flops per (query row, frozen entity): s = q.E_e and O += w(s) E_e
        D = wl["dim"] * (2 if wl["model"] == "ComplEx" else 1)
        flops = 4.0 * D * hot[1]
        achieved = flops / hot_union / 1e12 if hot_union > 0 else None
        kname = "kp_attn<%d,%s>" % (-(-D // 16), "ATT_SOFTMAX_O" if wl["model"] == "ComplEx" else "ATT_BCE_O")
        from kelpie_amd._lib import attention_contraction
        if attention_contraction() == "bf16x3":
            # kp_attn3: each fp32 product as six bf16 MFMA products (exact three-piece
            # operand splits), so the fp32-equivalent ceiling is the dense bf16 MFMA peak / 6
            peak = BF16_DENSE_TFLOPS / 6.0
            kname = kname.replace("kp_attn<", "kp_attn3<")
        else:
            peak = 157.3
        roof = {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                "frac": (achieved / peak) if achieved else None, "traffic": None, "kernel": kname,
                "peak_basis": ("dense bf16 MFMA peak / 6 (six bf16 products per fp32 product)"
                               if peak != 157.3 else "dense fp32 MFMA peak")}
    cc = committed_counters(args.workload, roof["kernel"])
    roof["traffic"] = (cc["read"] + (cc["write"] or 0.0)) if cc["read"] else None
    roof["traffic_read"], roof["traffic_write"] = cc["read"], cc["write"]
    roof["traffic_source"] = cc["source"] or cc.get("note")
    if wl["model"] == "TransE" and cc["sq"] and cc["sq"].get("SQ_INSTS_VALU") and hot[2] and hot_union > 0:
        # its actual bound: VALU issue, one wave64 instruction per 2 cycles per SIMD
        # (MI355X_MICROARCH.md constants), 1,024 SIMDs at 2.4 GHz
        ach = cc["sq"]["SQ_INSTS_VALU"] / (hot_union / hot[2])
        pk = 1024 * 2.4e9 / 2.0
        roof["valu"] = {"achieved": ach, "peak": pk, "unit": "wave64 VALU instructions/s", "frac": ach / pk,
                        "source": cc["source"]}
    roof["launches"] = hot[2]
    # per-launch durations (what rocprofv3 --kernel-trace reports); with two batches
    # in flight they include waiting for the other batch's workgroups
    roof["avg_launch_ms"] = (hot[0] / hot[2] * 1e3) if hot[2] else None
    roof["device_kernel_ms_per_launch"] = (hot_union / hot[2] * 1e3) if hot[2] else None
    roof["timing"] = ("achieved = algorithmic work / union of the launches' intervals (HIP events on a shared "
                      "time base); avg_launch_ms = mean launch duration")

    builder = None
    if args.builder_preds > 0:
        # the whole builder over the workload's first predictions (every rank, the slots of
        # each engine batch sharded as above), after the timed singleton region
        builder = builder_leg(model, ds, wl, args.builder_preds, kd.SlotSharding() if world > 1 else None)
        log(f"[rank {rank}] builder leg: {json.dumps(builder)}")

    cpu = None
    parity = None
    if rank == 0:
        # rank-delta match rate against the reference itself: the committed fixture's
        # prediction and candidates, run through the engine after the timed region
        fixture = load_fixture(args.workload)
        pred, cands, ents = jobs[-1][0]
        eng.sharding = None  # rank 0 alone: no collective on this path
        pred, cands_s, ents, parity = parity_sample(eng, wl, fixture, (pred, cands, ents))
        log(f"[rank 0] parity sample vs reference: {json.dumps(parity)}")
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is an N = 1 number
            n_cpu = 5  # the first candidate (with the prediction's base post-trainings) + 4 steady
            cpu_cands = (cands_s + [c for c in candidates_of(ds, pred, wl["candidates"]) if c not in cands_s])[:n_cpu]
            try:
                cpu = cpu_baseline(wl, ds, weights, pred, cpu_cands, ents, fixture)
            except Exception as exc:  # the oracle is test infrastructure; report, never fake
                log(f"[rank 0] cpu baseline failed: {exc!r}")

    log(f"[rank {rank}] per-step breakdown (s): " +
        ", ".join(f"{k}={v / max(args.steps, 1):.4f}" for k, v in breakdown.items()) +
        f", wall={elapsed / max(args.steps, 1):.4f}")
    if rank == 0:
        ms = elapsed_max / max(args.steps, 1) * 1e3
        from kelpie_amd._lib import attention_contraction
        # the attention contraction: fp32 operands split exactly into three bf16 pieces,
        # six bf16 MFMA products per fp32 product (dropped terms below 2^-24 relative)
        dtype = "f32" if wl["model"] == "TransE" or attention_contraction() != "bf16x3" else "bf16x3 (fp32-emulated)"
        line = {"metric": METRIC, "value": total_units / elapsed_max, "unit": "candidates/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": "synthetic",
                "config": {"workload": args.workload, "model": wl["model"], "graph": wl["shape"] + " (synthetic)",
                           "dim": wl["dim"], "mode": wl["mode"],
                           # units actually evaluated per timed step (a prediction has at most
                           # `candidates` singleton candidates; low-degree subjects have fewer)
                           "candidates_per_step": total_units / max(args.steps, 1),
                           "candidates_cap_per_prediction": wl["candidates"],
                           "predictions_per_step": per_step,
                           "conversion_entities": wl.get("convert"), "epochs": wl["hp"]["epochs"],
                           "batches_in_flight": depth,
                           "parallelism": f"each batch's post-trainings sharded over {world} rank(s), "
                                          f"each rank schedules only its claimed slots (generators walked for "
                                          f"the rest), one all-gather per batch"},
                "rank_delta_match_rate": (parity.get("fp32") or {}).get("match_rate"),
                "rank_delta_max_abs_diff": (parity.get("fp32") or {}).get("max_abs_diff"),
                "rank_delta_vs": "the reference (fp32, CPU) on the fixture "
                                 + ((fixture or {}).get("_file") or "tests/golden/fullsize/<workload>.json (absent)"),
                "rank_delta_match_rate_ref_fp64": (parity.get("fp64") or {}).get("match_rate"),
                "rank_delta_max_abs_diff_ref_fp64": (parity.get("fp64") or {}).get("max_abs_diff"),
                "reference_fp32_vs_fp64_max_abs_diff": parity.get("reference_fp32_vs_fp64_max_abs_diff"),
                # the timed steps' relevances, bit for bit (A/B runs of two builds compare it)
                "results_sha16": hashlib.sha256(np.asarray([r[0] for r in recs], np.float64).tobytes()).hexdigest()[:16],
                "roofline": roof, "cpu_baseline": cpu, "builder": builder}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()

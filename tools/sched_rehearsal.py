"""Host schedule cost per rank under slot sharding (CPU rehearsal, no GPU, no collective).

For a workload of bench.py, times the host scheduling of one engine batch of N x the
per-GPU predictions (weak scaling, as ``bench.py --gpus N``) on every rank r of N
(``SlotSharding(rank=r, world=N)``: the rank claims its slots and only advances the
generators for the others), against the same batch scheduled in full by one process.

    python tools/sched_rehearsal.py --workload complex-fb15k237-sufficient --world 8
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="complex-fb15k237-sufficient", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--batches", type=int, default=3)
    a = ap.parse_args()
    from kelpie_amd import NecessaryPostTrainingEngine, SufficientPostTrainingEngine
    from kelpie_amd import distributed as kd
    wl = bench.WORKLOADS[a.workload]
    ds, model, _ = bench.build(wl, 0, 0)
    cls = SufficientPostTrainingEngine if wl["mode"] == "sufficient" else NecessaryPostTrainingEngine
    eng = cls(model, ds, wl["hp"])
    per = wl.get("preds_per_step", 1)
    preds = bench.pick_preds(ds, a.batches * per * a.world, seed=1234)
    # conversion entities (sufficient): the fixture's, as the reference selected them for its
    # prediction (the rehearsal has no GPU for kp_convertible); the schedule's cost depends
    # on their degrees, not on which prediction they were selected for
    fx = bench.load_fixture(a.workload) or bench.load_fixture(a.workload + "__p0")
    ents = fx["entities_to_convert"] if fx and wl["mode"] == "sufficient" else None

    def items(b, n):
        ps = preds[b * n:(b + 1) * n]
        if wl["mode"] == "sufficient":
            return [(p, [[c] for c in bench.candidates_of(ds, p, wl["candidates"])], ents) for p in ps]
        return [(p, [[c] for c in bench.candidates_of(ds, p, wl["candidates"])]) for p in ps]

    def run(sharding, n):
        eng.sharding = sharding
        bench.seed_all(42)
        t, slots_total, own = 0.0, 0, 0
        for b in range(a.batches):
            eng.set_cache()
            t0 = time.perf_counter()
            with eng.rng.deferred():
                slots, _, _ = eng._schedule_all(items(b, n), None)
            t += time.perf_counter() - t0
            slots_total += len(slots)
            own += sum(s.own for s in slots)
        return {"schedule_ms_per_batch": 1e3 * t / a.batches, "slots_per_batch": slots_total / a.batches,
                "own_per_batch": own / a.batches}

    out = {"workload": a.workload, "world": a.world, "preds_per_batch_per_rank": per,
           "one_rank_its_share": run(None, per), "one_process_all": run(None, per * a.world)}
    out["ranks"] = [run(kd.SlotSharding(rank=r, world=a.world, device="cpu"), per * a.world) for r in range(a.world)]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Per-fixture parity table against the reference itself (GPU box; TEST INFRASTRUCTURE:
reads the committed fixtures tests/golden/fullsize/*.json only).

For every fixture: the GPU's rank deltas on the fixture's prediction and candidates
(bench.parity_sample: fresh caches, seeds 42), their match rate and largest difference
against each reference variant (fp32 as the reference runs, fp32 with a permuted
reduction order, fp64), the reference's own fp32-vs-fp64 spread, and the number of
elements outside the per-element rule of tests/test_fullsize_reference.py.  One JSON
line per fixture -> stdout (DESIGN.md section 3's table).

    python tools/fullsize_table.py [fixture-name ...]
"""
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import bench
    from test_fullsize_reference import elementwise_misses, mirror_only
    from kelpie_amd import NecessaryPostTrainingEngine, SufficientPostTrainingEngine
    args = [a for a in sys.argv[1:] if a != "all"]  # "all" (or nothing): every fixture
    names = args or sorted(os.path.basename(p)[:-5]
                           for p in glob.glob(os.path.join(ROOT, "tests", "golden", "fullsize", "*.json")))
    built = {}
    for name in names:
        with open(os.path.join(ROOT, "tests", "golden", "fullsize", name + ".json")) as f:
            fx = json.load(f)
        wl_name = fx["workload"]
        wl = bench.WORKLOADS[wl_name]
        if wl_name not in built:
            built.clear()  # one model resident at a time
            built[wl_name] = bench.build(wl, 0, 0)
        ds, model, _ = built[wl_name]
        cls = SufficientPostTrainingEngine if wl["mode"] == "sufficient" else NecessaryPostTrainingEngine
        eng = cls(model, ds, wl["hp"])
        _, _, _, par = bench.parity_sample(eng, wl, fx, None)
        par["fixture"] = name
        par["elements"] = len(par["gpu_rank_deltas"])
        par["elementwise_misses"] = elementwise_misses(fx, par["gpu_rank_deltas"])
        # accepted only through the rule's mirror clause (reported apart)
        par["mirror_only"] = mirror_only(fx, par["gpu_rank_deltas"])
        f64 = fx["runs"]["fp64"]["rank_deltas"]
        par["gpu_vs_fp64_equal"] = sum(a == b for a, b in zip(par["gpu_rank_deltas"], f64))
        r32 = fx["runs"]["fp32"]["rank_deltas"]
        par["ref_fp32_vs_perm_match"] = sum(a == b for a, b in zip(r32, fx["runs"]["fp32_perm"]["rank_deltas"])) \
            / len(r32) if "fp32_perm" in fx["runs"] else None
        par["ref_fp32_vs_fp64_match"] = sum(a == b for a, b in zip(r32, fx["runs"]["fp64"]["rank_deltas"])) / len(r32)
        print(json.dumps(par), flush=True)


if __name__ == "__main__":
    main()

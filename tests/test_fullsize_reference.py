"""Full-size parity against the reference itself, at the bench workloads' own shapes
and the reference's random initialisers (tests/golden/fullsize/<workload>.json,
written by tools/conditioning.py in the development container: the reference in
fp32 as it runs, the same run with a permuted reduction order, and in fp64).

At the reference init the post-training is ill-conditioned: the reference's fp32
result differs from its own fp64 result by up to a rank place and ~1e-3 relative in
score.  The tolerances below are the reference's own spread,
stated per component:

* rank deltas, element by element: where every reference variant gives the same rank
  delta the GPU must equal it; where they disagree it must lie between them;
* the post-trained target scores (every base and pt post-training of the sample),
  measured against the fp64 reference: their mean relative error at most twice the
  fp32 reference's mean relative error, and their largest relative error within the
  larger of twice the reference's largest and the north star's 1e-4 -- the GPU must be
  about as accurate as the reference.  (Per score the errors are random: either side
  can land closer on any one post-training.)

The host-side test checks the fixtures themselves (the sample is well formed and the
reference runs agree with each other to the recorded spread).
"""
import glob
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "fullsize", "*.json")))
IDS = [os.path.basename(p)[:-5] for p in FIXTURES]


def _load(path):
    with open(path) as f:
        return json.load(f)


def split_results(fx_run, n_cands, n_conv):
    """(base scores [n_conv], pt scores [n_cands][n_conv]) from the reference's call log:
    the first call logs (base, pt) per conversion entity (one for necessary mode), later
    calls the pt results only (the base results are cached)."""
    calls = fx_run["results"]
    first = calls[0]
    base = [r["score"] for r in first[0::2]]
    pts = [[r["score"] for r in first[1::2]]] + [[r["score"] for r in c] for c in calls[1:]]
    assert len(base) == n_conv and len(pts) == n_cands and all(len(p) == n_conv for p in pts)
    return base, pts


def spread(fx):
    r32 = fx["runs"]["fp32"]["rank_deltas"]
    return max(max(abs(a - b) for a, b in zip(r32, run["rank_deltas"]))
               for name, run in fx["runs"].items() if name != "fp32")


def elementwise_misses(fx, got):
    """Rank deltas of ``got`` outside the reference's own per-element spread: where every
    reference variant (fp32, fp32 with a permuted reduction order, fp64) gives the same
    rank delta the result must equal it; where they disagree it must lie between the
    smallest and the largest of them, or be no farther from the fp64 run (the exact
    arithmetic) than the reference's own fp32 run is -- three variants sample the
    reference's rounding spread only thinly, and a result on the mirror side of the fp64
    value at the fp32 run's distance is the same spread (ConvE YAGO3-10 p2: the fp32 run
    meets fp64 on 1 of 20 elements, up to 6 places apart).  Returns [(index, got,
    reference values)]."""
    runs = [run["rank_deltas"] for run in fx["runs"].values()]
    f32 = fx["runs"].get("fp32", {}).get("rank_deltas")
    f64 = fx["runs"].get("fp64", {}).get("rank_deltas")
    out = []
    for i, g in enumerate(got):
        vals = sorted({r[i] for r in runs})
        if vals[0] <= g <= vals[-1]:
            continue
        if len(vals) > 1 and f32 is not None and f64 is not None and abs(g - f64[i]) <= abs(f32[i] - f64[i]):
            continue
        out.append((i, g, vals))
    return out


def mirror_only(fx, got):
    """Indices of the elements of ``got`` that the element-wise rule accepts only through
    its mirror clause (outside every reference variant's range, but no farther from the
    fp64 run than the fp32 run is), reported apart from the in-spread ones."""
    runs = [run["rank_deltas"] for run in fx["runs"].values()]
    f32 = fx["runs"].get("fp32", {}).get("rank_deltas")
    f64 = fx["runs"].get("fp64", {}).get("rank_deltas")
    out = []
    for i, g in enumerate(got):
        vals = sorted({r[i] for r in runs})
        if not vals[0] <= g <= vals[-1] and len(vals) > 1 and f32 is not None and f64 is not None \
                and abs(g - f64[i]) <= abs(f32[i] - f64[i]):
            out.append(i)
    return out


def test_elementwise_rule():
    fx = {"runs": {"fp32": {"rank_deltas": [1, 5, 3]}, "fp64": {"rank_deltas": [1, 6, 3]},
                   "fp32_perm": {"rank_deltas": [1, 5, 3]}}}
    assert elementwise_misses(fx, [1, 5, 3]) == [] and elementwise_misses(fx, [1, 6, 3]) == []
    assert elementwise_misses(fx, [2, 5, 3]) == [(0, 2, [1])]
    assert elementwise_misses(fx, [1, 8, 3]) == [(1, 8, [5, 6])] and elementwise_misses(fx, [1, 7, 3]) == []
    # the mirror side of fp64 at the fp32 run's distance (here 1) is inside the spread
    fx2 = {"runs": {"fp32": {"rank_deltas": [10, 4]}, "fp64": {"rank_deltas": [9, 4]},
                    "fp32_perm": {"rank_deltas": [10, 4]}}}
    assert elementwise_misses(fx2, [8, 4]) == [] and elementwise_misses(fx2, [7, 4]) == [(0, 7, [9, 10])]
    assert elementwise_misses(fx2, [9, 5]) == [(1, 5, [4])]  # all variants agree: equal only
    assert mirror_only(fx2, [8, 4]) == [0] and mirror_only(fx2, [9, 4]) == [] and mirror_only(fx, [1, 7, 3]) == [1]


@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_fixture_well_formed(path):
    fx = _load(path)
    assert {"fp32", "fp64"} <= set(fx["runs"])
    n_conv = len(fx["entities_to_convert"]) if fx.get("entities_to_convert") else 1
    for run in fx["runs"].values():
        assert len(run["rank_deltas"]) == len(fx["candidates"]) * n_conv
        split_results(run, len(fx["candidates"]), n_conv)
    # the reference's own fp32 / fp64 / reduction-order spread (ConvE YAGO3-10: 5 places,
    # ComplEx DB100K sufficient: 10 places over 99,605 ranked rows)
    assert spread(fx) <= 16


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_gpu_vs_reference_fullsize(path):
    import bench
    from kelpie_amd import NecessaryPostTrainingEngine, SufficientPostTrainingEngine
    fx = _load(path)
    wl = bench.WORKLOADS[fx["workload"]]
    ds, model, _ = bench.build(wl, 0, 0)
    cls = SufficientPostTrainingEngine if wl["mode"] == "sufficient" else NecessaryPostTrainingEngine
    eng = cls(model, ds, wl["hp"])
    _, cands, ents, par = bench.parity_sample(eng, wl, fx, None)
    n_conv = len(ents) if ents else 1
    misses = elementwise_misses(fx, par["gpu_rank_deltas"])
    assert not misses, misses
    # scores: as accurate as the reference, both against the fp64 reference
    pairs = [pb for rj in eng.last_results for pb in rj] if wl["mode"] == "sufficient" else eng.last_results
    g = np.array([b["target_score"] for _, b in pairs[:n_conv]] + [pt["target_score"] for pt, _ in pairs])
    b32, p32 = split_results(fx["runs"]["fp32"], len(cands), n_conv)
    b64, p64 = split_results(fx["runs"]["fp64"], len(cands), n_conv)
    a = np.array(b32 + list(np.ravel(p32)))
    e = np.array(b64 + list(np.ravel(p64)))
    err_g, err_a = np.abs(g - e) / np.abs(e), np.abs(a - e) / np.abs(e)
    assert err_g.mean() <= 2.0 * err_a.mean() + 1e-6, (err_g.mean(), err_a.mean())
    assert err_g.max() <= max(2.0 * err_a.max(), 1e-4), (err_g.max(), err_a.max())

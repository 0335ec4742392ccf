"""``bench.py --gpus N`` starts its own ranks (host only, gloo on the CPU stand-in).

A plain ``python bench.py --gpus 2`` -- the driver's N = 1 command shape with N = 2 --
must run two ranks (torchrun as a child process, before any GPU call) and print one
line with ``n_gpus: 2``; the sharded run must give the same relevances, bit for bit
(``results_sha16``), as one rank doing the same predictions.  A WORLD_SIZE that
disagrees with ``--gpus`` is refused.
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
RUNNER = os.path.join(HERE, "bench_standin.py")
ARGS = ["--workload", "transe-fb15k237-necessary", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
        "--builder-preds", "1"]


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "2"
    return env


def _line(args, env=None):
    out = subprocess.run([sys.executable, RUNNER] + args, cwd=ROOT, env=env or _env(), capture_output=True,
                         text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks_and_matches_one():
    one = _line(["--gpus", "1", "--preds-per-step", "2"] + ARGS)
    two = _line(["--gpus", "2", "--preds-per-step", "1"] + ARGS)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["predictions_per_step"] == one["config"]["predictions_per_step"] == 2
    assert two["config"]["candidates_per_step"] == one["config"]["candidates_per_step"]
    assert two["results_sha16"] == one["results_sha16"]
    # the builder leg (one prediction end to end) on two ranks equals the one-rank leg
    assert two["builder"]["relevances"] == one["builder"]["relevances"] > 0
    assert two["builder"]["evaluated"] == one["builder"]["evaluated"]


def test_bench_world_size_mismatch_refused():
    env = _env()
    env.update({"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + ARGS, cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr
    assert not [x for x in out.stdout.splitlines() if x.startswith("{")]

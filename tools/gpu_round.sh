#!/bin/bash
# One GPU-box pass: parity tests, every bench workload, and per workload the
# rocprofv3 kernel summary plus the HBM-traffic (FETCH_SIZE) counter pass.
# Usage (from the repo root, on the GPU box): bash tools/gpu_round.sh <tag> [workloads...]
set -eo pipefail
TAG=${1:-r01}
shift || true
WLS=${*:-complex-fb15k237-sufficient complex-fb15k237-necessary transe-fb15k237-necessary conve-yago310-necessary}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ROOT=$(pwd)
timeout -k 10 480 python -m pytest tests -m gpu -q -x > "$OUT/tests.log" 2>&1
for w in $WLS; do
  timeout -k 10 400 python bench.py --workload "$w" --steps 3 --warmup 1 > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
done
export TMPDIR=/tmp
cd /tmp
for w in $WLS; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_$w" -o run -- \
    python3 "$ROOT/bench.py" --workload "$w" --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/$OUT/prof_$w.log" 2>&1
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$ROOT/$OUT/pmc_$w" -o run -- \
    python3 "$ROOT/bench.py" --workload "$w" --steps 2 --warmup 1 --no-cpu-baseline > "$ROOT/$OUT/pmc_$w.log" 2>&1
done

#!/bin/bash
# Kernel-trace summary of one bench workload (GPU box): bash tools/kstats.sh <out-dir> <workload> [steps]
set -eo pipefail
OUT=$1; WL=$2; ST=${3:-2}
R=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof_$WL" -o run -- \
  python3 "$R/bench.py" --workload "$WL" --steps "$ST" --warmup 1 --no-cpu-baseline > "$R/$OUT/prof_$WL.log" 2>&1

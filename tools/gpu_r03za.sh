#!/bin/bash
# r03za: GPU suite + driver-shaped default bench + kernel trace after the kp_cx_contrib rework
set -o pipefail
O=gpurun_out/r03za; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
cut -c1-300 $O/bench_default.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_default.log 2>&1 || exit 1
echo done

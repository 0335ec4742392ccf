#!/bin/bash
# r03zc: kernel trace of the attention micro-benchmark (dispatch durations vs the
# HIP-event per-launch time) and the LSE-merge change's ComplEx GPU tests
set -o pipefail
O=gpurun_out/r03zc; mkdir -p $O
R=$(pwd)
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/prof_micro -o run -- $R/variants/attn_micro_base 25 0 14541 3100 30 0.05 > $R/$O/micro.log 2>&1 || exit 1
cd $R
grep -h '"ms"' $O/micro.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "complex or fullsize or smoke or verification" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || exit 1
cut -c1-260 $O/bench_default.json

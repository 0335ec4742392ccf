#!/bin/bash
# r03zv: the pure-MFMA boundary probe, then the closing run of the round: GPU suite, smoke,
# the driver-shaped default bench line and its kernel-trace summary
set -o pipefail
O=gpurun_out/r03zv; mkdir -p $O
R=$(pwd)
KP_MICRO_MFMA=1 timeout -k 10 120 variants/attn_micro_base 25 0 14541 3100 30 0.05 > $O/mfma.jsonl || exit 1
cat $O/mfma.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
cut -c1-260 $O/bench_default.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_default.log 2>&1 || exit 1
echo done

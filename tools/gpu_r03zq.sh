#!/bin/bash
# r03zq: s_memrealtime calibration, GPU suite on the current tree, TransE and default bench lines
set -o pipefail
O=gpurun_out/r03zq; mkdir -p $O
KP_MICRO_RTCAL=1 timeout -k 10 60 variants/attn_micro_base 25 0 14541 3100 30 0.05 > $O/rtcal.jsonl || exit 1
cat $O/rtcal.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 6 --warmup 1 --no-cpu-baseline > $O/transe_$rep.json 2> $O/transe_$rep.err || exit 1
  echo "transe $(cut -c100-190 $O/transe_$rep.json) $(grep breakdown $O/transe_$rep.err | cut -c40-)"
done

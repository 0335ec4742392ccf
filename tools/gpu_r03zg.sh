#!/bin/bash
# r03zg: TransE bench, the draw scratch in ordinary memory (rngjv) vs in the page-locked
# arena (rngnew), alternating on one box
set -o pipefail
O=gpurun_out/r03zg; mkdir -p $O
for v in rngjv rngnew rngjv rngnew; do
  KP_RNG_STATS=1 KELPIE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary \
    --steps 6 --warmup 1 --no-cpu-baseline > $O/transe_$v.json 2>> $O/transe_$v.err || exit 1
  echo "$v $(cut -c100-200 $O/transe_$v.json)"; grep breakdown $O/transe_$v.err | tail -1
done

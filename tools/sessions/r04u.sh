#!/bin/bash
# r04u: where the ComplEx call blocks while enqueueing (KP_HOST_TIMES per-phase stamps).
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
for i in 1; do
  KP_HOST_TIMES=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  echo "$i $(grep -o '"value": [0-9.]*' $O/bench_$i.json) $(grep -o '"results_sha16": "[0-9a-f]*"' $O/bench_$i.json)"
done
grep "kp_cx\]" $O/bench_1.err | tail -8
echo done

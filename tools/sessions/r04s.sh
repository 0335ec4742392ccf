#!/bin/bash
# r04s: where the ComplEx library call's host time goes (KP_HOST_TIMES=1: checks and
# planning before the first upload, enqueueing, waiting), on the default bench.
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
KP_HOST_TIMES=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
grep -o '"value": [0-9.]*' $O/bench.json
grep "kp_cx\]" $O/bench.err | tail -30
echo done

#!/bin/bash
# A/B timing of the kp_attn3 work partitions on the GPU box (same box, same inputs):
#   bash tools/attn_ab.sh <tag>
# KP_ATTN_PART=streamk forces stream-K; the default chooses per launch (attn_plan_ctx).
set -o pipefail
T=$1
mkdir -p gpurun_out/$T
for wl in complex-fb15k237-sufficient complex-fb15k237-necessary conve-yago310-necessary; do
  for part in default streamk; do
    KP_ATTN_PART=$part timeout -k 10 300 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/$T/${part}_$wl.json 2> gpurun_out/$T/${part}_$wl.err || exit 1
  done
done

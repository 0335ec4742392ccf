#!/bin/bash
# A/B of the engine pipeline depth (GPU box): bash tools/depth_ab.sh <tag> [workloads...]
set -o pipefail
T=$1; shift
WLS=${*:-complex-fb15k237-sufficient complex-fb15k237-necessary conve-yago310-necessary transe-fb15k237-necessary}
mkdir -p gpurun_out/$T
for wl in $WLS; do
  for d in ${DEPTHS:-1 2}; do
    KELPIE_PIPELINE_DEPTH=$d timeout -k 10 300 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/$T/d${d}_$wl.json 2> gpurun_out/$T/d${d}_$wl.err || exit 1
  done
done

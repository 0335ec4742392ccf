#!/bin/bash
# r03zz: round-2/3 DMA-schedule variants re-timed at the settled clock (the micro-benchmark
# now runs 1 s of launches first), interleaved twice on one box
set -o pipefail
bash tools/attn_micro.sh run r03zz base spread2 spread0 early || exit 1
for v in base spread2 spread0 early; do echo "== $v"; cut -c1-34,100-175 gpurun_out/r03zz/$v.jsonl; done

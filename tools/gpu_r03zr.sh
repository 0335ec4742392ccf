#!/bin/bash
# r03zr: dispatch cost of kp_attn3's resource footprint (every workgroup exits at entry)
set -o pipefail
O=gpurun_out/r03zr; mkdir -p $O
for rep in 1 2; do for v in base early; do
  timeout -k 10 120 variants/attn_micro_$v 25 0 14541 3100 30 0.05 >> $O/$v.jsonl || exit 1
done; done
cat $O/base.jsonl $O/early.jsonl

#!/bin/bash
# r03zx: the attention's per-launch time after >= 2 s of back-to-back launches (clock settled)
# against the stamped launch's workgroup span, FB15k-237 and DB100K shapes
set -o pipefail
O=gpurun_out/r03zx; mkdir -p $O
for args in "25 0 14541 3100 30" "25 0 99604 1800 10" "13 2 123182 4270 10"; do
  timeout -k 10 120 variants/attn_micro_clock $args 0.05 >> $O/warm.jsonl || exit 1
done
cat $O/warm.jsonl

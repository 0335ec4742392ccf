#!/bin/bash
# r03zm: where the ~60 us per attention dispatch outside the workgroups go: the kernel
# without its O-partial stores (diagnostic) beside the product kernel, interleaved; then r03zl
set -o pipefail
O=gpurun_out/r03zm; mkdir -p $O
for rep in 1 2; do
  for v in base noostore; do
    timeout -k 10 120 variants/attn_micro_$v 25 0 14541 3100 30 0.05 >> $O/$v.jsonl || exit 1
    timeout -k 10 120 variants/attn_micro_$v 25 0 99604 1800 10 0.05 >> $O/$v.jsonl || exit 1
  done
done
for v in clock noostoreclock; do timeout -k 10 120 variants/attn_micro_$v 25 0 14541 3100 30 0.05 >> $O/spans.jsonl || exit 1; done
cat $O/base.jsonl $O/noostore.jsonl $O/spans.jsonl
bash tools/gpu_r03zl.sh

#!/bin/bash
# r03zi: dispatch cost of an empty kernel with kp_attn3's launch shape, then the attention
set -o pipefail
O=gpurun_out/r03zi; mkdir -p $O
KP_MICRO_EMPTY=1 timeout -k 10 120 variants/attn_micro_base 25 0 14541 3100 30 0.05 > $O/empty.jsonl || exit 1
KP_MICRO_EMPTY=1 timeout -k 10 120 variants/attn_micro_base 25 0 99604 1800 30 0.05 >> $O/empty.jsonl || exit 1
cat $O/empty.jsonl

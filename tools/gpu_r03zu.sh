#!/bin/bash
# r03zu: does a pure-MFMA kernel (no memory traffic) show the same time outside its workgroups?
set -o pipefail
O=gpurun_out/r03zu; mkdir -p $O
KP_MICRO_MFMA=1 timeout -k 10 120 variants/attn_micro_base 25 0 14541 3100 30 0.05 > $O/mfma.jsonl || exit 1
cat $O/mfma.jsonl

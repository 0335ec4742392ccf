#!/bin/bash
# r03zw: which part of the attention's traffic puts time outside the workgroups: a pure-MFMA
# kernel of the attention's launch shape plus LDS reads, plus global loads, plus both
set -o pipefail
O=gpurun_out/r03zw; mkdir -p $O
KP_MICRO_MFMA2=1 timeout -k 10 120 variants/attn_micro_base 25 0 14541 3100 30 0.05 > $O/mfma2.jsonl || exit 1
cat $O/mfma2.jsonl

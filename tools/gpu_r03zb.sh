#!/bin/bash
# r03zb: kp_attn3 workgroup spans (diagnostic clock build) and the TransE draw workers' busy times
set -o pipefail
O=gpurun_out/r03zb; mkdir -p $O
for args in "25 0 14541 3100 30" "25 0 14541 6200 30" "25 0 99604 1800 10"; do
  timeout -k 10 120 variants/attn_micro_clock $args 0.05 >> $O/attn_spans.jsonl || exit 1
done
cat $O/attn_spans.jsonl
KP_RNG_STATS=1 timeout -k 10 300 python tools/host_profile.py --repeats 3 > $O/host_profile.txt 2>&1 || exit 1
grep -E "kp_rng|batch" $O/host_profile.txt

#!/bin/bash
# r03zp: is s_memrealtime 100 MHz on this part?  (a spin kernel timed by HIP events)
set -o pipefail
O=gpurun_out/r03zp; mkdir -p $O
KP_MICRO_RTCAL=1 timeout -k 10 60 variants/attn_micro_base 25 0 14541 3100 30 0.05 > $O/rtcal.jsonl || exit 1
cat $O/rtcal.jsonl

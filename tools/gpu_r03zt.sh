#!/bin/bash
# r03zt: the attention dispatch's time outside its workgroups under other LDS-DMA forms:
# product (buffer-descriptor DMA), the per-lane global_load_lds form (KP_BUF_DMA=0), no DMA at all
# (diagnostic, wrong results): per-launch ms and workgroup spans
set -o pipefail
O=gpurun_out/r03zt; mkdir -p $O
for v in base nobuf nodma; do timeout -k 10 120 variants/attn_micro_$v 25 0 14541 3100 30 0.05 >> $O/ms.jsonl || exit 1; done
for v in clock nobufclock nodmaclock; do echo "== $v" >> $O/spans.jsonl; timeout -k 10 120 variants/attn_micro_$v 25 0 14541 3100 30 0.05 >> $O/spans.jsonl || exit 1; done
cut -c1-30,100-170 $O/ms.jsonl; cat $O/spans.jsonl

#!/bin/bash
# r03zh: GIL switch-interval A/B (TransE and the default workload) and the attention
# workgroup spans with the stamps as first / last instructions
set -o pipefail
O=gpurun_out/r03zh; mkdir -p $O
timeout -k 10 120 variants/attn_micro_clock 25 0 14541 3100 30 0.05 > $O/spans.jsonl || exit 1
cat $O/spans.jsonl
for rep in 1 2; do
for sw in "" 500; do
  KELPIE_GIL_SWITCH_US=$sw timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 6 --warmup 1 --no-cpu-baseline > $O/t.json 2> $O/t.err || exit 1
  echo "transe sw=$sw $(cut -c100-175 $O/t.json) $(grep breakdown $O/t.err | tail -1 | cut -c40-)"
done
done
for sw in "" 500; do
  KELPIE_GIL_SWITCH_US=$sw timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/d.json 2> $O/d.err || exit 1
  echo "default sw=$sw $(cut -c100-175 $O/d.json)"
done

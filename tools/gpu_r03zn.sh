#!/bin/bash
# r03zn: write-through (sc1) O-partial stores vs plain: micro (interleaved), workgroup spans,
# then the default bench alternating the two library builds
set -o pipefail
O=gpurun_out/r03zn; mkdir -p $O
bash tools/attn_micro.sh run r03zn base osc1 || exit 1
for v in clock osc1clock; do timeout -k 10 120 variants/attn_micro_$v 25 0 14541 3100 30 0.05 >> $O/spans.jsonl || exit 1; done
cat $O/base.jsonl $O/osc1.jsonl $O/spans.jsonl
for rep in 1 2; do
for v in cur osc1; do
  KELPIE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err || exit 1
  echo "$v $(cut -c100-190 $O/b_$v.json) frac $(python -c "import json;print(round(json.load(open('$O/b_$v.json'))['roofline']['frac'],4))")"
done
done

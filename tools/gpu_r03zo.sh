#!/bin/bash
# r03zo: the attention dispatch's time outside its workgroups -- product kernel vs no O
# stores (diagnostic) vs write-through (sc1) O stores: micro interleaved, workgroup spans;
# then the default bench alternating plain / sc1 builds; then r03zl (predictions per batch)
set -o pipefail
O=gpurun_out/r03zo; mkdir -p $O
bash tools/attn_micro.sh run r03zo base noostore osc1 || exit 1
for v in clock noostoreclock osc1clock; do echo "== $v" >> $O/spans.jsonl; timeout -k 10 120 variants/attn_micro_$v 25 0 14541 3100 30 0.05 >> $O/spans.jsonl || exit 1; done
for v in base noostore osc1; do echo "== $v"; cut -c1-40,100-200 $O/$v.jsonl; done
cat $O/spans.jsonl
for rep in 1 2; do
for v in cur osc1; do
  KELPIE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err || exit 1
  echo "$v $(cut -c100-190 $O/b_$v.json) frac $(python -c "import json;print(round(json.load(open('$O/b_$v.json'))['roofline']['frac'],4))")"
done
done
bash tools/gpu_r03zl.sh

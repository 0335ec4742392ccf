#!/bin/bash
# r03ze: O-partial store form A/B in the attention micro-benchmark (plain vs nontemporal),
# interleaved on one box, with the workgroup spans and the dispatch durations
set -o pipefail
O=gpurun_out/r03ze; mkdir -p $O
R=$(pwd)
bash tools/attn_micro.sh run r03ze base ont || exit 1
for v in clock ontclock; do timeout -k 10 120 variants/attn_micro_$v 25 0 14541 3100 30 0.05 >> $O/spans.jsonl || exit 1; done
export TMPDIR=/tmp
cd /tmp
for v in base ont; do
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/$O/prof_$v -o run -- $R/variants/attn_micro_$v 25 0 14541 3100 30 0.05 > $R/$O/trace_$v.log 2>&1 || exit 1
done
cd $R
cat $O/base.jsonl $O/ont.jsonl $O/spans.jsonl

#!/bin/bash
# r03y: TransE host-draw A/B (new kp_rng vs the previous commit's), then this round's
# kernel-trace summary and FETCH_SIZE pass of the default workload.
set -o pipefail
O=gpurun_out/r03y; mkdir -p $O
R=$(pwd)
for v in rngnew rngold rngnew rngold; do
  KELPIE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary \
    --steps 4 --warmup 1 --no-cpu-baseline > $O/transe_$v.json 2>> $O/transe_$v.err || exit 1
  tail -c 300 $O/transe_$v.json; echo
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_default.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_default -o run -- \
  python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $R/$O/pmc_default.log 2>&1 || exit 1

cd $R
# in-kernel clock of kp_attn3 (diagnostic build) beside the product build, FB15k-237 and DB100K shapes
for args in "25 0 14541 3100 30" "25 0 99604 1800 10"; do
  timeout -k 10 120 variants/attn_micro_base $args 0.05 >> $O/attn_clock.jsonl || exit 1
  timeout -k 10 120 variants/attn_micro_clock $args 0.05 >> $O/attn_clock.jsonl || exit 1
done
cat $O/attn_clock.jsonl

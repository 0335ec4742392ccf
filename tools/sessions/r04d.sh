#!/bin/bash
# r04d: the wave-pair attention kp_attn5 against kp_attn3 in the micro-benchmark (fp64
# check, settled clock, FB15k-237 and DB100K shapes, alternating), then r04c: ComplEx
# step split + fp64 TransE / ConvE ranks (parity, full-size fixtures, default bench A/B
# against the round-3 build, ConvE dropout parity, kernel trace).
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
R=$(pwd)
for rep in 1 2; do
  for k in 0 1; do
    for args in "25 0 14541 3100 30" "25 0 99604 1800 10"; do
      KP_MICRO_ATTN5=$k timeout -k 10 120 variants/attn_micro_cur $args 0.05 >> $O/micro.jsonl || { echo "micro failed k=$k $args"; exit 1; }
    done
  done
done
cut -c1-250 $O/micro.jsonl
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -v \
  -k "complex or fullsize" --timeout 120 --timeout-method thread > $O/tests_complex.txt 2>&1
echo "complex+fullsize tests rc=$?"; grep -E "FAILED|passed|failed" $O/tests_complex.txt | tail -8
for i in 1 2; do
  for v in r03 new; do
    L=$R/kelpie_amd/libkelpie_hip.so; [ $v = r03 ] && L=$R/variants/lib_r03.so
    KELPIE_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    cut -c1-200 $O/bench_${v}_$i.json
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "conve" --timeout 120 \
  --timeout-method thread > $O/tests_conve.txt 2>&1
echo "conve tests rc=$?"; grep -E "FAILED|passed|failed" $O/tests_conve.txt | tail -8
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_default.log 2>&1 || exit 1
echo done

#!/bin/bash
# r04e: the staggered wave-pair attention (kp_attn5: two groups one interval apart, so
# one wave's softmax sits beside the other's MFMAs) against kp_attn3 in the micro-
# benchmark (fp64 check, settled clock, alternating), then the ComplEx GPU parity tests
# and the default bench line with it switched on (KP_ATTN_PAIR=1); then the ConvE
# parity tests under the LDS-DMA diagnostic builds.
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
for rep in 1 2; do
  for k in 0 1; do
    for args in "25 0 14541 3100 30" "25 0 99604 1800 10"; do
      KP_MICRO_ATTN5=$k timeout -k 10 120 variants/attn_micro_cur $args 0.05 >> $O/micro.jsonl || { echo "micro failed k=$k $args"; exit 1; }
    done
  done
done
cut -c1-250 $O/micro.jsonl
KP_ATTN_PAIR=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -v \
  -k "complex" --timeout 120 --timeout-method thread > $O/tests_pair.txt 2>&1
echo "complex tests (pair) rc=$?"; grep -E "FAILED|passed|failed" $O/tests_pair.txt | tail -8
for i in 1 2; do
  for k in 0 1; do
    KP_ATTN_PAIR=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_pair${k}_$i.json 2> $O/bench_pair${k}_$i.err || exit 1
    cut -c1-200 $O/bench_pair${k}_$i.json
  done
done
# the ConvE LDS-DMA hazard: the spread DMA (KP_DMA_SPREAD_ALL) on the compiler-visible
# read form, alone and with each diagnostic (vmcnt(0) / lgkmcnt(0) after every piece, M0
# saved and restored around it): the ConvE GPU parity tests under each build
for v in spr spr_vm0 spr_lgkm0 spr_m0; do
  KELPIE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v \
    -k "conve" --timeout 120 --timeout-method thread > $O/tests_dma_$v.txt 2>&1
  echo "dma variant $v rc=$?"; grep -E "passed|failed" $O/tests_dma_$v.txt | tail -1
done
echo done

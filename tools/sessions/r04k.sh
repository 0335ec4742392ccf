#!/bin/bash
# r04k: ConvE attention on the asm read form (KP_ASM_ALL=1 with the per-lane DMA, so two
# workgroups still fit per CU; and with the buffer DMA, one per CU) against the product's
# compiler-visible form in the micro-benchmark; the ConvE GPU parity tests under the asm
# form; ConvE bench lines: round-4 tree before the kp_cv_update change (lib_cx03), this
# tree, this tree with the asm form.
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
R=$(pwd)
for rep in 1 2; do
  for v in cur asm13 asm13b; do
    timeout -k 10 120 variants/attn_micro_$v 13 2 123182 4270 10 0.05 >> $O/micro_$v.jsonl || { echo "micro $v failed"; exit 1; }
  done
done
for v in cur asm13 asm13b; do echo "$v: $(cut -c1-200 $O/micro_$v.jsonl | tr '\n' ' ')"; done
KELPIE_HIP_LIB=$R/variants/lib_asm13.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py \
  -m gpu -v -k "conve" --timeout 120 --timeout-method thread > $O/tests_conve_asm13.txt 2>&1
echo "conve tests (asm13) rc=$?"; grep -E "FAILED|passed|failed" $O/tests_conve_asm13.txt | tail -5
lib() { case $1 in cx03) echo $R/variants/lib_cx03.so ;; asm13) echo $R/variants/lib_asm13.so ;; *) echo $R/kelpie_amd/libkelpie_hip.so ;; esac; }
for i in 1 2; do
  for v in cx03 cur asm13; do
    KELPIE_HIP_LIB=$(lib $v) timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 4 --warmup 1 \
      --no-cpu-baseline > $O/bench_conve_${v}_$i.json 2> $O/bench_conve_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"value": [0-9.]*' $O/bench_conve_${v}_$i.json) $(grep -o '"results_sha16": "[0-9a-f]*"' $O/bench_conve_${v}_$i.json)"
  done
done
echo done

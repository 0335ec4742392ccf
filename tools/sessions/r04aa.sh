#!/bin/bash
# r04aa: grown device buffers kept until teardown (no mid-run hipFree, which waits for every
# context) and the ConvE rank buffers on the context: ConvE and ComplEx GPU parity tests,
# two ConvE lines with the host-time split, two default lines.
set -o pipefail
O=gpurun_out/r04aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -v \
  -k "conve or complex" --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $O/tests.txt | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for i in 1 2; do
  KP_HOST_TIMES=1 timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 4 --warmup 1 \
    --no-cpu-baseline > $O/bench_conve_$i.json 2> $O/bench_conve_$i.err || exit 1
  echo "conve $i $(grep -o '"value": [0-9.]*' $O/bench_conve_$i.json)"
done
grep "kp_cv\]" $O/bench_conve_2.err | tail -6
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_default_$i.json 2> $O/bench_default_$i.err || exit 1
  echo "default $i $(grep -o '"value": [0-9.]*' $O/bench_default_$i.json) $(grep -o '"results_sha16": "[0-9a-f]*"' $O/bench_default_$i.json)"
done
echo done

#!/bin/bash
# r04t: the ranking's uploads ahead of the ComplEx step loop (no host round trip between the
# loop and the rank kernels): ComplEx GPU parity tests, three default bench lines with the
# host-time diagnostic.
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "complex" --timeout 200 \
  --timeout-method thread > $O/tests_complex.txt 2>&1
rc=$?
echo "complex tests rc=$rc"; grep -E "FAILED|passed|failed" $O/tests_complex.txt | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for i in 1 2 3; do
  KP_HOST_TIMES=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  echo "$i $(grep -o '"value": [0-9.]*' $O/bench_$i.json) $(grep -o '"results_sha16": "[0-9a-f]*"' $O/bench_$i.json)"
done
grep "kp_cx\]" $O/bench_1.err | tail -8
echo done

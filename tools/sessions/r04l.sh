#!/bin/bash
# r04l: the shared-encoder split of the fused ConvE path (kelpie-row, pair and relation
# terms of the FC; kp_cv_fused.hpp): the ConvE GPU parity tests, then ConvE bench lines
# with it off (KP_CV_SHARED=0) and on, alternating.
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -v \
  -k "conve" --timeout 120 --timeout-method thread > $O/tests_conve.txt 2>&1
rc=$?
echo "conve tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $O/tests_conve.txt | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for i in 1 2; do
  for v in 0 1; do
    KP_CV_SHARED=$v timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 4 --warmup 1 \
      --no-cpu-baseline > $O/bench_conve_shared${v}_$i.json 2> $O/bench_conve_shared${v}_$i.err || exit 1
    echo "shared=$v $i $(grep -o '"value": [0-9.]*' $O/bench_conve_shared${v}_$i.json) $(grep -o '"rank_delta_match_rate[a-z_0-9]*": [0-9.]*' $O/bench_conve_shared${v}_$i.json | tr '\n' ' ')"
  done
done
echo done

#!/bin/bash
# r04r: the DBpedia50 GPU pipeline test under the element-wise rule, then the pipeline's
# early start (the next batch starts on a freed context before the finished batch's results
# are collected) against collect-then-start (KELPIE_PIPELINE_EARLY_START=0), alternating.
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dbpedia50.py -m gpu -v --timeout 200 --timeout-method thread \
  > $O/tests_dbpedia50.txt 2>&1
echo "dbpedia50 rc=$?"; grep -E "FAILED|passed|failed" $O/tests_dbpedia50.txt | tail -3
for i in 1 2 3; do
  for v in 0 1; do
    KELPIE_PIPELINE_EARLY_START=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_early${v}_$i.json 2> $O/bench_early${v}_$i.err || exit 1
    echo "early=$v $i $(grep -o '"value": [0-9.]*' $O/bench_early${v}_$i.json)"
  done
done
echo done

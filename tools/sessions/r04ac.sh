#!/bin/bash
# r04ac: batches in flight 3 against 4 again now that no mid-run hipFree stalls a batch
# thread behind the other contexts: default line three times, ConvE twice, alternating.
set -o pipefail
O=gpurun_out/r04ac; mkdir -p $O
for i in 1 2 3; do
  for d in 3 4; do
    KELPIE_PIPELINE_DEPTH=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_depth${d}_$i.json 2> $O/bench_depth${d}_$i.err || exit 1
    echo "default depth=$d $i $(grep -o '"value": [0-9.]*' $O/bench_depth${d}_$i.json)"
  done
done
for i in 1 2; do
  for d in 3 4; do
    KELPIE_PIPELINE_DEPTH=$d timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 4 --warmup 1 \
      --no-cpu-baseline > $O/bench_conve_depth${d}_$i.json 2> $O/bench_conve_depth${d}_$i.err || exit 1
    echo "conve depth=$d $i $(grep -o '"value": [0-9.]*' $O/bench_conve_depth${d}_$i.json)"
  done
done
echo done

#!/bin/bash
# r03zj: round-3 bench line of every workload on the current tree (default driver-shaped
# with the CPU baseline; the others --steps 3 --warmup 1 without it)
set -o pipefail
O=gpurun_out/r03zj; mkdir -p $O
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
cut -c1-200 $O/bench_default.json
for w in complex-fb15k237-necessary transe-fb15k237-necessary complex-db100k-necessary complex-db100k-sufficient \
         conve-yago310-necessary complex-fb15k237-sufficient-k50 complex-fb15k237-sufficient-k100; do
  timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  echo "$w $(cut -c100-200 $O/bench_$w.json)"
done

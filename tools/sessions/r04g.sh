#!/bin/bash
# r04g: the full-size parity table (every fixture against the reference variants) and the
# bench lines of the other workloads.
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 600 python -u tools/fullsize_table.py > $O/fullsize_table.jsonl 2> $O/fullsize_table.err || { tail -5 $O/fullsize_table.err; exit 1; }
cut -c1-220 $O/fullsize_table.jsonl
for w in conve-yago310-necessary transe-fb15k237-necessary complex-fb15k237-necessary complex-db100k-sufficient; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  cut -c1-160 $O/bench_$w.json
done
# TransE at 20 steps (the 3-step line above includes the first batch's unoverlapped
# schedule) with the draw workers' busy times per batch on stderr
KP_RNG_STATS=1 timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 20 --warmup 3 \
  --no-cpu-baseline > $O/bench_transe20.json 2> $O/bench_transe20.err || exit 1
cut -c1-160 $O/bench_transe20.json
echo done

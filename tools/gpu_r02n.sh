set -eo pipefail
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 4 --warmup 1 > $O/bench_transe.json 2> $O/bench_transe.err
timeout -k 10 300 python tools/host_profile.py --workload transe-fb15k237-necessary > $O/host_profile_transe.txt 2>&1
bash tools/kstats.sh $O complex-fb15k237-sufficient 4
bash tools/attn_pmc.sh $O/pmc complex-fb15k237-sufficient
for w in complex-fb15k237-necessary complex-db100k-necessary complex-db100k-sufficient conve-yago310-necessary; do
  timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 > $O/bench_$w.json 2> $O/bench_$w.err
done

set -eo pipefail
# round-2 closing run: every GPU test, smoke, the default bench with its kernel summary and
# counter passes, and the TransE / ConvE / baseline-engine benches
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
cat $O/bench_default.json
bash tools/kstats.sh $O complex-fb15k237-sufficient 4
bash tools/attn_pmc.sh $O/pmc complex-fb15k237-sufficient
timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 4 --warmup 1 > $O/bench_transe.json 2> $O/bench_transe.err
timeout -k 10 900 python bench.py --workload conve-yago310-necessary --steps 3 --warmup 1 > $O/bench_conve.json 2> $O/bench_conve.err
timeout -k 10 300 python tools/baselines_bench.py --preds 16 > $O/baselines.jsonl 2> $O/baselines.err
echo done

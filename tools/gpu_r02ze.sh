set -eo pipefail
# re-entry check after the container rebuild: every GPU test, smoke, the default and TransE benches
O=gpurun_out/r02ze; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
cat $O/bench_default.json
timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 4 --warmup 1 > $O/bench_transe.json 2> $O/bench_transe.err
cat $O/bench_transe.json
echo done

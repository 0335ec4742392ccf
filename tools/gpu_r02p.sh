set -eo pipefail
O=gpurun_out/r02p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
cat $O/bench_default.json
timeout -k 10 900 python bench.py --workload conve-yago310-necessary --steps 3 --warmup 1 > $O/bench_conve.json 2> $O/bench_conve.err
timeout -k 10 300 python bench.py --workload complex-fb15k237-necessary --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_cxn.json 2> $O/bench_cxn.err
timeout -k 10 400 python bench.py --workload complex-db100k-sufficient --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_dbs.json 2> $O/bench_dbs.err

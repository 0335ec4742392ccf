set -o pipefail
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && tail -1 $O/smoke.txt &&
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err && cat $O/bench_default.json

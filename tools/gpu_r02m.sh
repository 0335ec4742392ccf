set -eo pipefail
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_rng_protocol.py -q > $O/rng_tests.log 2>&1 || { tail -30 $O/rng_tests.log; exit 1; }
tail -1 $O/rng_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 4 --warmup 1 > $O/bench_transe.json 2> $O/bench_transe.err
timeout -k 10 300 python tools/host_profile.py --workload transe-fb15k237-necessary > $O/host_profile_transe.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
cat $O/bench_default.json

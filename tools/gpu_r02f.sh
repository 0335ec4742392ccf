set -eo pipefail
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -50 $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err

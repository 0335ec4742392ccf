set -eo pipefail
O=gpurun_out/r02g; mkdir -p $O
bash tools/attn_micro.sh run r02g head ilv ilvburst ilv13 off
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json

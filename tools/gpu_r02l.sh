set -eo pipefail
O=gpurun_out/r02l; mkdir -p $O
bash tools/attn_micro.sh run r02l buf full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
cat $O/bench_default.json
bash tools/kstats.sh $O complex-fb15k237-sufficient 4
bash tools/attn_pmc.sh $O/pmc complex-fb15k237-sufficient

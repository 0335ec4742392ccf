set -eo pipefail
O=gpurun_out/r02za; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 4 --warmup 1 > $O/bench_transe.json 2> $O/bench_transe.err
grep "breakdown" $O/bench_transe.err
python -c "import json;d=json.load(open('$O/bench_transe.json'));print('transe', round(d['value'],1), round(d['ms_per_step'],2))"
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));print('default', round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],3))"

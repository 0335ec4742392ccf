set -eo pipefail
# closing run of the round's final tree (default environment): every GPU test, smoke, the
# default bench and its kernel summary
O=gpurun_out/r02zj; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'], d['roofline']['frac'], d['roofline']['device_kernel_ms_per_launch'])"
bash tools/kstats.sh $O complex-fb15k237-sufficient 4
echo done

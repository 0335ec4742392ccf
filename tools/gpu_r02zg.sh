set -eo pipefail
# every GPU test, smoke, the default bench; TransE with the AVX-512 twist against the portable one
O=gpurun_out/r02zg; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
grep -m1 -o "avx512f" /proc/cpuinfo || echo "no avx512f"
for m in new old new old; do
  if [ $m = old ]; then export KP_RNG_NO_AVX512=1; else unset KP_RNG_NO_AVX512; fi
  timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 4 --warmup 1 --no-cpu-baseline > $O/t_$m.json 2> $O/t_$m.err
  python -c "import json;d=json.load(open('$O/t_$m.json'));print('$m', round(d['value'],1), round(d['ms_per_step'],2))"
  grep breakdown $O/t_$m.err || true
done
unset KP_RNG_NO_AVX512
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'], d['roofline']['frac'], d['roofline']['device_kernel_ms_per_launch'])"
echo done

set -eo pipefail
# GIL switch interval of the pipeline: 5 ms (CPython default) vs 0.2 ms, TransE and default benches, alternating
O=gpurun_out/r02zc; mkdir -p $O
for sw in 0.005 0.0002 0.005 0.0002; do
  KELPIE_SWITCH_INTERVAL=$sw timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 4 --warmup 1 --no-cpu-baseline > $O/t_$sw.json 2> $O/t_$sw.err
  python -c "import json;d=json.load(open('$O/t_$sw.json'));print('transe sw $sw', round(d['value'],1), round(d['ms_per_step'],2))"
  grep breakdown $O/t_$sw.err
done
for sw in 0.005 0.0002; do
  KELPIE_SWITCH_INTERVAL=$sw timeout -k 10 300 python bench.py --no-cpu-baseline > $O/d_$sw.json 2> $O/d_$sw.err
  python -c "import json;d=json.load(open('$O/d_$sw.json'));print('default sw $sw', round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],3))"
done

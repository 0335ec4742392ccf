set -eo pipefail
# TransE bench A/B on one box: the Python package before / after the pack and view changes, alternating
O=gpurun_out/r02zb; mkdir -p $O
for v in old new old new; do
  if [ $v = old ]; then B=variants/oldpy/bench.py; else B=bench.py; fi
  timeout -k 10 300 python $B --workload transe-fb15k237-necessary --steps 4 --warmup 1 --no-cpu-baseline > $O/t_$v.json 2> $O/t_$v.err
  python -c "import json;d=json.load(open('$O/t_$v.json'));print('$v', round(d['value'],1), round(d['ms_per_step'],2))"
  grep breakdown $O/t_$v.err
done

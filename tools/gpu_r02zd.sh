set -eo pipefail
# TransE: how a batch's draws reach the library (arena view by recorded offsets / by address queries / fresh copy)
O=gpurun_out/r02zd; mkdir -p $O
for m in fast old copy fast old copy; do
  KELPIE_DRAWS_MODE=$m timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 4 --warmup 1 --no-cpu-baseline > $O/t_$m.json 2> $O/t_$m.err
  python -c "import json;d=json.load(open('$O/t_$m.json'));print('$m', round(d['value'],1), round(d['ms_per_step'],2))"
  grep breakdown $O/t_$m.err
done

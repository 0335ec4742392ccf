set -eo pipefail
# the final tree's other ComplEx workloads (necessary FB15k-237, DB100K necessary / sufficient)
O=gpurun_out/r02zn; mkdir -p $O
for w in complex-fb15k237-necessary complex-db100k-sufficient complex-db100k-necessary; do
  timeout -k 10 600 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/$w.json 2> $O/$w.err
  python -c "import json;d=json.load(open('$O/$w.json'));print('$w', round(d['value'],1), round(d['ms_per_step'],1), d.get('rank_delta_match_rate'), round(d['roofline']['frac'],3))"
done
echo done

set -eo pipefail
# pipeline depth study: batches in flight on 2 / 3 / 4 device contexts
O=gpurun_out/r02v; mkdir -p $O
for d in 2 3 4; do
  KELPIE_PIPELINE_DEPTH=$d timeout -k 10 300 python bench.py --no-cpu-baseline > $O/def_d$d.json 2> $O/def_d$d.err
  python -c "import json;d=json.load(open('$O/def_d$d.json'));print('default depth $d', round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],3))"
done
for d in 2 3; do
  KELPIE_PIPELINE_DEPTH=$d timeout -k 10 300 python bench.py --workload complex-fb15k237-necessary --steps 3 --warmup 1 --no-cpu-baseline > $O/nec_d$d.json 2> $O/nec_d$d.err
  python -c "import json;d=json.load(open('$O/nec_d$d.json'));print('necessary depth $d', round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],3))"
done

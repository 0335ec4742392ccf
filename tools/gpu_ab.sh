#!/bin/bash
# Alternating A/B of one environment switch on one bench workload (GPU box):
#   bash tools/gpu_ab.sh <tag> <workload> <VAR> <value>... [-- <steps> <reps>]
# -> gpurun_out/<tag>/ab_<VAR>_<value>_<rep>.json, one summary line per run on stdout
set -eo pipefail
tag=$1; wl=$2; var=$3; shift 3
vals=(); steps=3; reps=2
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then steps=$2; reps=$3; break; fi
  vals+=("$1"); shift
done
O=gpurun_out/$tag; mkdir -p $O
for rep in $(seq 1 $reps); do
  for v in "${vals[@]}"; do
    f=$O/ab_${var}_${v}_$rep
    env "$var=$v" timeout -k 10 600 python bench.py --workload "$wl" --steps "$steps" --warmup 1 --no-cpu-baseline \
      > $f.json 2> $f.err
    python -c "import json;d=json.load(open('$f.json'));print('$var=$v', round(d['value'],1), 'cand/s', round(d['ms_per_step'],1), 'ms/step', 'match', d.get('rank_delta_match_rate'), 'frac', d['roofline']['frac'])"
  done
done

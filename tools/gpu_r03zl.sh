#!/bin/bash
# r03zl: the default workload at 1, 2 and 4 predictions per engine batch, alternating on one box
set -o pipefail
O=gpurun_out/r03zl; mkdir -p $O
for rep in 1 2; do
for p in 1 2 4; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --preds-per-step $p > $O/p$p.json 2> $O/p$p.err || exit 1
  python - "$O/p$p.json" "$p" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
print("preds/step", sys.argv[2], "value", round(d["value"], 1), "ms/step", round(d["ms_per_step"], 2), "cand/step", d["config"]["candidates_per_step"], "frac", round(r["frac"], 4), "fp64 match", d.get("rank_delta_match_rate_ref_fp64"))
PY
done
done

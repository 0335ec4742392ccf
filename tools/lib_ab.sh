#!/bin/bash
# A/B timing of library builds under variants/ (GPU box), one batch in flight:
#   bash tools/lib_ab.sh <tag> <variant>...   (variants/lib_<v>.so)
set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
for wl in ${WLS:-complex-fb15k237-sufficient complex-fb15k237-necessary conve-yago310-necessary}; do
  for v in "$@"; do
    KELPIE_PIPELINE_DEPTH=1 KELPIE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python bench.py --workload $wl \
      --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$T/${v}_$wl.json 2> gpurun_out/$T/${v}_$wl.err || exit 1
  done
done

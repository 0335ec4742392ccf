#!/bin/bash
# Phase ablation of kp_attn3 (GPU box; timing only -- the diagnostic builds compute
# wrong results): bash tools/attn_phase_ab.sh <tag> <variant>...   (variants/lib_<v>.so)
set -eo pipefail
T=$1; shift
R=$(pwd)
mkdir -p "gpurun_out/$T"
export TMPDIR=/tmp KELPIE_PIPELINE_DEPTH=1
for v in "$@"; do
  (cd /tmp && KELPIE_HIP_LIB=$R/variants/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
     -d "$R/gpurun_out/$T/$v" -o run -- python3 "$R/bench.py" --workload complex-fb15k237-necessary --steps 1 \
     --warmup 1 --no-cpu-baseline > "$R/gpurun_out/$T/$v.log" 2>&1)
done

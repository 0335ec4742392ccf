#!/bin/bash
# Build kp_attn3 micro-benchmark variants (CPU container, no GPU needed):
#   bash tools/attn_micro.sh build <name> <src_dir> [defines...]   -> variants/attn_micro_<name>
# Run them on the GPU box (same box, same inputs, interleaved twice):
#   bash tools/attn_micro.sh run <tag> <name>...
set -eo pipefail
cmd=$1; shift
if [ "$cmd" = build ]; then
  name=$1; src=$2; shift 2
  mkdir -p variants
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -I"$src" "$@" \
    tools/attn_micro.hip -o variants/attn_micro_$name
  exit 0
fi
tag=$1; shift
O=gpurun_out/$tag; mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    # ComplEx FB15k-237 (D = 400, 3,100 queries), ComplEx DB100K, ConvE YAGO3-10 (D = 208)
    for args in "25 0 14541 3100 30" "25 0 99604 1800 10" "13 2 123182 4270 10"; do
      timeout -k 10 120 variants/attn_micro_$v $args 0.05 >> $O/$v.jsonl || exit 1
    done
  done
done

#!/bin/bash
# r04v: ComplEx contrib at 48 registers (split weights from a one-thread-per-row kp_cx_prep,
# one split at a time: two waves fit beside a resident attention wave; variants/lib_prep1.so)
# against this tree's (one wave per row doing its own fp64 transcendentals, 64 registers),
# alternating three times; same results hash expected.
set -o pipefail
O=gpurun_out/r04v; mkdir -p $O
R=$(pwd)
lib() { case $1 in prep1) echo $R/variants/lib_prep1.so ;; *) echo $R/kelpie_amd/libkelpie_hip.so ;; esac; }
for i in 1 2 3; do
  for v in cur prep1; do
    KELPIE_HIP_LIB=$(lib $v) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"value": [0-9.]*' $O/bench_${v}_$i.json) $(grep -o '"results_sha16": "[0-9a-f]*"' $O/bench_${v}_$i.json)"
  done
done
echo done

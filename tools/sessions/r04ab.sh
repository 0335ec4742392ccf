#!/bin/bash
# r04ab: the device-buffer change (grown buffers kept until teardown; no mid-run hipFree)
# against the library built just before it (variants/lib_predevbuf.so), alternating three
# times on the default line, then twice on ConvE.
set -o pipefail
O=gpurun_out/r04ab; mkdir -p $O
R=$(pwd)
lib() { case $1 in pre) echo $R/variants/lib_predevbuf.so ;; *) echo $R/kelpie_amd/libkelpie_hip.so ;; esac; }
for i in 1 2 3; do
  for v in pre cur; do
    KELPIE_HIP_LIB=$(lib $v) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"value": [0-9.]*' $O/bench_${v}_$i.json) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.json)"
  done
done
for i in 1 2; do
  for v in pre cur; do
    KELPIE_HIP_LIB=$(lib $v) timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 4 --warmup 1 \
      --no-cpu-baseline > $O/bench_conve_${v}_$i.json 2> $O/bench_conve_${v}_$i.err || exit 1
    echo "conve $v $i $(grep -o '"value": [0-9.]*' $O/bench_conve_${v}_$i.json)"
  done
done
echo done

set -eo pipefail
# ConvE bench A/B: previous FC GEMM tiles (variants/lib_fcold.so) vs wide tiles, alternating
O=gpurun_out/r02y; mkdir -p $O
for v in old new old new; do
  if [ $v = old ]; then L=$PWD/variants/lib_fcold.so; else L=$PWD/kelpie_amd/libkelpie_hip.so; fi
  KELPIE_HIP_LIB=$L timeout -k 10 900 python bench.py --workload conve-yago310-necessary --steps 3 --warmup 1 --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err
  python -c "import json;d=json.load(open('$O/b_$v.json'));print('$v', round(d['value'],1), round(d['ms_per_step'],1))"
done

set -eo pipefail
O=gpurun_out/r02s; mkdir -p $O
for v in crst crst512; do
  KELPIE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python tools/baselines_bench.py --preds 16 > $O/st_$v.log 2>&1
  grep "cr stamps" $O/st_$v.log | head -3
done

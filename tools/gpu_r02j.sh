set -eo pipefail
O=gpurun_out/r02j; mkdir -p $O
bash tools/attn_micro.sh run r02j ilv sp2 sp3 stamps sp2stamps sp3stamps

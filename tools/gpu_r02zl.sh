set -eo pipefail
# closing run of the round's final tree, then the one-stage bf16x3 FC GEMM A/B
bash tools/gpu_r02zj.sh
bash tools/gpu_r02zk.sh

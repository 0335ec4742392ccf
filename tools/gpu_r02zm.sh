set -eo pipefail
# counter passes of the final tree's default workload (FETCH_SIZE; SQ; GRBM / TCC)
O=gpurun_out/r02zm; mkdir -p $O
bash tools/attn_pmc.sh $O/pmc complex-fb15k237-sufficient
echo done

#!/bin/bash
# r03zs: the driver's N > 1 invocation rehearsed on one GPU: two ranks (gloo, both on cuda:0)
# through torch.distributed.run, default workload
set -o pipefail
O=gpurun_out/r03zs; mkdir -p $O
KELPIE_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 6 --warmup 2 > $O/n2.json 2> $O/n2.err || { tail -30 $O/n2.err; exit 1; }
cat $O/n2.json
grep -E "breakdown|parity" $O/n2.err | cut -c1-250

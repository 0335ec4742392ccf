#!/bin/bash
# r03zk = r03zi (empty-kernel dispatch probe) + r03zj (every workload's bench line)
set -o pipefail
bash tools/gpu_r03zi.sh && bash tools/gpu_r03zj.sh

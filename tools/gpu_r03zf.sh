#!/bin/bash
# r03zf = r03ze (attention O-store A/B) then r03zd (TransE arena / permutation switches)
set -o pipefail
bash tools/gpu_r03ze.sh && bash tools/gpu_r03zd.sh

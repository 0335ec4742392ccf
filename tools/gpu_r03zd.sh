#!/bin/bash
# r03zd: TransE draw workers on the box under the arena / permutation-placement switches
set -o pipefail
O=gpurun_out/r03zd; mkdir -p $O
for cfg in "KP_PINNED_ARENAS=6 KP_RNG_PERMS_INLINE=0" "KP_PINNED_ARENAS=0 KP_RNG_PERMS_INLINE=0" \
           "KP_PINNED_ARENAS=6 KP_RNG_PERMS_INLINE=1" "KP_PINNED_ARENAS=0 KP_RNG_PERMS_INLINE=1"; do
  echo "== $cfg" >> $O/host.txt
  env $cfg KP_RNG_STATS=1 timeout -k 10 200 python tools/host_profile.py --repeats 3 2>&1 | grep -E "kp_rng|batch" >> $O/host.txt || exit 1
done
cat $O/host.txt
for cfg in "KP_PINNED_ARENAS=6" "KP_PINNED_ARENAS=0"; do
  env $cfg timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 4 --warmup 1 --no-cpu-baseline > $O/transe.json 2> $O/transe.err || exit 1
  echo "$cfg $(cut -c100-190 $O/transe.json)"; grep breakdown $O/transe.err
done

#!/bin/bash
# r03z: host-side TransE draw chains on the box's CPU (tools/rng_bench.cpp) and the
# engine's scheduling breakdown (tools/host_profile.py)
set -o pipefail
O=gpurun_out/r03z; mkdir -p $O
nproc > $O/cpu.txt; grep -m1 "model name" /proc/cpuinfo >> $O/cpu.txt; taskset -pc $$ >> $O/cpu.txt 2>&1
timeout -k 10 120 variants/rng_bench 6 > $O/rng_bench.txt 2>&1 || exit 1
timeout -k 10 120 variants/rng_bench 1 p >> $O/rng_bench.txt 2>&1 || exit 1
cat $O/rng_bench.txt
timeout -k 10 300 python tools/host_profile.py --repeats 3 > $O/host_profile.txt 2>&1 || exit 1
head -8 $O/host_profile.txt

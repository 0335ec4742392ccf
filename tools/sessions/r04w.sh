#!/bin/bash
# r04w: kp_cx_update writing the next step's query rows (no kp_cx_stepq launch after step 0)
# against the separate launch (KP_CX_FUSE_Q=0), alternating three times (same results hash
# expected), then the ComplEx GPU parity tests with it.
set -o pipefail
O=gpurun_out/r04w; mkdir -p $O
for i in 1 2 3; do
  for v in 0 1; do
    KP_CX_FUSE_Q=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_fuse${v}_$i.json 2> $O/bench_fuse${v}_$i.err || exit 1
    echo "fuse=$v $i $(grep -o '"value": [0-9.]*' $O/bench_fuse${v}_$i.json) $(grep -o '"results_sha16": "[0-9a-f]*"' $O/bench_fuse${v}_$i.json)"
  done
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -v -k "complex" \
  --timeout 200 --timeout-method thread > $O/tests_complex.txt 2>&1
echo "complex tests rc=$?"; grep -E "FAILED|passed|failed" $O/tests_complex.txt | tail -3
echo done

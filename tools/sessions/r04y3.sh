#!/bin/bash
# r04y3: the whole GPU test suite on the final library (two parts) and smoke().
set -o pipefail
O=gpurun_out/r04y3; mkdir -p $O
timeout -k 10 560 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -v \
  --timeout 200 --timeout-method thread > $O/gpu_tests_parity.txt 2>&1
rc1=$?
echo "parity + fullsize rc=$rc1"; grep -E "FAILED|passed|failed" $O/gpu_tests_parity.txt | tail -5
[ $rc1 -eq 0 ] || [ $rc1 -eq 1 ] || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  --ignore=tests/test_gpu_parity.py --ignore=tests/test_fullsize_reference.py > $O/gpu_tests_rest.txt 2>&1
rc2=$?
echo "rest rc=$rc2"; grep -E "FAILED|passed|failed" $O/gpu_tests_rest.txt | tail -5
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
tail -1 $O/smoke.txt
echo done

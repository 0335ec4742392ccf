set -eo pipefail
O=gpurun_out/r02k; mkdir -p $O
bash tools/attn_micro.sh run r02k ilv buf bufsp2 bufstamps bufsp2stamps
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log

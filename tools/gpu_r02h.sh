set -eo pipefail
O=gpurun_out/r02h; mkdir -p $O
bash tools/attn_micro.sh run r02h ilv ilvbi nodma nos noo asmspread bispread
KELPIE_HIP_LIB=$PWD/variants/lib_bispread.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "conve" -v --timeout 240 --timeout-method thread > $O/bispread_tests.log 2>&1 || true
tail -5 $O/bispread_tests.log

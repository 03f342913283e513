# published-bases public encrypt on the n-adic kernel: GPU tests, then rates vs FTHE_PB_MONT=1 (Montgomery rows)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_public_exact.py tests/test_gpu_nadic.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r02zg_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/pbx_rate.py 1048576 > gpurun_out/r02zg_pbx_nadic.jsonl 2>/dev/null || exit 2
FTHE_PB_MONT=1 timeout -k 10 300 python -u tools/pbx_rate.py 1048576 > gpurun_out/r02zg_pbx_mont.jsonl 2>/dev/null || exit 3

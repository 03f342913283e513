# P-adic kernel without the end-of-product digit moves (A/B vs the paired kernel) + the library tests
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in nomove g2 nomove g2; do
  timeout -k 10 120 tools/bin/test_padic tools/bin/padic_$v.hsaco 393216 0 >> gpurun_out/r02u_nomove.jsonl 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_padic.py tests/test_gpu_direct_y.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02u_tests.txt 2>&1 || exit 2

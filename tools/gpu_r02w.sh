# exact fixed-base randomizer on the P-adic kernel: its tests, the P-adic tests, then the bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fixed_base_exact.py tests/test_gpu_padic.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02w_tests.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/r02w_bench.json 2> gpurun_out/r02w_bench.err || exit 2

# P-adic kernel for Paillier-1024 (K = 19, own slots): targeted tests, then the bench's configs[1] numbers
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_padic.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_direct_y.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02v_tests.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/r02v_bench.json 2> gpurun_out/r02v_bench.err || exit 2

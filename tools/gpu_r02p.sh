mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_padic.py tests/test_gpu_direct_y.py tests/test_gpu_parity.py tests/test_gpu_split_streams.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02p_tests.txt 2>&1 || exit 1
timeout -k 10 700 python bench.py --steps 3 --warmup 1 > gpurun_out/r02p_bench.json 2> gpurun_out/r02p_bench.err || exit 2

mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_padic.py tests/test_gpu_configs.py tests/test_gpu_fixed_base_exact.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02z_tests.txt 2>&1 || exit 1

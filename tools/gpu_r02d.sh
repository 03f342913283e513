mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_integration_shim.py tests/test_gpu_histogram_dev.py tests/test_gpu_decrypt_shared.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02d_pytest.txt 2>&1 || exit 1

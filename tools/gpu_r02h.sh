mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_add_classical.py tests/test_gpu_parity.py tests/test_gpu_histogram_dev.py tests/test_gpu_mont_rows.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02h_tests.txt 2>&1 || exit 1
FTHE_AB_FB=0 FTHE_AB_KWAY=1 timeout -k 10 200 python tools/ab_rates.py > gpurun_out/r02h_ab.jsonl 2>gpurun_out/r02h_ab.err || exit 2

# round-2 HEAD: full GPU suite, default bench, the same bench under rocprofv3 kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02k_pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 700 python bench.py --steps 3 --warmup 1 > gpurun_out/r02k_bench.json 2> gpurun_out/r02k_bench.err || exit 2

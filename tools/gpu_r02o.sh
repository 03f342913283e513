# P-adic stage B in the library: full GPU suite, then the bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02o_pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 700 python bench.py --steps 3 --warmup 1 > gpurun_out/r02o_bench.json 2> gpurun_out/r02o_bench.err || exit 2

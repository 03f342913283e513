#!/bin/bash
# GPU parity suite + default bench (no profiler).  Usage: bash tools/gpu_suite_bench.sh TAG
R=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${R}_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${R}_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/${R}_pytest_gpu.txt
timeout -k 10 400 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${R}_bench.err; exit 1; }
cat gpurun_out/${R}_bench.json

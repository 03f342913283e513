#!/bin/bash
# One GPU call: GPU parity suite, default bench, kernel-trace profile of the same bench.
# Usage (via gpurun): bash tools/gpu_round.sh TAG
R=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${R}_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${R}_pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/${R}_pytest_gpu.txt
timeout -k 10 400 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${R}_bench.err; exit 1; }
cat gpurun_out/${R}_bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_trace -o bench -- python3 bench.py > gpurun_out/${R}_bench_traced.json 2> gpurun_out/${R}_trace.log || { echo "rocprof failed"; tail -30 gpurun_out/${R}_trace.log; exit 1; }
echo done

#!/bin/bash
# Round-6 final check at HEAD: the whole GPU suite, smoke(), the driver's default bench command.
T=${1:-r06v}
set -o pipefail
mkdir -p gpurun_out
echo "[r06v] pytest -m gpu at $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest_gpu.txt 2>&1 || { echo "GPU suite failed"; tail -40 gpurun_out/${T}_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu.txt
echo "[r06v] smoke at $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
echo "[r06v] bench at $(date +%T)"
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
head -c 600 gpurun_out/${T}_bench.json; echo
echo "[r06v] done at $(date +%T)"

#!/bin/bash
# mfz add kernel, latency round: GPU add tests, then the A/B against the pre-mfz library.
T=${1:-r06x}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_addb.py > gpurun_out/${T}_test_gpu_addb.txt 2>&1 \
  || { echo "FAILED addb"; tail -30 gpurun_out/${T}_test_gpu_addb.txt; exit 1; }
tail -1 gpurun_out/${T}_test_gpu_addb.txt
bash tools/addb_lib_ab.sh $T tools/bin/libfthe_pre_mfz.so | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); r=d['res']; print(d['variant'], r['addb']['median_per_s'], r['addb_again']['median_per_s'], r['same_rows'])"

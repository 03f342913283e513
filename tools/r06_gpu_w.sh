#!/bin/bash
# Round-6 add kernel with the matrix-core product (gen_addb.py section 2M): its GPU tests, configs[3], and the
# A/B against the library built just before it.
T=${1:-r06w}
set -o pipefail
mkdir -p gpurun_out
for t in tests/test_gpu_addb.py tests/test_gpu_configs.py; do
  echo "[$T] $t at $(date +%T)"
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread $t > gpurun_out/${T}_$(basename $t .py).txt 2>&1 \
    || { echo "FAILED $t"; tail -30 gpurun_out/${T}_$(basename $t .py).txt; exit 1; }
  tail -2 gpurun_out/${T}_$(basename $t .py).txt
done
echo "[$T] A/B at $(date +%T)"
bash tools/addb_lib_ab.sh $T tools/bin/libfthe_pre_mfz.so

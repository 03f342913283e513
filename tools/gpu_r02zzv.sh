#!/bin/bash
# shared-queue linger (target = callers of the previous round) A/B + queue tests
mkdir -p gpurun_out
O=gpurun_out/r02zzv_linger_ab.jsonl
for L in 200 0; do
  FTHE_LINGER_US=$L timeout -k 10 120 python -u tools/shared_rounds.py >> $O 2>gpurun_out/r02zzv_err.txt || { echo "rounds failed"; tail gpurun_out/r02zzv_err.txt; exit 1; }
  for t in 16 64; do
    echo "{\"FTHE_LINGER_US\": $L}" >> $O
    FTHE_LINGER_US=$L timeout -k 10 120 ./tools/bin/ghpair_rate 2048 $t 512 16 >> $O || { echo "rate failed"; exit 1; }
  done
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_decrypt_shared.py tests/test_integration_shim.py > gpurun_out/r02zzv_queue_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r02zzv_queue_tests.txt; exit 1; }
tail -1 gpurun_out/r02zzv_queue_tests.txt

#!/bin/bash
# waiter spin A/B (linger on; the spin was a build-time trial, reverted) on the C++ histogram loop (integration/ghpair_rate.cpp) + the queue tests
mkdir -p gpurun_out
O=gpurun_out/r02zzs_linger_ab.jsonl
for L in 300 0; do
  for t in 1 16 64; do
    echo "{\"FTHE_SPIN_US\": $L}" >> $O
    FTHE_SPIN_US=$L timeout -k 10 120 ./tools/bin/ghpair_rate 2048 $t 512 16 >> $O || { echo "rate failed"; exit 1; }
  done
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_decrypt_shared.py tests/test_integration_shim.py > gpurun_out/r02zzs_queue_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r02zzs_queue_tests.txt; exit 1; }
tail -1 gpurun_out/r02zzs_queue_tests.txt

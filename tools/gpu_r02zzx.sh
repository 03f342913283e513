#!/bin/bash
# single-stream small host pair ops A/B (FTHE_SMALL_HOST): op latency, histogram loop, shared rounds + tests
mkdir -p gpurun_out
O=gpurun_out/r02zzx_smallhost_ab.jsonl
for S in 4096 0; do
  echo "{\"FTHE_SMALL_HOST\": $S}" >> $O
  FTHE_SMALL_HOST=$S timeout -k 10 120 python -u tools/op_latency.py >> $O 2>gpurun_out/r02zzx_err.txt || { echo "oplat failed"; tail gpurun_out/r02zzx_err.txt; exit 1; }
  FTHE_SMALL_HOST=$S timeout -k 10 120 python -u tools/shared_rounds.py >> $O 2>>gpurun_out/r02zzx_err.txt || { echo "rounds failed"; exit 1; }
  for t in 16 64; do
    FTHE_SMALL_HOST=$S timeout -k 10 120 ./tools/bin/ghpair_rate 2048 $t 512 16 >> $O || { echo "rate failed"; exit 1; }
  done
done
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_decrypt_shared.py tests/test_integration_shim.py tests/test_gpu_parity.py tests/test_gpu_add_classical.py > gpurun_out/r02zzx_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r02zzx_tests.txt; exit 1; }
tail -1 gpurun_out/r02zzx_tests.txt

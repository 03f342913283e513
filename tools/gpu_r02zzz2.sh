#!/bin/bash
# FTHE_LINGER_US sweep on the shared queues (tools/shared_rounds.py, integration/ghpair_rate.cpp)
mkdir -p gpurun_out
O=gpurun_out/r02zzz2_linger_sweep.jsonl
for L in 100 200 400 800; do
  FTHE_LINGER_US=$L timeout -k 10 120 python -u tools/shared_rounds.py >> $O 2>gpurun_out/r02zzz2_err.txt || { echo "rounds failed"; exit 1; }
  for t in 16 64; do
    echo "{\"FTHE_LINGER_US\": $L}" >> $O
    FTHE_LINGER_US=$L timeout -k 10 120 ./tools/bin/ghpair_rate 2048 $t 512 16 >> $O || { echo "rate failed"; exit 1; }
  done
done
echo done

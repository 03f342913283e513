#!/bin/bash
mkdir -p gpurun_out
rm -f gpurun_out/chunk_ab.jsonl
for i in 1 2; do
  FTHE_AB_FB=0 timeout -k 10 200 python tools/ab_rates.py --n 1572864 >> gpurun_out/chunk_ab.jsonl 2>>gpurun_out/chunk_ab.err || exit 1
  FTHE_AB_FB=0 FTHE_CHUNK=1572864 timeout -k 10 200 python tools/ab_rates.py --n 1572864 >> gpurun_out/chunk_ab.jsonl 2>>gpurun_out/chunk_ab.err || exit 1
done
cat gpurun_out/chunk_ab.jsonl

#!/bin/bash
# A/B of two builds of libfthe.so on the public-key encrypt (tools/nadic_ab.py: the n-adic kernel against the
# Montgomery s152 program in the same process), alternating twice.
#   bash tools/nadic_lib_ab.sh TAG A_SO B_SO
T=${1:?tag}; A=${2:?}; B=${3:?}
mkdir -p gpurun_out
for r in 1 2; do
  for so in $A $B; do
    FTHE_LIB=$so timeout -k 10 180 python tools/nadic_ab.py 393216 > gpurun_out/${T}_one.json || { echo "nadic_ab $so failed"; exit 1; }
    echo "{\"lib\": \"$(basename $so)\", \"run\": $r, \"res\": $(tail -1 gpurun_out/${T}_one.json)}" >> gpurun_out/${T}_nadic_lib_ab.jsonl
  done
done
cat gpurun_out/${T}_nadic_lib_ab.jsonl

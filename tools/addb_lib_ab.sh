#!/bin/bash
# A/B of two builds of libfthe.so on the P-2048 add (tools/addb_ab.py: fthe_addb_q152 against the classical
# product in the same process, so each line carries its own box normalisation), alternating 3 times.
#   bash tools/addb_lib_ab.sh TAG BASE_SO     (B = the in-tree fedtree_amd/libfthe.so)
T=${1:?tag}; A=${2:?base .so}
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export FTHE_LIB=$A; else unset FTHE_LIB; fi
    timeout -k 10 180 python tools/addb_ab.py 1048576 5 > gpurun_out/${T}_one.json || { echo "addb_ab $v failed"; exit 1; }
    echo "{\"variant\": \"$v\", \"run\": $r, \"res\": $(tail -1 gpurun_out/${T}_one.json)}" >> gpurun_out/${T}_addb_lib_ab.jsonl
  done
done
cat gpurun_out/${T}_addb_lib_ab.jsonl

#!/bin/bash
# Timing of fthe_addb_q152 knock-out builds (FTHE_GEN_ADDB_DBG, timing only, wrong results) against the in-tree
# library: one tools/addb_ab.py run per library (1M adds, the classical product in the same process).
#   bash tools/addb_dbg_ab.sh TAG LIB [LIB ...]      (libraries under tools/bin/)
T=${1:?tag}; shift
mkdir -p gpurun_out
for so in fedtree_amd/libfthe.so "$@"; do
  FTHE_LIB=$so timeout -k 10 180 python tools/addb_ab.py 1048576 5 > gpurun_out/${T}_one.json 2>/dev/null \
    || { echo "addb_ab $so failed"; exit 1; }
  echo "{\"lib\": \"$(basename $so)\", \"res\": $(tail -1 gpurun_out/${T}_one.json)}" >> gpurun_out/${T}_addb_dbg_ab.jsonl
done
cat gpurun_out/${T}_addb_dbg_ab.jsonl

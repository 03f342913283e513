#!/bin/bash
# Timing of fthe_nadic_b76 knock-out builds (FTHE_GEN_NADICB_DBG, timing only, wrong results) against the in-tree
# library: one tools/nadicb_ab.py run per library (393,216 public-key encrypts, the Montgomery form alongside).
#   bash tools/nadicb_dbg_ab.sh TAG LIB [LIB ...]      (libraries under tools/bin/)
T=${1:?tag}; shift
mkdir -p gpurun_out
for so in fedtree_amd/libfthe.so "$@"; do
  FTHE_LIB=$so timeout -k 10 180 python tools/nadicb_ab.py 393216 2 > gpurun_out/${T}_one.json 2>/dev/null \
    || { echo "nadicb_ab $so failed"; exit 1; }
  echo "{\"lib\": \"$(basename $so)\", \"res\": $(tail -1 gpurun_out/${T}_one.json)}" >> gpurun_out/${T}_nadicb_dbg_ab.jsonl
done
cat gpurun_out/${T}_nadicb_dbg_ab.jsonl

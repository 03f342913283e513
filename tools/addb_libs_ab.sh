#!/bin/bash
# A/B/... of several builds of libfthe.so on the P-2048 add (tools/addb_ab.py, 1M adds, median of 5 after a warm-up
# call in the same process), rounds alternating over the builds; "-" = the in-tree fedtree_amd/libfthe.so.
#   bash tools/addb_libs_ab.sh TAG ROUNDS SO [SO ...]
T=${1:?tag}; R=${2:?rounds}; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for so in "$@"; do
    if [ "$so" = "-" ]; then unset FTHE_LIB; name=in-tree; else export FTHE_LIB=$so; name=$(basename $so); fi
    timeout -k 10 180 python tools/addb_ab.py 1048576 5 > gpurun_out/${T}_one.json || { echo "addb_ab $so failed"; exit 1; }
    echo "{\"lib\": \"$name\", \"run\": $r, \"res\": $(tail -1 gpurun_out/${T}_one.json)}" >> gpurun_out/${T}_addb_libs_ab.jsonl
  done
done
unset FTHE_LIB
python3 - "$T" <<'PY'
import json, sys, collections
v = collections.defaultdict(list)
for l in open(f"gpurun_out/{sys.argv[1]}_addb_libs_ab.jsonl"):
    d = json.loads(l)
    v[d["lib"]].append(d["res"]["addb_again"]["median_per_s"])
for k, xs in v.items():
    print(k, sorted(xs), "median", sorted(xs)[len(xs) // 2])
PY

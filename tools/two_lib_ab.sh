#!/bin/bash
# Two builds of libfthe.so, alternating twice, on the public-key encrypt (tools/nadicb_ab.py) and the P-2048 add
# (tools/addb_ab.py): one JSON line per run.   bash tools/two_lib_ab.sh TAG BASE_SO
T=${1:?tag}; A=${2:?base .so}
mkdir -p gpurun_out
for r in 1 2; do
  for so in $A fedtree_amd/libfthe.so; do
    FTHE_LIB=$so timeout -k 10 300 python tools/nadicb_ab.py 393216 1 > gpurun_out/${T}_one.json 2>/dev/null \
      || { echo "nadicb_ab $so failed"; exit 1; }
    echo "{\"lib\": \"$(basename $so)\", \"run\": $r, \"pub\": $(tail -1 gpurun_out/${T}_one.json)}" >> gpurun_out/${T}_two_lib_ab.jsonl
    FTHE_LIB=$so timeout -k 10 180 python tools/addb_ab.py 1048576 5 > gpurun_out/${T}_one.json 2>/dev/null \
      || { echo "addb_ab $so failed"; exit 1; }
    echo "{\"lib\": \"$(basename $so)\", \"run\": $r, \"add\": $(tail -1 gpurun_out/${T}_one.json)}" >> gpurun_out/${T}_two_lib_ab.jsonl
  done
done
python3 - "$T" <<'PY'
import json, sys
for l in open(f"gpurun_out/{sys.argv[1]}_two_lib_ab.jsonl"):
    d = json.loads(l)
    if "pub" in d:
        print(d["lib"], d["run"], "pub barrett ms", d["pub"]["barrett_ms"], "mont ms", d["pub"]["mont_ms"])
    else:
        print(d["lib"], d["run"], "add ms", d["add"]["addb"]["ms"][:3], "median/s", d["add"]["addb"]["median_per_s"])
PY

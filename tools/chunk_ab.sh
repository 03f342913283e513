#!/bin/bash
# The headline encrypt at several launch sizes (FTHE_CHUNK lanes per exponentiation launch): one bench line
# each (no CPU baseline, no secondaries), appended to TAG_chunk_ab.jsonl.
#   bash tools/chunk_ab.sh TAG CHUNK [CHUNK ...]
T=${1:?tag}; shift
mkdir -p gpurun_out
for ch in "$@"; do
  FTHE_CHUNK=$ch timeout -k 10 240 python bench.py --steps 2 --warmup 1 --no-cpu --no-secondary \
    > gpurun_out/${T}_chunk_one.json 2> gpurun_out/${T}_chunk_err.txt || { echo "bench chunk $ch failed"; tail -5 gpurun_out/${T}_chunk_err.txt; exit 1; }
  echo "{\"chunk\": $ch, \"res\": $(tail -1 gpurun_out/${T}_chunk_one.json)}" >> gpurun_out/${T}_chunk_ab.jsonl
done
python3 - "$T" <<'PY'
import json, sys
for l in open(f"gpurun_out/{sys.argv[1]}_chunk_ab.jsonl"):
    d = json.loads(l)
    print(d["chunk"], d["res"]["value"], d["res"]["ms_per_step"])
PY

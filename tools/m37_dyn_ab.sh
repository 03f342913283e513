#!/bin/bash
# fthe_padic_m37 with dynamic jobs (FTHE_GEN_M37_AB=dyn, tools/bin/libfthe_m37_dyn.so, launched under
# FTHE_M37_DYN=1) against the in-tree library: parity first (the direct-y and CRT encrypt tests on the dyn
# library), then the wave timelines of both (stamp builds) and one bench line each.
#   bash tools/m37_dyn_ab.sh TAG
T=${1:?tag}
mkdir -p gpurun_out
FTHE_LIB=tools/bin/libfthe_m37_dyn.so FTHE_M37_DYN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_direct_y.py \
  tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_m37dyn_tests.txt 2>&1 \
  || { echo "dyn parity failed"; tail -20 gpurun_out/${T}_m37dyn_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_m37dyn_tests.txt
FTHE_LIB=tools/bin/libfthe_m37_stamp.so timeout -k 10 200 python tools/m37_stamps.py 1048576 > gpurun_out/${T}_m37_stamps.json \
  || { echo "static stamps failed"; exit 1; }
cat gpurun_out/${T}_m37_stamps.json
FTHE_LIB=tools/bin/libfthe_m37_dynstamp.so FTHE_M37_DYN=1 timeout -k 10 200 python tools/m37_stamps.py 1048576 \
  > gpurun_out/${T}_m37dyn_stamps.json || { echo "dyn stamps failed"; exit 1; }
cat gpurun_out/${T}_m37dyn_stamps.json
for v in base dyn base dyn; do
  if [ $v = dyn ]; then export FTHE_LIB=tools/bin/libfthe_m37_dyn.so FTHE_M37_DYN=1; else unset FTHE_LIB FTHE_M37_DYN; fi
  timeout -k 10 240 python bench.py --steps 2 --warmup 1 --no-cpu --no-secondary > gpurun_out/${T}_m37ab_one.json \
    2> gpurun_out/${T}_m37ab_err.txt || { echo "bench $v failed"; tail -5 gpurun_out/${T}_m37ab_err.txt; exit 1; }
  echo "{\"variant\": \"$v\", \"res\": $(tail -1 gpurun_out/${T}_m37ab_one.json)}" >> gpurun_out/${T}_m37_dyn_ab.jsonl
done
unset FTHE_LIB FTHE_M37_DYN
python3 - "$T" <<'PY'
import json, sys
for l in open(f"gpurun_out/{sys.argv[1]}_m37_dyn_ab.jsonl"):
    d = json.loads(l)
    print(d["variant"], d["res"]["value"], d["res"]["ms_per_step"], d["res"].get("roofline", {}).get("avg_expo_launch_ms"))
PY

#!/bin/bash
# A/B/... of fthe_padic_m37 code objects in the standalone harness (tools/bin/test_padic, checked against
# GMP on sampled lanes), round-robin over the variants three times; stops at the first failure.
#   bash tools/m37_ab.sh TAG V1 V2 [V3 ...]     (tools/bin/m37_V.hsaco; lanes: M37_LANES, default 393216)
T=${1:?tag}; shift
N=${M37_LANES:-393216}
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in "$@"; do
    # variants named pp* are ping-pong schedules (512-thread workgroups)
    blk=256; [[ $v == pp* ]] && blk=512
    M37_BLOCK=$blk timeout -k 10 120 tools/bin/test_padic tools/bin/m37_$v.hsaco $N 0 fthe_padic_m37 > gpurun_out/${T}_one.json
    rc=$?
    # timing-only variants (nomfma, noswap, nonop: wrong results by design) may report bad lanes (rc 1)
    if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [[ $v == nomfma* || $v == noswap* || $v == nonop* ]]; }; then
      echo "m37 $v failed (rc $rc)"; cat gpurun_out/${T}_one.json; exit 1
    fi
    echo "{\"variant\": \"$v\", \"run\": $r, \"res\": $(tail -1 gpurun_out/${T}_one.json)}" >> gpurun_out/${T}_m37ab.jsonl
  done
done
cat gpurun_out/${T}_m37ab.jsonl

#!/bin/bash
# A/B of two fthe_padic_m37 code objects in the standalone harness (tools/bin/test_padic, checked against
# GMP on sampled lanes), alternating A B A B A B; stops at the first failure.
#   bash tools/m37_ab.sh TAG A B [lanes]      (tools/bin/m37_A.hsaco, tools/bin/m37_B.hsaco)
T=${1:?tag}; A=${2:?}; B=${3:?}; N=${4:-393216}
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in $A $B; do
    timeout -k 10 120 tools/bin/test_padic tools/bin/m37_$v.hsaco $N 0 fthe_padic_m37 > gpurun_out/${T}_one.json \
      || { echo "m37 $v failed"; cat gpurun_out/${T}_one.json; exit 1; }
    echo "{\"variant\": \"$v\", \"run\": $r, \"res\": $(tail -1 gpurun_out/${T}_one.json)}" >> gpurun_out/${T}_m37ab.jsonl
  done
done
cat gpurun_out/${T}_m37ab.jsonl

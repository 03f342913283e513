#!/bin/bash
# fthe_padic_m37: workgroup-parity start offset (s_sleep) so the two waves of a SIMD reach their MFMA phases apart
mkdir -p gpurun_out
H=fedtree_amd/csrc/gen
run() { timeout -k 10 120 ./tools/bin/test_padic "$1" 393216 0 fthe_padic_$2 | tail -1; }
for rep in 1 2; do
  echo "{\"variant\": \"m37\", \"r\": $(run $H/padic_m37.hsaco m37)}" >> gpurun_out/r02zt_ab.jsonl || exit 1
  for n in 1 2 4; do echo "{\"variant\": \"desync$n\", \"r\": $(run tools/bin/m37_desync$n.hsaco m37)}" >> gpurun_out/r02zt_ab.jsonl; done
  echo "{\"variant\": \"k37\", \"r\": $(run $H/padic_k37.hsaco k37)}" >> gpurun_out/r02zt_ab.jsonl
done
cat gpurun_out/r02zt_ab.jsonl

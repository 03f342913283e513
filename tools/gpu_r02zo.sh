#!/bin/bash
# fthe_padic_m37 (OR pack, two-chain chunks, A-tile prefetch): raw digits, bring-up programs, exponentiation timing
mkdir -p gpurun_out
H=fedtree_amd/csrc/gen
timeout -k 10 60 ./tools/bin/test_padic $H/padic_m37.hsaco 4096 5 fthe_padic_m37 && cp gpurun_out/padic_dump.txt gpurun_out/padic_dump_m37.txt
for m in 2 3 4; do
  timeout -k 10 60 ./tools/bin/test_padic $H/padic_m37.hsaco 4096 $m fthe_padic_m37 > gpurun_out/r02zo_m37_mode$m.txt 2>&1 || { echo "mode $m failed"; tail -3 gpurun_out/r02zo_m37_mode$m.txt; exit 1; }
done
for m in 0 1; do
  timeout -k 10 120 ./tools/bin/test_padic $H/padic_m37.hsaco 393216 $m fthe_padic_m37 | tail -1 | tee -a gpurun_out/r02zo_exp.jsonl || exit 2
done
timeout -k 10 120 ./tools/bin/test_padic $H/padic_k37.hsaco 393216 0 fthe_padic_k37 | tail -1 | tee -a gpurun_out/r02zo_exp.jsonl

#!/bin/bash
# latency variants of fthe_padic_m37 (timing only)
mkdir -p gpurun_out
H=fedtree_amd/csrc/gen
run() { timeout -k 10 120 ./tools/bin/test_padic "$1" 393216 0 fthe_padic_$2 | tail -1; }
echo "{\"variant\": \"m37\", \"r\": $(run $H/padic_m37.hsaco m37)}" >> gpurun_out/r02zn_ab.jsonl || exit 1
for v in twochain orpack twochain_orpack "twochain_orpack,nomfma"; do echo "{\"variant\": \"$v\", \"r\": $(run "tools/bin/m37_$v.hsaco" m37)}" >> gpurun_out/r02zn_ab.jsonl; done
echo "{\"variant\": \"k37\", \"r\": $(run $H/padic_k37.hsaco k37)}" >> gpurun_out/r02zn_ab.jsonl
cat gpurun_out/r02zn_ab.jsonl

#!/bin/bash
# fthe_padic_m37 without the wait-state nops where the fold already separates MFMA and exchange: check + A/B
mkdir -p gpurun_out
H=fedtree_amd/csrc/gen
timeout -k 10 60 ./tools/bin/test_padic $H/padic_m37.hsaco 4096 5 fthe_padic_m37 && cp gpurun_out/padic_dump.txt gpurun_out/padic_dump_m37.txt
for m in 2 3 4; do
  timeout -k 10 60 ./tools/bin/test_padic $H/padic_m37.hsaco 4096 $m fthe_padic_m37 > gpurun_out/r02zzi_mode$m.txt 2>&1 || { echo "mode $m failed"; tail -3 gpurun_out/r02zzi_mode$m.txt; exit 1; }
done
run() { timeout -k 10 120 ./tools/bin/test_padic "$1" 393216 $3 fthe_padic_$2 | tail -1; }
for rep in 1 2 3; do
  for md in 0 1; do echo "{\"variant\": \"m37_spill\", \"r\": $(run $H/padic_m37.hsaco m37 $md)}" >> gpurun_out/r02zzi_ab.jsonl || exit 2; done
  echo "{\"variant\": \"m37_prev\", \"r\": $(run tools/bin/m37_prev.hsaco m37 0)}" >> gpurun_out/r02zzi_ab.jsonl
  echo "{\"variant\": \"k37\", \"r\": $(run $H/padic_k37.hsaco k37 0)}" >> gpurun_out/r02zzi_ab.jsonl
done
cat gpurun_out/r02zzi_ab.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_padic_mfma.py tests/test_gpu_parity.py tests/test_gpu_direct_y.py > gpurun_out/r02zzi_pytest.txt 2>&1 || { tail -20 gpurun_out/r02zzi_pytest.txt; exit 5; }; tail -1 gpurun_out/r02zzi_pytest.txt

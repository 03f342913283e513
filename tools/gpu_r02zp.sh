#!/bin/bash
# fthe_padic_m37 v2 with the rebuilt harness (tile image incl. the c column); engine P-adic tests with FTHE_PADIC_MFMA=1
mkdir -p gpurun_out
H=fedtree_amd/csrc/gen
for m in 0 1; do
  timeout -k 10 120 ./tools/bin/test_padic $H/padic_m37.hsaco 393216 $m fthe_padic_m37 | tail -1 | tee -a gpurun_out/r02zp_exp.jsonl || exit 2
  timeout -k 10 120 ./tools/bin/test_padic $H/padic_k37.hsaco 393216 $m fthe_padic_k37 | tail -1 | tee -a gpurun_out/r02zp_exp.jsonl || exit 3
done
FTHE_PADIC_MFMA=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_padic.py tests/test_gpu_direct_y.py tests/test_gpu_parity.py -k "not launches_run" > gpurun_out/r02zp_pytest_mfma.txt 2>&1 || { tail -30 gpurun_out/r02zp_pytest_mfma.txt; exit 4; }
tail -2 gpurun_out/r02zp_pytest_mfma.txt

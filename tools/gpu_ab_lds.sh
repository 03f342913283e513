#!/bin/bash
# GPU suite on the default build, then A/B of the four-lane hand-off (default vs FTHE_GEN_HANDOFF64 build)
mkdir -p gpurun_out
rm -f gpurun_out/lds_ab.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lds_pytest.txt 2>&1 || { tail -30 gpurun_out/lds_pytest.txt; exit 1; }
tail -2 gpurun_out/lds_pytest.txt
for i in 1 2; do
  FTHE_AB_FB=0 timeout -k 10 200 python tools/ab_rates.py >> gpurun_out/lds_ab.jsonl 2>>gpurun_out/lds_ab.err || exit 1
  FTHE_AB_FB=0 FTHE_LIB=build/ab/libfthe_lds64.so timeout -k 10 200 python tools/ab_rates.py >> gpurun_out/lds_ab.jsonl 2>>gpurun_out/lds_ab.err || exit 1
done
cat gpurun_out/lds_ab.jsonl

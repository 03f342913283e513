#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/direct_pytest.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/direct_pytest.txt; exit 1; }
tail -2 gpurun_out/direct_pytest.txt
for i in 1 2; do
  FTHE_AB_FB=0 timeout -k 10 200 python tools/ab_rates.py >> gpurun_out/direct_ab.jsonl 2>>gpurun_out/direct_ab.err || exit 1
  FTHE_AB_FB=0 FTHE_NO_DIRECT_Y=1 timeout -k 10 200 python tools/ab_rates.py >> gpurun_out/direct_ab.jsonl 2>>gpurun_out/direct_ab.err || exit 1
done
cat gpurun_out/direct_ab.jsonl

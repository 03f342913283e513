#!/bin/bash
# GPU suite, then A/B of the row-I/O launch size (default 4 chunks vs FTHE_ROWIO_CHUNK=393216)
mkdir -p gpurun_out
rm -f gpurun_out/rowio_ab.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rowio_pytest.txt 2>&1 || { tail -30 gpurun_out/rowio_pytest.txt; exit 1; }
tail -2 gpurun_out/rowio_pytest.txt
for i in 1 2; do
  FTHE_AB_KWAY=1 FTHE_AB_FB=0 timeout -k 10 200 python tools/ab_rates.py --n 1572864 >> gpurun_out/rowio_ab.jsonl 2>>gpurun_out/rowio_ab.err || exit 1
  FTHE_ROWIO_CHUNK=393216 FTHE_AB_KWAY=1 FTHE_AB_FB=0 timeout -k 10 200 python tools/ab_rates.py --n 1572864 >> gpurun_out/rowio_ab.jsonl 2>>gpurun_out/rowio_ab.err || exit 1
done
cat gpurun_out/rowio_ab.jsonl

#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_histogram_dev.py -x -v --timeout 200 --timeout-method thread > gpurun_out/hist_pytest.txt 2>&1 || { echo "hist pytest failed"; tail -40 gpurun_out/hist_pytest.txt; exit 1; }
tail -3 gpurun_out/hist_pytest.txt
timeout -k 10 200 python tools/hist_rate.py > gpurun_out/hist_rate.json 2> gpurun_out/hist_rate.err || { echo "rate failed"; tail -20 gpurun_out/hist_rate.err; exit 1; }
cat gpurun_out/hist_rate.json

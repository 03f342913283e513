#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fixed_base.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fb_pytest.txt 2>&1 || { echo "fb pytest failed"; tail -40 gpurun_out/fb_pytest.txt; exit 1; }
tail -2 gpurun_out/fb_pytest.txt
FTHE_FB_WINDOW=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_fixed_base.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fb8_pytest.txt 2>&1 || { echo "fb8 pytest failed"; tail -40 gpurun_out/fb8_pytest.txt; exit 1; }
tail -2 gpurun_out/fb8_pytest.txt
timeout -k 10 200 python tools/ab_rates.py > gpurun_out/fb_rates.json 2> gpurun_out/fb_rates.err || { echo "rates failed"; tail -20 gpurun_out/fb_rates.err; exit 1; }
cat gpurun_out/fb_rates.json

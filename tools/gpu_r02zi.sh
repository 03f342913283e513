#!/bin/bash
# MFMA-Barrett P-adic kernel bring-up: P-adic parity tests, then an encrypt-rate A/B against fthe_padic_k37
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_padic.py tests/test_gpu_direct_y.py > gpurun_out/r02zi_pytest_padic.txt 2>&1 || { tail -40 gpurun_out/r02zi_pytest_padic.txt; exit 1; }
tail -3 gpurun_out/r02zi_pytest_padic.txt
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --no-secondary > gpurun_out/r02zi_bench_mfma.json 2> gpurun_out/r02zi_bench_mfma.err || { tail -20 gpurun_out/r02zi_bench_mfma.err; exit 2; }
FTHE_NO_PADIC_MFMA=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --no-secondary > gpurun_out/r02zi_bench_k37.json 2> gpurun_out/r02zi_bench_k37.err || exit 3
python - <<'PY'
import json
for t in ("mfma", "k37"):
    d = json.load(open(f"gpurun_out/r02zi_bench_{t}.json"))
    print(t, d["value"], d["roofline"].get("avg_expo_launch_ms_by_kernel"))
PY

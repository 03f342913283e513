mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python tools/bench_ops.py > gpurun_out/ops.json 2> gpurun_out/ops.err && \
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err

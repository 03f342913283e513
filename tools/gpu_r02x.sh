# HEAD after the P-adic kernel: GPU suite, bench, bench under rocprof kernel trace, PMC passes
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02x_pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/r02x_bench.json 2> gpurun_out/r02x_bench.err || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02x_trace -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-secondary > gpurun_out/r02x_bench_under_rocprof.json 2> gpurun_out/r02x_rocprof.err || exit 3
bash tools/pmc_round.sh r02x || exit 4

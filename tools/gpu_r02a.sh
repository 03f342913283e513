mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_direct_y.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a_directy.txt 2>&1 || exit 1
FTHE_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --pairs 1000000 --no-cpu > gpurun_out/r02a_rehearse.json 2> gpurun_out/r02a_rehearse.err || exit 2
timeout -k 10 700 python bench.py --steps 3 --warmup 1 > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err || exit 3

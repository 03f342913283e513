mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02l_trace -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-secondary > gpurun_out/r02l_bench_under_rocprof.json 2> gpurun_out/r02l_rocprof.err || exit 3
bash tools/pmc_round.sh r02l || exit 4

# HEAD with the n-adic public encrypt: bench, bench under rocprof kernel trace, PMC passes (enc, add, kway, pub)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/r02zs_bench.json 2> gpurun_out/r02zs_bench.err || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02zs_trace -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-secondary > gpurun_out/r02zs_bench_under_rocprof.json 2> gpurun_out/r02zs_rocprof.err || exit 3
bash tools/pmc_round.sh r02zs || exit 4

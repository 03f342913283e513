#!/bin/bash
# End-of-round kernel trace at HEAD: the default bench (timed region only) under rocprofv3 --kernel-trace --stats
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r02zzz
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_trace -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-secondary > gpurun_out/${R}_bench_under_rocprof.json 2> gpurun_out/${R}_rocprof.err || { tail -20 gpurun_out/${R}_rocprof.err; exit 3; }
echo done

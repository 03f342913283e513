mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01c_ops_trace -o ops -- python3 tools/prof_ops.py --n 393216 > gpurun_out/r01c_ops.log 2>&1

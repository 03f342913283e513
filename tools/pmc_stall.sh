#!/bin/bash
# Wave-state breakdown of the montprog kernels (one counter pass per workload).
R=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
CT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_IFETCH"
timeout -s KILL 120 rocprofv3 --pmc $CT --output-format csv -d gpurun_out/${R}_stall_enc -- python3 bench.py --pairs 262144 --steps 1 --warmup 0 --no-cpu --no-secondary > gpurun_out/${R}_stall_enc.log 2>&1 || { echo enc failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $CT --output-format csv -d gpurun_out/${R}_stall_add -- python3 tools/prof_ops.py --n 1048576 --ops add > gpurun_out/${R}_stall_add.log 2>&1 || { echo add failed; exit 1; }
echo stall done

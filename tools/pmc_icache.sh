#!/bin/bash
# Instruction-fetch side of the s74 encrypt kernel: wave-state breakdown and SQC instruction
# cache hits / misses (two counter passes, no tracing).
R=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
ENC="python3 bench.py --pairs 262144 --steps 1 --warmup 0 --no-cpu --no-secondary"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_IFETCH --output-format csv -d gpurun_out/${R}_stall_enc -- $ENC > gpurun_out/${R}_stall_enc.log 2>&1 || { echo stall failed; tail -5 gpurun_out/${R}_stall_enc.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${R}_icache_enc -- $ENC > gpurun_out/${R}_icache_enc.log 2>&1 || { echo icache failed; tail -5 gpurun_out/${R}_icache_enc.log; exit 1; }
echo icache done

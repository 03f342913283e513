#!/bin/bash
# Profile the bench command on the GPU box: kernel trace (stats) of the default
# bench, then separate PMC passes (never combined with tracing) on a 2-chunk run.
# Usage (via gpurun): bash tools/profile_round.sh r01
set -e
R=${1:-r01}
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_trace -o bench -- python3 bench.py > gpurun_out/${R}_bench_traced.json 2> gpurun_out/${R}_trace.log
B="python3 bench.py --pairs 262144 --steps 1 --warmup 0 --no-cpu --no-secondary"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${R}_pmc_fetch -- $B > /dev/null 2> gpurun_out/${R}_pmc.log
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${R}_pmc_write -- $B > /dev/null 2>> gpurun_out/${R}_pmc.log
timeout -k 10 300 rocprofv3 --pmc VALUBusy --output-format csv -d gpurun_out/${R}_pmc_valubusy -- $B > /dev/null 2>> gpurun_out/${R}_pmc.log
timeout -k 10 300 rocprofv3 --pmc OccupancyPercent --output-format csv -d gpurun_out/${R}_pmc_occ -- $B > /dev/null 2>> gpurun_out/${R}_pmc.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${R}_pmc_sq -- $B > /dev/null 2>> gpurun_out/${R}_pmc.log
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH --output-format csv -d gpurun_out/${R}_pmc_ic -- $B > /dev/null 2>> gpurun_out/${R}_pmc.log
echo profile done

#!/bin/bash
# Kernel trace, then PMC passes (each its own run, no tracing) on the s80 small-batch probe.
# Usage (via gpurun): bash tools/pmc_s80.sh TAG
set -e
R=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 tools/s80_probe.py"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_s80_trace -o probe -- $B > /dev/null 2> gpurun_out/${R}_s80_pmc.log
timeout -s KILL 120 rocprofv3 --pmc VALUBusy --output-format csv -d gpurun_out/${R}_s80_pmc_valubusy -- $B > /dev/null 2>> gpurun_out/${R}_s80_pmc.log
timeout -s KILL 120 rocprofv3 --pmc OccupancyPercent --output-format csv -d gpurun_out/${R}_s80_pmc_occ -- $B > /dev/null 2>> gpurun_out/${R}_s80_pmc.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${R}_s80_pmc_sq -- $B > /dev/null 2>> gpurun_out/${R}_s80_pmc.log
echo pmc done

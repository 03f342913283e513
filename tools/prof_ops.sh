#!/bin/bash
# Kernel trace + separate counter passes of tools/prof_ops.py (via gpurun).
set -e
R=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_ops_trace -o ops -- python3 tools/prof_ops.py > gpurun_out/${R}_ops.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${R}_ops_pmc_sq -- python3 tools/prof_ops.py --ops add > /dev/null 2>> gpurun_out/${R}_ops.log
timeout -k 10 300 rocprofv3 --pmc VALUBusy --output-format csv -d gpurun_out/${R}_ops_pmc_vb -- python3 tools/prof_ops.py --ops add > /dev/null 2>> gpurun_out/${R}_ops.log
timeout -k 10 300 rocprofv3 --pmc OccupancyPercent --output-format csv -d gpurun_out/${R}_ops_pmc_occ -- python3 tools/prof_ops.py --ops add > /dev/null 2>> gpurun_out/${R}_ops.log
echo ops profile done

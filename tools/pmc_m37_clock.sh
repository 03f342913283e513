#!/bin/bash
# PMC (GRBM / SQ cycles, VALU instructions) with the kernel trace on three m37 code objects in the standalone
# harness: the clock and the cycles of the default schedule, of the timing-only variant without MFMAs and of prio3.
set -e
export TMPDIR=/tmp
for v in base nomfma prio3; do
  M37_BLOCK=256 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-trace --stats --output-format csv -d gpurun_out/r03x_clk_$v -- tools/bin/test_padic tools/bin/m37_$v.hsaco 393216 0 fthe_padic_m37 > gpurun_out/r03x_clk_$v.log 2>&1 || [ $v = nomfma ]
done
echo done

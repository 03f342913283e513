#!/bin/bash
# PMC of the add kernel's matrix-core product variant (mfz) on the pmc:add workload, beside the default kernel's.
export FTHE_LIB=tools/bin/libfthe_mfz.so
bash tools/gpu.sh r06z_mfz pmc:add || exit 1
unset FTHE_LIB
bash tools/gpu.sh r06z_def pmc:add

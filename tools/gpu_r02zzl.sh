#!/bin/bash
# instruction-cache counters of the two P-adic kernels on the standalone harness (one PMC pass each)
mkdir -p gpurun_out
export TMPDIR=/tmp
H=fedtree_amd/csrc/gen
for v in m37 k37; do
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d gpurun_out/r02zzl_ic_$v -- ./tools/bin/test_padic $H/padic_$v.hsaco 393216 0 fthe_padic_$v > gpurun_out/r02zzl_ic_$v.log 2>&1 || { echo "pass $v failed"; tail -5 gpurun_out/r02zzl_ic_$v.log; exit 1; }
done
echo done

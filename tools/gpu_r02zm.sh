#!/bin/bash
# fthe_padic_m37 vs fthe_padic_k37: timing-only variants, then PMC passes on the standalone harness
mkdir -p gpurun_out
export TMPDIR=/tmp
H=fedtree_amd/csrc/gen
run() { timeout -k 10 120 ./tools/bin/test_padic $1 393216 0 $2 | tail -1; }
for v in m37 k37; do echo "{\"variant\": \"$v\", \"r\": $(run $H/padic_$v.hsaco fthe_padic_$v)}" >> gpurun_out/r02zm_ab.jsonl || exit 1; done
for v in noswap nonop nomfma noswap_nonop; do echo "{\"variant\": \"$v\", \"r\": $(run tools/bin/m37_$v.hsaco fthe_padic_m37)}" >> gpurun_out/r02zm_ab.jsonl; done
cat gpurun_out/r02zm_ab.jsonl
for v in m37 k37; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d gpurun_out/r02zm_pmc_${v}_a -- ./tools/bin/test_padic $H/padic_$v.hsaco 393216 0 fthe_padic_$v > gpurun_out/r02zm_pmc_${v}_a.log 2>&1 || { echo "pmc a $v failed"; tail -5 gpurun_out/r02zm_pmc_${v}_a.log; }
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/r02zm_pmc_${v}_b -- ./tools/bin/test_padic $H/padic_$v.hsaco 393216 0 fthe_padic_$v > gpurun_out/r02zm_pmc_${v}_b.log 2>&1 || { echo "pmc b $v failed"; tail -5 gpurun_out/r02zm_pmc_${v}_b.log; }
done
exit 0

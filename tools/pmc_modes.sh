#!/bin/bash
# Counters of the four-lane kernel in the opt-in modes: Montgomery-resident add and the party
# encrypt from published bases (gathered 4096-bit products).  One counter group per run.
R=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in mont pbx; do
  C="python3 tools/prof_ops.py --n 786432 --ops $w"
  for t in "vb VALUBusy" "fetch FETCH_SIZE" "write WRITE_SIZE"; do
    set -- $t
    timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/${R}_pmc_${w}_$1 -- $C > gpurun_out/${R}_pmc_${w}_$1.log 2>&1 || { echo "pass $w $1 failed"; tail -5 gpurun_out/${R}_pmc_${w}_$1.log; exit 1; }
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_modes_trace -o modes -- python3 tools/prof_ops.py --n 786432 --ops mont,pbx > gpurun_out/${R}_modes_trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo modes done

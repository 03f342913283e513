#!/bin/bash
# Separate PMC passes (never combined with tracing; one counter group per run) on
#   enc : the bench's encrypt at 262,144 pairs (montprog s37 / s74, modexp)
#   add : one device-resident P-2048 add of 1M ciphertexts (montprog s152, row I/O)
#   kway: one 8-party merge of 262,144 bins (montprog s152, row I/O)
#   pub : public-key encrypt of 131,072 ciphertexts on the n-adic kernel, then on the Montgomery s152
#         program (tools/nadic_ab.py)
# Usage (via gpurun): bash tools/pmc_round.sh TAG
R=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
ENC="python3 bench.py --pairs 262144 --steps 1 --warmup 0 --no-cpu --no-secondary"
ADD="python3 tools/prof_ops.py --n 1048576 --ops add"
KWAY="python3 tools/prof_ops.py --n 262144 --ops kway"
PUB="python3 tools/nadic_ab.py 131072"
pass() {  # tag counters... -- cmd
  local tag=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done; shift
  timeout -s KILL 120 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d gpurun_out/${R}_pmc_${tag} -- "$@" > gpurun_out/${R}_pmc_${tag}.log 2>&1 || { echo "pass $tag failed"; tail -5 gpurun_out/${R}_pmc_${tag}.log; exit 1; }
}
for w in enc add kway pub; do
  case $w in enc) C=$ENC;; add) C=$ADD;; kway) C=$KWAY;; pub) C=$PUB;; esac
  pass ${w}_fetch FETCH_SIZE -- $C
  pass ${w}_write WRITE_SIZE -- $C
  pass ${w}_vb VALUBusy -- $C
  pass ${w}_occ OccupancyPercent -- $C
  pass ${w}_sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -- $C
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_ops_trace -o ops -- python3 tools/prof_ops.py --n 1048576 --ops add,kway > gpurun_out/${R}_ops_trace.log 2>&1 || { echo "ops trace failed"; exit 1; }
echo pmc done

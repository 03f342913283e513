#!/bin/bash
# Final HEAD validation: GPU suite, default bench, smoke, bench under rocprof kernel trace, PMC of the encrypt
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r02zzc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.txt 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_trace -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-secondary > gpurun_out/${R}_bench_under_rocprof.json 2> gpurun_out/${R}_rocprof.err || exit 3
ENC="python3 bench.py --pairs 262144 --steps 1 --warmup 0 --no-cpu --no-secondary"
pass() {
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${R}_pmc_enc_${tag} -- $ENC > gpurun_out/${R}_pmc_enc_${tag}.log 2>&1 || { echo "pass $tag failed"; tail -5 gpurun_out/${R}_pmc_enc_${tag}.log; exit 4; }
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass vb VALUBusy
pass occ OccupancyPercent
pass sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
pass mf SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
echo done

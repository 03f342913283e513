#!/bin/bash
# The one GPU lease script: run the named steps in order on the gpurun box, stop at the first failure.
#   bash tools/gpu.sh TAG STEP [STEP ...]
# Steps (outputs under gpurun_out/, prefixed with TAG):
#   suite          python -m pytest tests -m gpu (thread timeouts: a hang names its test)
#   test:FILE      python -m pytest FILE -m gpu (one test file, same timeouts)
#   smoke          __graft_entry__.smoke()
#   bench          python bench.py (the driver's default line)              -> TAG_bench.json
#   bench:ARGS     python bench.py ARGS (comma-separated, e.g. bench:--steps,3)
#   trace          the bench's timed region under rocprofv3 --kernel-trace --stats
#   pmc:W          separate PMC passes (one counter group per run, never with tracing) over workload W:
#                    enc  the bench's encrypt at 393,216 pairs: one full 786,432-lane launch per prime (fthe_padic_m37 + s74 tails)
#                    add  one device-resident P-2048 add of 1M distinct ciphertext pairs (fthe_addb_q152)
#                    addsame  the same with x = y (each row read once for both operands: counter calibration)
#                    kway three 8-party merges of 1,048,576 bins
#                    pub  public-key encrypt of 196,608 ciphertexts on fthe_nadic_b76 and fthe_nadic_m76
#                         (tools/nadicb_ab.py; the PMC summary separates the kernels by name)
#                  then: python tools/rocprof_summary.py pmc gpurun_out/TAG_pmc_W_* out.json (CPU side)
#   opstrace       kernel trace of tools/prof_ops.py add,kway (the add / merge launch durations for pmc:add)
#   rehearse       FTHE_BENCH_REHEARSE=1 bench.py --gpus 2 (two ranks on the one GPU over gloo; ghpair_e2e_node
#                  over two contexts, NODE_PAIRS pairs per device, default 2M)
#   ghpair         tools/bin/ghpair_rate twice at 16 threads (7 interleaved rounds each), tools/bin/ghpair_e2e
#   marshal        tools/bin/marshal_rate: host mpz <-> row marshalling of 1, 2, 4, 8 concurrent shards (no kernels)
#   ghsub          the operator- A/B: tools/bin/ghpair_rate at 16 threads, host powm vs FTHE_SHIM_MUL_ENGINE=1
#   py:SCRIPT[,ARGS]  python SCRIPT ARGS (a tools/ measurement), appended to TAG_SCRIPT.jsonl
R=${1:?tag}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${R}
fail() { echo "step $1 failed (rc $2)"; tail -30 "$3" 2>/dev/null; exit 1; }
pmc_pass() {  # workload tag counters...
  local w=$1 tag=$2; shift 2
  local cmd
  case $w in
    enc)  cmd="python3 bench.py --pairs 393216 --steps 1 --warmup 0 --no-cpu --no-secondary";;
    add)  cmd="python3 tools/prof_ops.py --n 1048576 --ops add";;
    addsame) cmd="python3 tools/prof_ops.py --n 1048576 --ops addsame";;
    kway) cmd="python3 tools/prof_ops.py --n 1048576 --ops kway";;
    pub)  cmd="python3 tools/nadicb_ab.py 196608 1";;
    *) echo "unknown pmc workload $w"; exit 2;;
  esac
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d ${O}_pmc_${w}_${tag} -- $cmd \
    > ${O}_pmc_${w}_${tag}.log 2>&1 || fail "pmc:$w:$tag" $? ${O}_pmc_${w}_${tag}.log
}
for step in "$@"; do
  echo "[gpu.sh] $step at $(date +%T)"
  case $step in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > ${O}_pytest_gpu.txt 2>&1 || fail suite $? ${O}_pytest_gpu.txt
      tail -3 ${O}_pytest_gpu.txt;;
    test:*)
      f=${step#test:}
      timeout -k 10 600 python -u -m pytest $f -m gpu -x -v --timeout 300 --timeout-method thread \
        > ${O}_$(basename $f .py).txt 2>&1 || fail "$step" $? ${O}_$(basename $f .py).txt
      tail -3 ${O}_$(basename $f .py).txt;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.txt 2>&1 \
        || fail smoke $? ${O}_smoke.txt
      cat ${O}_smoke.txt;;
    bench)
      timeout -k 10 900 python bench.py > ${O}_bench.json 2> ${O}_bench.err || fail bench $? ${O}_bench.err
      cut -c1-600 ${O}_bench.json;;
    bench:*)
      args=${step#bench:}
      timeout -k 10 900 python bench.py ${args//,/ } > ${O}_bench_args.json 2> ${O}_bench_args.err \
        || fail "$step" $? ${O}_bench_args.err
      cut -c1-600 ${O}_bench_args.json;;
    trace)
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_trace -o bench -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu --no-secondary > ${O}_bench_under_rocprof.json \
        2> ${O}_rocprof.err || fail trace $? ${O}_rocprof.err;;
    pmc:*)
      w=${step#pmc:}
      pmc_pass $w fetch FETCH_SIZE
      pmc_pass $w write WRITE_SIZE
      pmc_pass $w vb VALUBusy
      pmc_pass $w occ OccupancyPercent
      pmc_pass $w sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
      pmc_pass $w mf SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
      pmc_pass $w lds SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU;;
    opstrace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_ops_trace -o ops -- \
        python3 tools/prof_ops.py --n 1048576 --ops add,kway > ${O}_ops_trace.log 2>&1 || fail opstrace $? ${O}_ops_trace.log;;
    rehearse)
      FTHE_BENCH_REHEARSE=1 FTHE_BENCH_NODE_PAIRS=${NODE_PAIRS:-2000000} timeout -k 10 600 python bench.py --gpus 2 \
        --pairs 1048576 --steps 2 --warmup 1 \
        > ${O}_rehearse_2rank_1gpu.json 2> ${O}_rehearse.err || fail rehearse $? ${O}_rehearse.err
      cut -c1-600 ${O}_rehearse_2rank_1gpu.json;;
    ghpair)
      for t in 16 16; do
        timeout -k 10 300 tools/bin/ghpair_rate 2048 $t 8192 16 4096 7 >> ${O}_ghpair_rate.jsonl 2>> ${O}_ghpair.err \
          || fail ghpair_rate $? ${O}_ghpair.err
      done
      timeout -k 10 300 tools/bin/ghpair_e2e 2048 2000000 2 >> ${O}_ghpair_e2e.jsonl 2>> ${O}_ghpair.err \
        || fail ghpair_e2e $? ${O}_ghpair.err
      cat ${O}_ghpair_rate.jsonl ${O}_ghpair_e2e.jsonl;;
    marshal)
      timeout -k 10 300 tools/bin/marshal_rate 2048 1048576 3 1,2,4,8 >> ${O}_marshal.jsonl 2>> ${O}_marshal.err \
        || fail marshal $? ${O}_marshal.err
      cat ${O}_marshal.jsonl;;
    ghsub)
      for v in 0 1 0 1; do
        FTHE_SHIM_MUL_ENGINE=$v timeout -k 10 300 tools/bin/ghpair_rate 2048 16 8192 16 4096 > ${O}_one.json 2>> ${O}_ghsub.err \
          || fail ghsub $? ${O}_ghsub.err
        echo "{\"mul_engine\": $v, \"res\": $(tail -1 ${O}_one.json)}" >> ${O}_ghsub_ab.jsonl
      done
      cat ${O}_ghsub_ab.jsonl;;
    py:*)
      spec=${step#py:}
      script=${spec%%,*}
      args=""
      [ "$script" != "$spec" ] && args=${spec#*,}
      name=$(basename $script .py)
      timeout -k 10 600 python $script ${args//,/ } >> ${O}_${name}.jsonl 2>> ${O}_${name}.err \
        || fail "$step" $? ${O}_${name}.err
      tail -5 ${O}_${name}.jsonl;;
    *) echo "unknown step $step"; exit 2;;
  esac
done
echo "[gpu.sh] done at $(date +%T)"

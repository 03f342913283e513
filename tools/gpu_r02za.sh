# n-adic public encrypt at HEAD: full GPU suite, then the pub PMC passes and a kernel trace of the A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02za_pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02za_pub_trace -o pub -- python3 tools/nadic_ab.py 393216 > gpurun_out/r02za_pub_trace.log 2>&1 || exit 2
for c in "FETCH_SIZE" "WRITE_SIZE" "VALUBusy" "OccupancyPercent" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  t=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r02za_pmc_pub_$t -- python3 tools/nadic_ab.py 131072 > gpurun_out/r02za_pmc_pub_$t.log 2>&1 || exit 3
done
echo done

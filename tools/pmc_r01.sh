export TMPDIR=/tmp
B="python3 bench.py --pairs 262144 --steps 1 --warmup 0 --no-cpu --no-secondary"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -- $B > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -- $B > gpurun_out/pmc_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc VALUBusy --output-format csv -d gpurun_out/pmc_valubusy -- $B > gpurun_out/pmc_vb.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc OccupancyPercent --output-format csv -d gpurun_out/pmc_occ -- $B > gpurun_out/pmc_occ.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -- $B > gpurun_out/pmc_sq.log 2>&1

mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_add_classical.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02e_add.txt 2>&1 || exit 1
FTHE_AB_FB=0 FTHE_AB_KWAY=1 timeout -k 10 200 python tools/ab_rates.py > gpurun_out/r02e_ab.jsonl 2>gpurun_out/r02e_ab.err || exit 2
FTHE_ADD_MONT=1 FTHE_AB_FB=0 timeout -k 10 200 python tools/ab_rates.py >> gpurun_out/r02e_ab.jsonl 2>>gpurun_out/r02e_ab.err || exit 3

mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python tools/ab_rates.py >> gpurun_out/ab.jsonl 2>>gpurun_out/ab.err || exit 1
  FTHE_LIB=build/ab/libfthe_noring.so timeout -k 10 200 python tools/ab_rates.py >> gpurun_out/ab.jsonl 2>>gpurun_out/ab.err || exit 1
done

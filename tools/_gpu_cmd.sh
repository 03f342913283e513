mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python tools/ab_rates.py >> gpurun_out/ab.jsonl 2>>gpurun_out/ab.err || exit 1
  FTHE_LIB=build/ab/libfthe_qlo.so timeout -k 10 200 python tools/ab_rates.py >> gpurun_out/ab.jsonl 2>>gpurun_out/ab.err || exit 1
done

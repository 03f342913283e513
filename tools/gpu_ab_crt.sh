#!/bin/bash
# A/B of the CRT glue (register mul_add_out, CRT tail in the p program, per-word digits):
# default build vs build/ab/libfthe_prev.so, encrypt rates of every CRT mode, twice each.
mkdir -p gpurun_out
rm -f gpurun_out/crt_ab.jsonl
for i in 1 2; do
  timeout -k 10 200 python tools/fbx_rate.py 1572864 >> gpurun_out/crt_ab.jsonl 2>>gpurun_out/crt_ab.err || exit 1
  FTHE_LIB=build/ab/libfthe_prev.so timeout -k 10 200 python tools/fbx_rate.py 1572864 >> gpurun_out/crt_ab.jsonl 2>>gpurun_out/crt_ab.err || exit 1
done
cat gpurun_out/crt_ab.jsonl

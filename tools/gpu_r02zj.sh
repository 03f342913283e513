#!/bin/bash
# fthe_padic_m37 bring-up: one Barrett (LOADP; STOREP), a squaring, a product, then the exponentiations
mkdir -p gpurun_out
H=fedtree_amd/csrc/gen
for m in 2 3 4 0 1; do
  timeout -k 10 60 ./tools/bin/test_padic $H/padic_m37.hsaco 4096 $m fthe_padic_m37 >> gpurun_out/r02zj_m37.txt 2>&1
  echo "mode $m rc $?" >> gpurun_out/r02zj_m37.txt
done
timeout -k 10 60 ./tools/bin/test_padic $H/padic_k37.hsaco 4096 2 fthe_padic_k37 >> gpurun_out/r02zj_m37.txt 2>&1
cat gpurun_out/r02zj_m37.txt

#!/bin/bash
# timing-only variants of fthe_padic_m37 for the standalone harness (tools/bin/m37_<variant>.hsaco)
set -e
L=/opt/rocm/lib/llvm/bin
for v in ${M37_AB:-noswap nonop nomfma noswap,nonop}; do
  n=${v//,/_}; n=${n/pingpong/pp}
  FTHE_GEN_M37_AB=$v python3 fedtree_amd/csrc/gen_padic_mfma.py -o /tmp/m37_$n.s
  $L/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=gfx950 -c /tmp/m37_$n.s -o /tmp/m37_$n.o
  $L/ld.lld -shared /tmp/m37_$n.o -o tools/bin/m37_$n.hsaco
done

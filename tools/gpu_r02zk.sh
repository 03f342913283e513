#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 60 ./tools/bin/test_padic fedtree_amd/csrc/gen/padic_m37.hsaco 4096 5 fthe_padic_m37 && cp gpurun_out/padic_dump.txt gpurun_out/padic_dump_m37.txt
timeout -k 10 60 ./tools/bin/test_padic fedtree_amd/csrc/gen/padic_k37.hsaco 4096 5 fthe_padic_k37 && cp gpurun_out/padic_dump.txt gpurun_out/padic_dump_k37.txt

# P-adic kernel A/B: accumulator chains per column (2, 3, 4), standalone harness, full chunk
mkdir -p gpurun_out
for n in 2 3 4 2; do
  timeout -k 10 120 tools/bin/test_padic tools/bin/padic_c$n.hsaco 393216 0 >> gpurun_out/r02q_chains.jsonl 2>&1 || exit 1
done

# P-adic kernel A/B: column pairing vs two chains per column, standalone harness, full chunk
mkdir -p gpurun_out
for v in pair nopair pair nopair; do
  timeout -k 10 120 tools/bin/test_padic tools/bin/padic_$v.hsaco 393216 0 >> gpurun_out/r02r_pair.jsonl 2>&1 || exit 1
done

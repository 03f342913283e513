# P-adic kernel A/B: columns accumulated side by side (2, 3, 4), standalone harness, full chunk
mkdir -p gpurun_out
for g in 2 3 4 2 3 4; do
  timeout -k 10 120 tools/bin/test_padic tools/bin/padic_g$g.hsaco 393216 0 >> gpurun_out/r02t_group.jsonl 2>&1 || exit 1
done

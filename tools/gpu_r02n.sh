# P-adic exponentiation kernel bring-up: bit-exact vs GMP on sampled lanes + timing (standalone harness)
mkdir -p gpurun_out
timeout -k 10 120 tools/bin/test_padic tools/bin/padic_k37.hsaco 65536 0 > gpurun_out/r02n_padic.jsonl 2>&1 || exit 1
timeout -k 10 120 tools/bin/test_padic tools/bin/padic_k37.hsaco 393216 0 >> gpurun_out/r02n_padic.jsonl 2>&1 || exit 2
timeout -k 10 120 tools/bin/test_padic tools/bin/padic_k37.hsaco 393216 1 >> gpurun_out/r02n_padic.jsonl 2>&1 || exit 3

#!/bin/bash
# A/B of FTHE_ENC_PIPE (large device-resident CRT encrypts: chunks pipelined over two slot-region pairs, the p half
# of chunk i + 1 beside the q half of chunk i) against the chunk-by-chunk split: the bench's timed encrypt (10M
# pairs, no secondary), alternating arms.  Output: gpurun_out/TAG_pipe_ab.jsonl, one line per run.
#   bash tools/enc_pipe_ab.sh TAG [rounds]
T=${1:?tag}; R=${2:-2}
mkdir -p gpurun_out
O=gpurun_out/${T}_pipe_ab.jsonl
for r in $(seq 1 $R); do
  for v in 0 1; do
    FTHE_ENC_PIPE=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-secondary \
      > gpurun_out/${T}_pipe_b.json 2> gpurun_out/${T}_pipe_b.err || { echo "bench failed ($v)"; tail -5 gpurun_out/${T}_pipe_b.err; exit 1; }
    python3 - "$v" "$r" gpurun_out/${T}_pipe_b.json >> $O <<'PY'
import json, sys
v, r, b = sys.argv[1:4]
bl = json.loads(open(b).read().strip().splitlines()[-1])
ro = bl["roofline"]
print(json.dumps({"enc_pipe": int(v), "round": int(r), "encrypts_per_s": bl["value"], "ms_per_step": bl["ms_per_step"],
                  "avg_expo_launch_ms": ro.get("avg_expo_launch_ms"),
                  "avg_expo_launch_ms_in_flight": ro.get("avg_expo_launch_ms_in_flight"), "frac": ro.get("frac")}))
PY
    tail -1 $O
  done
done

#!/bin/bash
# A/B of FTHE_SPLIT_ALL (both CRT halves of every chunk of a large encrypt / decrypt on two streams) against the
# default (the halves in turn on one stream): the bench's timed encrypt (10M pairs, no secondary) and
# tools/dec_rate.py, alternating arms.  Output: gpurun_out/TAG_split_ab.jsonl, one line per run.
#   bash tools/split_all_ab.sh TAG [rounds]
T=${1:?tag}; R=${2:-2}
mkdir -p gpurun_out
O=gpurun_out/${T}_split_ab.jsonl
for r in $(seq 1 $R); do
  for v in 0 1; do
    FTHE_SPLIT_ALL=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-secondary \
      > gpurun_out/${T}_split_b.json 2> gpurun_out/${T}_split_b.err || { echo "bench failed ($v)"; tail -5 gpurun_out/${T}_split_b.err; exit 1; }
    FTHE_SPLIT_ALL=$v timeout -k 10 120 python tools/dec_rate.py 3145728 > gpurun_out/${T}_split_d.json \
      2> gpurun_out/${T}_split_d.err || { echo "dec_rate failed ($v)"; tail -5 gpurun_out/${T}_split_d.err; exit 1; }
    python3 - "$v" "$r" gpurun_out/${T}_split_b.json gpurun_out/${T}_split_d.json >> $O <<'PY'
import json, sys
v, r, b, d = sys.argv[1:5]
bl = json.loads(open(b).read().strip().splitlines()[-1]); dl = json.loads(open(d).read().strip().splitlines()[-1])
print(json.dumps({"split_all": int(v), "round": int(r), "encrypts_per_s": bl["value"], "ms_per_step": bl["ms_per_step"],
                  "avg_expo_launch_ms": bl["roofline"].get("avg_expo_launch_ms"), "decrypt_per_s": dl["decrypt_per_s"],
                  "decrypt_ok": dl["decrypt_ok"]}))
PY
    tail -1 $O
  done
done

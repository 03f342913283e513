#!/bin/bash
# The parties' public-key encrypt (fthe_nadic_b76) at several launch sizes (FTHE_PUB_CHUNK, lanes per launch: four per
# ciphertext): 1,572,864 ciphertexts device-resident, best of 2, alternating twice.  gpurun_out/TAG_pub_chunk_ab.jsonl
#   bash tools/pub_chunk_ab.sh TAG CHUNK [CHUNK ...]
T=${1:?tag}; shift
mkdir -p gpurun_out
for r in 1 2; do
  for ch in "$@"; do
    FTHE_PUB_CHUNK=$ch timeout -k 10 300 python tools/nadicb_ab.py 1572864 2 > gpurun_out/${T}_one.json 2>/dev/null \
      || { echo "nadicb_ab $ch failed"; exit 1; }
    echo "{\"pub_chunk\": $ch, \"run\": $r, \"res\": $(tail -1 gpurun_out/${T}_one.json)}" >> gpurun_out/${T}_pub_chunk_ab.jsonl
    tail -1 gpurun_out/${T}_pub_chunk_ab.jsonl | cut -c1-200
  done
done

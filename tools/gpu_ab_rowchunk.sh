# A/B: row-I/O launch size (FTHE_ROWIO_CHUNK lanes) for the 1M-add call of the bench
mkdir -p gpurun_out
export FTHE_AB_FB=0
for v in 1572864 4194304 8388608 2097152; do
  FTHE_ROWIO_CHUNK=$v timeout -k 10 120 python -u tools/ab_rates.py --n 1048576 --reps 5 | sed "s/^/{\"rowio_chunk\": $v, \"r\": /; s/\$/}/" >> gpurun_out/r02zc_ab_rowchunk.jsonl || exit 1
done

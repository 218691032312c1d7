#!/bin/bash
# Resident row-table A/B after the round-3 sort changes: rows 4 vs 8 at 2^20
# and 2^21, 2 vs 4 at 2^22, interleaved, then the default bench with 8 rows.
# Usage (through gpurun): bash tools/gpu_rows_ab.sh
set -o pipefail
OUT=gpurun_out/rows_ab
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for cfg in 20:4 20:8 21:4 21:8 22:2 22:4; do
    lg=${cfg%%:*}; rows=${cfg##*:}
    PM_RESIDENT_ROWS=$rows RESIDENT=1 LOGN=$lg REPS=40 timeout -k 10 120 python tools/msm_timing.py > $OUT/r${rep}_${lg}_${rows}.jsonl 2>&1 || { echo "$cfg failed"; tail -20 $OUT/r${rep}_${lg}_${rows}.jsonl; exit 1; }
    echo "$rep $cfg $(grep -o '"wall_ms": [0-9.]*' $OUT/r${rep}_${lg}_${rows}.jsonl)"
  done
done
for rows in 4 8; do
  PM_RESIDENT_ROWS=$rows timeout -k 10 300 python bench.py > $OUT/bench_rows$rows.json 2> $OUT/bench_rows$rows.err || { echo "bench failed"; tail -20 $OUT/bench_rows$rows.err; exit 1; }
  echo "bench rows $rows $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_rows$rows.json | head -1)"
done

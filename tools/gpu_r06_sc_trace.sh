#!/bin/bash
# Round 6: kernel + memory-copy trace of the split scalar copy (2^20, resident
# row table, host scalars): one round of tools/split_copy_ab.py.
set -o pipefail
OUT=gpurun_out/${TAG:-r06_sc_trace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
LOGN=20 ROUNDS=1 REPS=5 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d $OUT/prof -o trace -- python3 tools/split_copy_ab.py > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
find $OUT/prof -name "*.csv" | head

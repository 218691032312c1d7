#!/bin/bash
# Round 6: lanes per term of k_acc_termadd (pm_ctx_set_accum_split) at
# mid batches, interleaved: auto (8 lanes from B ~ 64), 16, 32 lanes.
set -o pipefail
OUT=gpurun_out/${TAG:-r06_split}
mkdir -p $OUT
for rep in 1 2; do
  for sp in auto 4 5; do
    if [ $sp = auto ]; then S=""; else S=$sp; fi
    SPLIT=$S BS=${BS:-64,128,192,256,384,512,768} REPS=20 timeout -k 10 150 python -u tools/accum_scaling.py >> $OUT/split.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  done
done
python3 -c "
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); k = d['kernels_ms']
    print(d['B'], d['split'], d['ms_per_batch'], k['acc_termmul'], k['acc_ladder'], k['acc_sum'])
" $OUT/split.jsonl

#!/bin/bash
# Round 6: the auto decode-fence rule across B, twice, plus the parity tests of the options.
set -o pipefail
OUT=gpurun_out/r06_d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_proof_gpu.py tests/test_accum_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  BS=16,32,64,128,192,256,384,512,768,1024,1536,2048,3072,4096 REPS=20 timeout -k 10 300 python -u tools/accum_scaling.py >> $OUT/sweep.jsonl 2>> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
done

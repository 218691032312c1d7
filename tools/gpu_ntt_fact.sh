#!/bin/bash
# A/B of the three-pass NTT factorisation (PM_NTT_LOG1) and block width
# (PM_NTT_MAXLOGC), one call.  Usage (through gpurun): bash tools/gpu_ntt_fact.sh TAG
set -o pipefail
TAG=${1:-ntt_fact}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PM_NTT_LOG1=7 PM_NTT_MAXLOGC=4 timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_knobs.log 2>&1 || { tail -20 $OUT/pytest_knobs.log; exit 1; }
tail -1 $OUT/pytest_knobs.log
for rep in 1 2; do
  for cfg in "0 2" "7 4" "7 2" "8 3" "6 4" "0 4"; do
    set -- $cfg
    PM_NTT_LOG1=$1 PM_NTT_MAXLOGC=$2 LOGN=${LOGNS:-20,23,24,25} timeout -k 10 120 python tools/ntt_timing.py 2>/dev/null | \
      sed "s/^/{\"log1\": $1, \"maxlogc\": $2, \"rep\": $rep, \"r\": /; s/\$/}/" >> $OUT/ab.jsonl || exit 1
  done
done
python3 - $OUT/ab.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    x = json.loads(l)
    d[(x["log1"], x["maxlogc"], x["r"]["log_n"])].append(x["r"]["wall_ms"])
for k in sorted(d): print(k, d[k])
PY

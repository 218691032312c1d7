#!/bin/bash
# NTT threads-per-block A/B (lib_xp build with -DPM_NTT_THREADS=512) against
# the tree's library, alternated twice in one call.
set -o pipefail
mkdir -p gpurun_out/ntt_ab2
export TMPDIR=/tmp
for rep in 1 2; do
for v in base t512; do
  if [ $v = base ]; then L=""; else L=halo2-aggregation_amd/lib_xp/libxp_$v.so; fi
  PM_LIB=$L LOGN=16,20,22,23,24,25 timeout -k 10 120 python tools/ntt_timing.py 2>/dev/null | sed "s/^/{\"v\": \"$v\", \"rep\": $rep, \"r\": /; s/\$/}/" >> gpurun_out/ntt_ab2/ab.jsonl || exit 1
done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ntt_ab2/ab.jsonl"):
    x = json.loads(l); d[(x["v"], x["r"]["log_n"])].append(x["r"]["wall_ms"])
for k in sorted(d): print(k, d[k])
PY

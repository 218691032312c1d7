#!/bin/bash
# Same-box A/B of the NTT LDS swizzle: the tree's lds_swz against the first
# round-3 form (lib_xp build with -DPM_NTT_SWZ_OLD=1), alternated 3 times.
set -o pipefail
mkdir -p gpurun_out/ntt_ab4
export TMPDIR=/tmp
for rep in 1 2 3; do
for v in new old; do
  if [ $v = new ]; then L=""; else L=halo2-aggregation_amd/lib_xp/libxp_swzold.so; fi
  PM_LIB=$L LOGN=20,22,23,24,25 timeout -k 10 120 python tools/ntt_timing.py 2>/dev/null | sed "s/^/{\"v\": \"$v\", \"rep\": $rep, \"r\": /; s/\$/}/" >> gpurun_out/ntt_ab4/ab.jsonl || exit 1
done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ntt_ab4/ab.jsonl"):
    x = json.loads(l); d[(x["r"]["log_n"], x["v"])].append(x["r"]["wall_ms"])
for k in sorted(d): print(k, d[k])
PY

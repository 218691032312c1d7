#!/bin/bash
# NTT threads per block (PM_NTT_THREADS2 / PM_NTT_THREADS3: 256 or 512),
# alternated twice in one call, plus the NTT tests at the 512 setting.
set -o pipefail
mkdir -p gpurun_out/ntt_ab3
export TMPDIR=/tmp
PM_NTT_THREADS2=512 PM_NTT_THREADS3=512 timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ntt_ab3/pytest512.log 2>&1 || { tail -20 gpurun_out/ntt_ab3/pytest512.log; exit 1; }
tail -1 gpurun_out/ntt_ab3/pytest512.log
for rep in 1 2; do
for v in 256 512; do
  PM_NTT_THREADS2=$v PM_NTT_THREADS3=$v LOGN=16,20,22,23,24,25 timeout -k 10 120 python tools/ntt_timing.py 2>/dev/null | sed "s/^/{\"threads\": $v, \"rep\": $rep, \"r\": /; s/\$/}/" >> gpurun_out/ntt_ab3/ab.jsonl || exit 1
done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ntt_ab3/ab.jsonl"):
    x = json.loads(l); d[(x["threads"], x["r"]["log_n"])].append(x["r"]["wall_ms"])
for k in sorted(d, key=lambda k: (k[1], k[0])): print(k, d[k])
PY

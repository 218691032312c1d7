#!/bin/bash
set -o pipefail
for pf in 0 1; do
  PM_PREFETCH=$pf LOGN=20,22 timeout -k 10 300 python tools/msm_timing.py 2>/dev/null | grep logn || exit 1
done

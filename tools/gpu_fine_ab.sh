#!/bin/bash
# Fine-sort LDS A/B (through gpurun, from the repo root): bash tools/gpu_fine_ab.sh TAG
#   parity of the LDS-resident modes on the known-dlog / golden MSM tests, then
#   tools/msm_timing.py per (PM_FINE_CACHE_KB, PM_FINE_CHUNK_KB) setting
set -o pipefail
TAG=${1:-fine}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PARITY=${PARITY:-0:0 8:8}
for CFG in $PARITY; do
  C=${CFG%%:*}; K=${CFG##*:}
  PM_FINE_CACHE_KB=$C PM_FINE_CHUNK_KB=$K timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "${PK:-golden or known_dlog or giant or resident_row}" > $OUT/parity_${C}_${K}.log 2>&1 \
    || { echo "parity $CFG failed"; tail -30 $OUT/parity_${C}_${K}.log; exit 1; }
  echo "parity $CFG: $(tail -1 $OUT/parity_${C}_${K}.log)"
done
CFGS=${CFGS:-0:0 b3:0 8:8 32:32}
for REP in 1 2; do
for CFG in $CFGS; do
  C=${CFG%%:*}; K=${CFG##*:}; L=halo2-aggregation_amd/lib/libpasta_msm.so
  case $C in [a-z]*) L=halo2-aggregation_amd/lib_xp/libxp_$C.so; C=0 ;; esac
  echo "cfg=$CFG rep=$REP"
  PM_LIB=$L PM_FINE_CACHE_KB=$C PM_FINE_CHUNK_KB=$K RESIDENT=1 LOGN=${LOGN:-19,20,22} timeout -k 10 180 python tools/msm_timing.py 2>/dev/null \
    | grep logn | sed "s/^{/{\"fine\": \"$CFG\", /" | tee -a $OUT/fine.jsonl | cut -c1-330 || { echo "timing $CFG failed"; exit 1; }
done
done

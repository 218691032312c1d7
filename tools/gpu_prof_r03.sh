#!/bin/bash
# Round-3 profiles (through gpurun, from the repo root): bash tools/gpu_prof_r03.sh TAG [parts]
#   kt    rocprofv3 --kernel-trace --stats of the headline-only bench
#   pmc   k_accumulate PMC passes (SQ / FETCH_SIZE / WRITE_SIZE) on the resident row-table MSM at 2^19,
#         2^20, 2^22 (pmc/) and the raw-bases MSM at 2^20 (pmc_raw/)
#   ntt   NTT 2^25 FETCH_SIZE / WRITE_SIZE
#   proj  strong-scaling projection of the 2^22 Vesta MSM (tools/strong_projection.py)
set -o pipefail
TAG=${1:-prof}
PARTS=${2:-"kt pmc ntt proj"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for P in $PARTS; do
  echo "== $P"
  case $P in
    kt)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o run -- python3 bench.py --no-cpu \
        --logn22 0 --strong-logn 0 --fixed 0 --ntt-logn 0 --ntt-large-logn 0 --accum-batch 0 --accum-b16 0 --small-n 0 \
        > $OUT/kt.log 2>&1 || { echo "kernel trace failed"; tail -20 $OUT/kt.log; exit 1; }
      find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
      cut -c1-150 $OUT/kernel_stats.csv | head -14 ;;
    pmc)
      RESIDENT=1 LOGNS="19 20 22" bash tools/gpu_pmc_r02.sh $TAG/pmc || exit 1
      RESIDENT=0 LOGNS="20" bash tools/gpu_pmc_r02.sh $TAG/pmc_raw || exit 1 ;;
    ntt)
      NTT_ARGS="--ntt-logn 0 --ntt-large-logn 25" bash tools/gpu_ntt_pmc.sh $TAG/ntt25 || exit 1 ;;
    proj)
      timeout -k 10 300 python tools/strong_projection.py 22 1 | tee $OUT/strong_projection.jsonl || exit 1 ;;
  esac
done

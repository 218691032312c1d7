# A/B timing of experiment builds (PM_LIB) on one box: bash tools/gpu_xp.sh "0 16 15" [env]
set -o pipefail
for X in $1; do
  if [ $X = 0 ]; then L=halo2-aggregation_amd/lib/libpasta_msm.so; else L=halo2-aggregation_amd/lib_xp/libxp$X.so; fi
  echo "xp=$X $2"
  env $2 PM_LIB=$L LOGN=${LOGN:-20} timeout -k 10 120 python tools/msm_timing.py 2>/dev/null | tail -n +2 || exit 1
done

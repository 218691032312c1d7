# A/B NTT timing of experiment builds (PM_LIB): bash tools/gpu_xp_ntt.sh "0 512"
set -o pipefail
for X in $1; do
  if [ $X = 0 ]; then L=halo2-aggregation_amd/lib/libpasta_msm.so; else L=halo2-aggregation_amd/lib_xp/libxp$X.so; fi
  echo "xp=$X"
  PM_LIB=$L LOGN=${LOGN:-16,20,22} timeout -k 10 120 python tools/ntt_timing.py 2>/dev/null || exit 1
done

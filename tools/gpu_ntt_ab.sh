set -o pipefail
mkdir -p gpurun_out/ntt_ab
export TMPDIR=/tmp
for rep in 1 2; do
for v in base t512 p10; do
  if [ $v = base ]; then L=""; else L=halo2-aggregation_amd/lib_xp/libxp_$v.so; fi
  PM_LIB=$L LOGN=16,20,22,24,25 timeout -k 10 120 python tools/ntt_timing.py 2>/dev/null | sed "s/^/{\"v\": \"$v\", \"rep\": $rep, \"r\": /; s/\$/}/" >> gpurun_out/ntt_ab/ab.jsonl || exit 1
done
done
cut -c1-200 gpurun_out/ntt_ab/ab.jsonl

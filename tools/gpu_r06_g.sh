#!/bin/bash
# Round 6: the headline-only bench under rocprofv3 --kernel-trace --stats
# (the k_accumulate summary the roofline's HIP-event average must agree
# with), and a 2-rank rehearsal of the N > 1 bench on the one GPU
# (PM_BENCH_SHARE_GPU=1: gloo collectives on host copies; numbers say
# nothing about scaling, the flow and the output line are what is checked).
set -o pipefail
OUT=gpurun_out/r06_g
mkdir -p $OUT
export TMPDIR=/tmp
HEAD="--no-cpu --logn22 0 --strong-logn 0 --fixed 0 --fixed23 0 --ntt-logn 0 --ntt-large-logn 0 --accum-batch 0 --accum-b16 0 --accum-b32 0 --accum-large 0 --inst-batch 0 --small-n 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o run -- python3 bench.py $HEAD --detail $OUT/kt_headline_detail.json > $OUT/kt_headline.log 2>&1 || { tail -20 $OUT/kt_headline.log; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/kt_headline_kernel_stats.csv \;
rm -rf $OUT/kt
tail -1 $OUT/kt_headline.log | cut -c1-400
PM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --fixed23 0 --ntt-large-logn 0 --small-n 0 --detail $OUT/share2_detail.json > $OUT/share2.log 2>&1 || { tail -30 $OUT/share2.log; exit 1; }
tail -1 $OUT/share2.log | cut -c1-600

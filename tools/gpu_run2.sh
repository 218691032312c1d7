set -o pipefail
OUT=gpurun_out/s2b; mkdir -p $OUT
timeout -k 10 120 ./tools/microbench_lat > $OUT/microbench_lat.jsonl 2>&1; echo "mb rc=$?"; cat $OUT/microbench_lat.jsonl
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
LOGN=18,20,22 timeout -k 10 300 python tools/msm_timing.py > $OUT/msm_timing.jsonl 2>&1 || { tail -30 $OUT/msm_timing.jsonl; exit 1; }
cat $OUT/msm_timing.jsonl

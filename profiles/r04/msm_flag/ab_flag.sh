set -o pipefail
mkdir -p gpurun_out/flag
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_msm_gpu.py tests/test_msm_small_gpu.py tests/test_fixed_gpu.py tests/test_accum_gpu.py > gpurun_out/flag/tests.log 2>&1 &&
for i in 1 2; do
 timeout -k 10 120 env RESIDENT=1 LOGN=16,20,22 REPS=40 python -u tools/msm_timing.py > gpurun_out/flag/new_$i.jsonl 2>&1 &&
 timeout -k 10 120 env PM_LIB=ab/libpasta_msm_head.so RESIDENT=1 LOGN=16,20,22 REPS=40 python -u tools/msm_timing.py > gpurun_out/flag/head_$i.jsonl 2>&1 || exit 1
done &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/flag/bench.json 2> gpurun_out/flag/bench.err

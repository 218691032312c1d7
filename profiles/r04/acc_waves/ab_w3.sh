set -o pipefail
O=gpurun_out/w3; mkdir -p $O
for i in 1 2 3; do
 timeout -k 10 120 env RESIDENT=1 LOGN=20,22 REPS=30 python -u tools/msm_timing.py > $O/w4_$i.jsonl 2>&1 &&
 timeout -k 10 120 env PM_LIB=tools/xpbin/libpasta_msm_w3.so RESIDENT=1 LOGN=20,22 REPS=30 python -u tools/msm_timing.py > $O/w3_$i.jsonl 2>&1 || exit 1
done &&
timeout -k 10 120 env PM_LIB=tools/xpbin/libpasta_msm_w3.so python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_msm_gpu.py -k "headline or vs_c_port" > $O/tests_w3.log 2>&1

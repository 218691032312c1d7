set -o pipefail
O=gpurun_out/ev2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_proof_gpu.py tests/test_accum_gpu.py > $O/tests.log 2>&1 &&
for i in 1 2 3; do
 timeout -k 10 150 env STEPS=60 python -u tools/accum_pipelined.py > $O/new_$i.jsonl 2>&1 &&
 timeout -k 10 150 env STEPS=60 PM_LIB=tools/xpbin/libpasta_msm_prev.so python -u tools/accum_pipelined.py > $O/prev_$i.jsonl 2>&1 || exit 1
done

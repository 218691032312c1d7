set -o pipefail
O=gpurun_out/dbl; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_accum_gpu.py tests/test_proof_gpu.py > $O/tests.log 2>&1 &&
timeout -k 10 120 ./tools/microbench_chain > $O/chain_new.jsonl 2>&1 &&
timeout -k 10 120 ./tools/xpbin/microbench_chain_head > $O/chain_head.jsonl 2>&1 &&
for i in 1 2; do
 timeout -k 10 150 python -u tools/accum_timing.py > $O/acc_new_$i.jsonl 2>&1 &&
 timeout -k 10 150 env PM_LIB=tools/xpbin/libpasta_msm_head.so python -u tools/accum_timing.py > $O/acc_head_$i.jsonl 2>&1 || exit 1
done &&
timeout -k 10 150 python -u tools/accum_pipelined.py > $O/pipelined.jsonl 2>&1

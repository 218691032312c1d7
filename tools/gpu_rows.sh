set -o pipefail
mkdir -p gpurun_out/rows gpurun_out/ntt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "fixed or ntt" --timeout 200 --timeout-method thread > gpurun_out/rows/pytest.txt 2>&1 || { tail -30 gpurun_out/rows/pytest.txt; exit 1; }
tail -2 gpurun_out/rows/pytest.txt
for R in 2 4 0; do FIXED_ROWS=$R FIXED_C=16 LOGN=19,20,22 timeout -k 10 200 python tools/msm_timing.py 2>/dev/null | grep '"fixed"' || exit 1; done > gpurun_out/rows/timing.jsonl
LOGN=19,20,22 timeout -k 10 200 python tools/msm_timing.py 2>/dev/null | grep logn >> gpurun_out/rows/timing.jsonl || exit 1
bash tools/gpu_xp_ntt.sh "2r256 512 1024 0 4r512 4r1024" > gpurun_out/ntt/out.txt 2>&1 || exit 1

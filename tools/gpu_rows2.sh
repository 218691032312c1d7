set -o pipefail
mkdir -p gpurun_out/rows2 gpurun_out/ntt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "resident or msm_gpu" --timeout 200 --timeout-method thread > gpurun_out/rows2/pytest.txt 2>&1 || { tail -30 gpurun_out/rows2/pytest.txt; exit 1; }
tail -2 gpurun_out/rows2/pytest.txt
bash tools/gpu_xp_ntt.sh "2r256 512 1024 0 4r512 4r1024" > gpurun_out/ntt/out.txt 2>&1 || { tail -20 gpurun_out/ntt/out.txt; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/rows2/bench.json 2> gpurun_out/rows2/bench.err || { tail -30 gpurun_out/rows2/bench.err; exit 1; }

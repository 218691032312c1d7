set -o pipefail
NTT_ARGS="--ntt-logn 20 --ntt-large-logn 0" bash tools/gpu_ntt_pmc.sh r03ntt20 && NTT_ARGS="--ntt-logn 0 --ntt-large-logn 25" bash tools/gpu_ntt_pmc.sh r03ntt25

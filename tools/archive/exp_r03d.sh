set -o pipefail
bash tools/gpu_round.sh r03d || exit 1
bash tools/exp_variants.sh rbab3 old base || exit 1

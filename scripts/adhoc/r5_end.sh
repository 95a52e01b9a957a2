set -o pipefail
scripts/gpu.sh tests r5_end2/t && scripts/gpu.sh smoke r5_end2

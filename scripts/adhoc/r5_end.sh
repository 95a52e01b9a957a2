set -o pipefail
scripts/gpu.sh tests r5_end/t && scripts/gpu.sh smoke r5_end

set -o pipefail
scripts/gpu.sh all r5_final && scripts/gpu.sh trace r5_final/dist --force_allreduce

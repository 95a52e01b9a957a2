set -o pipefail
scripts/gpu.sh tests r5_last/t "dist_chains or verify_chain or xgmi or bench_ or dist_chain"

set -o pipefail
scripts/gpu.sh sweep r5_fp32dist "f||--force_allreduce" "b64f||--force_allreduce --batch_size 64 --no_fp32"

set -o pipefail
scripts/gpu.sh all r5_final2 && scripts/gpu.sh bench r5_final2/dist --force_allreduce --no_fp32 && scripts/gpu.sh bench r5_final2/b64 --batch_size 64 --no_fp32

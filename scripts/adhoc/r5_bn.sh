set -o pipefail
scripts/gpu.sh tests r5_bn/t "resnet or bn_ or conv_gemm or halo" &&
scripts/gpu.sh resnet r5_bn &&
scripts/gpu.sh trace r5_bn/dist --force_allreduce --no_breakdown

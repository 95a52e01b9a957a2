set -o pipefail
scripts/gpu.sh sweep r5_m3knobs "base||--no_fp32 --force_allreduce" "fr2||--no_fp32 --force_allreduce --fuse_reduce 2" "base2||--no_fp32 --force_allreduce" "fr2b||--no_fp32 --force_allreduce --fuse_reduce 2"

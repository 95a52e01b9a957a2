set -o pipefail
scripts/gpu.sh sweep r5_m2sweep "m2_128||--no_fp32 --force_allreduce --dist_mode 2 --xar_blocks 128" "m2_173||--no_fp32 --force_allreduce --dist_mode 2 --xar_blocks 173" "m3_cap128|DDP_AMD_XGMI_GRID_CAP=128|--no_fp32 --force_allreduce" "m3|| --no_fp32 --force_allreduce"

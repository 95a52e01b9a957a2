set -o pipefail
out=gpurun_out/r5_nofence; mkdir -p $out
scripts/gpu.sh tests r5_nofence/t "dist_chains or verify_chain or xgmi_world1 or dist_chain or bench_forced" &&
scripts/gpu.sh sweep r5_nofence "m3||--no_fp32 --force_allreduce" "m2||--no_fp32 --force_allreduce --dist_mode 2" "m2b||--no_fp32 --force_allreduce --dist_mode 2 --xar_blocks 96" &&
scripts/gpu.sh trace r5_nofence/dist --force_allreduce --no_breakdown

set -o pipefail
out=gpurun_out/r5_xar; mkdir -p $out

timeout -k 10 200 python scripts/adhoc/xar_debug.py 2>&1 | grep -v amdgpu.ids | tail -4
scripts/gpu.sh tests r5_xar/t "premul or engine_xgmi or rccl_allreduce or comm_tune or module_ddp_world1" || exit 1
scripts/gpu.sh sweep r5_xar "fx||--no_fp32 --force_allreduce --comm xgmi" "fx1||--no_fp32 --force_allreduce --comm xgmi --dist_mode 1" "fr||--no_fp32 --force_allreduce --comm rccl" "fx32||--dtype fp32 --force_allreduce --comm xgmi" || exit 1
scripts/gpu.sh trace r5_xar/trace_fx --force_allreduce --comm xgmi --no_breakdown || exit 1
timeout -k 10 200 python scripts/stamps.py --graph --force_allreduce --comm xgmi > $out/stamps_fx.txt 2>&1 && grep -v amdgpu.ids $out/stamps_fx.txt
timeout -k 10 200 python scripts/stamps.py --graph > $out/stamps_local.txt 2>&1 && grep -v amdgpu.ids $out/stamps_local.txt

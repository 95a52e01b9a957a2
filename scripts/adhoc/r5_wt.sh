set -o pipefail
scripts/gpu.sh tests r5_wt/t "dist_chains or fused_optimizer or level3_ragged or xgmi_world1" &&
scripts/gpu.sh ab r5_wt "so=ab_so/_C_base.so" "so=pytorch-distributed-data-parallel-ddp-trainer_amd/_C.so" 2 &&
scripts/gpu.sh ab r5_wt/dist "so=ab_so/_C_base.so" "so=pytorch-distributed-data-parallel-ddp-trainer_amd/_C.so" 2 --force_allreduce

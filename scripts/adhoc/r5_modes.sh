set -o pipefail
out=gpurun_out/r5_pair2; mkdir -p $out
timeout -k 10 200 python scripts/stamps.py --force_allreduce --comm xgmi > $out/stamps_m3.txt 2>&1 && grep "^xgmi\|grad_reduce\|fc_bwd" $out/stamps_m3.txt | cut -c1-330 &&
scripts/gpu.sh tests r5_pair2/t "dist_chains or verify_chain or xgmi_world1 or dist_chain or premul" &&
scripts/gpu.sh sweep r5_pair2 "m3||--force_allreduce --comm xgmi"

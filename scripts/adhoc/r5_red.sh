set -o pipefail
out=gpurun_out/r5_red2; mkdir -p $out
scripts/gpu.sh tests r5_red2/t "fused_reduce or level3 or fp32 or grad_reduce or wgrad or dist_chains or b64 or resnet" &&
timeout -k 10 200 python scripts/stamps.py --graph --batch_size 64 > $out/stamps_b64.txt 2>&1 &&
timeout -k 10 200 python scripts/stamps.py --graph --dtype fp32 > $out/stamps_fp32.txt 2>&1 &&
grep -h "grad_reduce\|wgrad " $out/stamps_b64.txt $out/stamps_fp32.txt | cut -c1-300 &&
scripts/gpu.sh sweep r5_red2 "b32||" "b64||--batch_size 64 --no_fp32"

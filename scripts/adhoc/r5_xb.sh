set -o pipefail
out=gpurun_out/r5_xb; mkdir -p $out
timeout -k 10 200 python scripts/stamps.py --graph --force_allreduce --comm xgmi --xgmi_blocks > $out/stamps.txt 2>&1

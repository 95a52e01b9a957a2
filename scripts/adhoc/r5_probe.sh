set -o pipefail
out=gpurun_out/r5_probe; mkdir -p $out
timeout -k 10 200 python scripts/stamps.py --graph --batch_size 64 > $out/stamps_b64.txt 2>&1 &&
timeout -k 10 200 python scripts/stamps.py --graph --dtype fp32 > $out/stamps_fp32.txt 2>&1 &&
timeout -k 10 200 python scripts/stamps.py --graph > $out/stamps_b32.txt 2>&1 &&
grep -h "blocks" $out/stamps_b64.txt $out/stamps_fp32.txt | cut -c1-300

set -o pipefail
out=gpurun_out/r5_stamps_final; mkdir -p $out
timeout -k 10 200 python scripts/stamps.py --graph --pxt_fwd 1 > $out/stamps_pf1.txt 2>&1 &&
timeout -k 10 200 python scripts/stamps.py --graph > $out/stamps_pf2.txt 2>&1 &&
timeout -k 10 200 python scripts/stamps.py --graph --force_allreduce --comm xgmi > $out/stamps_dist.txt 2>&1 &&
grep -h "blocks" $out/stamps_pf1.txt | cut -c1-200

set -o pipefail
out=gpurun_out/r5_xar4; mkdir -p $out
for x in 0 1 2; do
DDP_AMD_XAR_EXPT=$x timeout -k 10 200 python scripts/stamps.py --force_allreduce --comm xgmi > $out/stamps_x$x.txt 2>&1; echo "expt $x"; grep "^xgmi\|grad_reduce" $out/stamps_x$x.txt | cut -c1-330
done

set -o pipefail
out=gpurun_out/r5_pf1; mkdir -p $out
for r in 1 2 3; do
  for v in pf2 pf1; do
    a=""; [ $v = pf1 ] && a="--pxt_fwd 1"
    timeout -k 10 120 python bench.py --no_fp32 --steps 20 --warmup 5 $a > $out/d_${v}_$r.json 2>> $out/err.log || exit 1
    timeout -k 10 200 python bench.py --no_fp32 $a > $out/l_${v}_$r.json 2>> $out/err.log || exit 1
    echo "$v run $r: driver $(grep -o '"value": [0-9.]*' $out/d_${v}_$r.json) | 1000 $(grep -o '"value": [0-9.]*' $out/l_${v}_$r.json)"
  done
done
timeout -k 10 200 python bench.py --no_fp32 --force_allreduce --pxt_fwd 1 > $out/l_dist_pf1.json 2>> $out/err.log && echo "dist pf1: $(grep -o '"value": [0-9.]*' $out/l_dist_pf1.json)"

set -o pipefail
out=gpurun_out/r5_gsweep; mkdir -p $out
for r in 1 2 3; do
  for g in 20 10 5 2; do
    timeout -k 10 120 python bench.py --no_fp32 --steps 20 --warmup 5 --graph_steps $g > $out/g${g}_$r.json 2>> $out/err.log || exit 1
    echo "g$g run $r: $(grep -o '"value": [0-9.]*' $out/g${g}_$r.json)"
  done
done

#!/bin/bash
# bf16 B=32 tiling sweep (in-call 1000-step and driver-shaped runs), results in gpurun_out/$1
out=gpurun_out/${1:-sweep}; mkdir -p $out
run() {
  tag=$1; shift
  timeout -k 10 200 python bench.py --no_fp32 "$@" > $out/l_$tag.json 2>>$out/err.log || exit 1
  timeout -k 10 200 python bench.py --no_fp32 --steps 20 --warmup 5 "$@" > $out/d_$tag.json 2>>$out/err.log || exit 1
  echo "$tag: 1000 $(grep -o '"value": [0-9.]*' $out/l_$tag.json) | driver $(grep -o '"value": [0-9.]*' $out/d_$tag.json)"
}
run base
run R4 --wgrad_rows 4
run R14 --wgrad_rows 14
run pf1 --pxt_fwd 1
run a0 --store_a1 0
run a2 --store_a1 2
run base2

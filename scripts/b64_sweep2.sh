# B = 64 knobs on top of the two-blocks-per-CU level-3 forward (+ B = 32 regression check)
out=gpurun_out/${1:-r4_k}; mkdir -p $out
run() { tag=$1; shift
  timeout -k 10 200 python bench.py --no_fp32 "$@" > $out/l_$tag.json 2>>$out/err.log || exit 1
  timeout -k 10 200 python bench.py --no_fp32 --steps 20 --warmup 5 "$@" > $out/d_$tag.json 2>>$out/err.log || exit 1
  echo "$tag: 1000 $(grep -o '"value": [0-9.]*' $out/l_$tag.json) | driver $(grep -o '"value": [0-9.]*' $out/d_$tag.json)"
}
run b32 
run b64 --batch_size 64
DDP_AMD_FC_FIRST=1 run b64_ff1 --batch_size 64
run b64_R14 --batch_size 64 --wgrad_rows 14
run b64_R4 --batch_size 64 --wgrad_rows 4
run b64_pd1 --batch_size 64 --pxt_dgrad 1
DDP_AMD_BWD_INTERLEAVE=0 run b64_il0 --batch_size 64
run b32_2

mkdir -p gpurun_out/r4_g
for ff in 0 1; do for px in 1 2; do
  DDP_AMD_FC_FIRST=$ff timeout -k 10 200 python bench.py --batch_size 64 --no_fp32 --pxt_fwd $px > gpurun_out/r4_g/b64_ff${ff}_px$px.json 2>>gpurun_out/r4_g/err.log || exit 1
  echo "B64 fc_first $ff pxt_fwd $px: $(grep -o '"value": [0-9.]*' gpurun_out/r4_g/b64_ff${ff}_px$px.json)"
done; done

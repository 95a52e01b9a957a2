# N-rank rehearsal of the fused engine's xGMI data plane on ONE GPU (gloo control plane,
# every rank on cuda:0): checks the 4- and 8-way all-reduce protocol end to end.  The
# ranks time-share one GPU, so the all-reduce grid is capped and the barrier bound raised.
set -o pipefail
out=gpurun_out/reh
mkdir -p $out
export DDP_AMD_XGMI_GRID_CAP=${DDP_AMD_XGMI_GRID_CAP:-16} DDP_AMD_XGMI_TIMEOUT_S=${DDP_AMD_XGMI_TIMEOUT_S:-20}
for n in ${NS:-4 8}; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --backend gloo --comm xgmi --steps 200 --warmup 20 \
    > $out/bench_n$n.log 2>&1 || { echo "n=$n failed"; exit 1; }
done
echo exit=0

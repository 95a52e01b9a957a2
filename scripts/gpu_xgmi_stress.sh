set -o pipefail
# usage: bash scripts/gpu_xgmi_stress.sh TAG STEPS "ENV=.. ENV=.." ["ENV.." ...]  (one run per env set, default oneshot plan)
out=gpurun_out/${1:-xs}
steps=${2:-40}
shift 2
mkdir -p $out
k=0
for envs in "$@"; do
  k=$((k+1))
  echo "== env: $envs"
  env DDP_AMD_XGMI_TIMEOUT_S=5 $envs timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 \
    scripts/xgmi_stress.py --steps $steps > $out/s_$k.log 2>&1 || { echo rc=$?; tail -20 $out/s_$k.log; exit 1; }
  grep -A3 "bad_steps" $out/s_$k.log; grep "first xGMI" $out/s_$k.log
done

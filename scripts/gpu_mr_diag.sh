set -o pipefail
out=gpurun_out/${1:-mrd}
mkdir -p $out
cd $out
R=$GRAFT_REPO_ROOT
run() { timeout -k 10 240 python -u $R/train_ddp.py --world_size 2 --backend gloo --device gpu --data synthetic --verify_replicas --epochs 3 --batch_size 32 --max_steps 30 --log_every 1000 --no_save --engine module "$@"; }
for i in 1 2; do
  echo "== verify-each-step $i"; DDP_AMD_VERIFY_EACH_STEP=1 run > v_$i.log 2>&1; echo rc=$?; grep -h -o "step [0-9]*: replicas differ.*\|differing tensors.*\|identical after epoch [0-9]" v_$i.log
done

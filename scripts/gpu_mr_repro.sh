set -o pipefail
for args in "--oneshot_max 65536" "--oneshot_max 65536 --check_grads" "--oneshot_max 65536 --sync_step" "--oneshot_max 65536 --sync_fwd" "--oneshot_max 65536 --sync" "" ; do
  echo "args: $args"
  timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 scripts/mr_repro.py --steps 40 $args 2>&1 | grep "first divergent" || exit $?
done

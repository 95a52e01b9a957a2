# alternating ResNet-18 bench sweep on one box: gpu_resnet_sweep.sh OUT "args1" "args2" ...
set -o pipefail
out=gpurun_out/${1:-rs}; shift
mkdir -p $out
for rep in 1 2 3; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python -u bench.py --model resnet18 --steps 200 --warmup 10 $v > $out/r_${i}_$rep.json 2>> $out/err.log || exit $?
    python -c "import json; d=json.loads([l for l in open('$out/r_${i}_$rep.json') if l.startswith('{')][-1]); print('[$v]', d['value'], d['ms_per_step'])"
  done
done

# halo wgrad: ResNet GPU tests, then the ResNet bench with the halo kernel on / off / target sweep
set -o pipefail
out=gpurun_out/${1:-hw}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for v in "1 256" "0 256" "1 512" "1 128"; do
    set -- $v
    timeout -k 10 200 python -u bench.py --model resnet18 --steps 100 --warmup 10 --wgrad_halo $1 --wgrad_halo_target $2 > $out/r_$1_$2_$rep.json 2>> $out/err.log || exit $?
    python -c "import json; d=json.load(open('$out/r_$1_$2_$rep.json')); print('halo $1 target $2', d['value'], d['ms_per_step'])"
  done
done

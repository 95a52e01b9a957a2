set -o pipefail
out=gpurun_out/${1:-hab}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2 3; do
  for h in 1 0; do
    timeout -k 10 200 python -u bench.py --model resnet18 --steps 200 --warmup 10 --wgrad_halo $h > $out/r_${h}_$rep.json 2>> $out/err.log || exit $?
    grep -o '"value": [0-9.]*' $out/r_${h}_$rep.json | head -1 | sed "s/^/halo $h /"
  done
done

# module-path multi-rank: ResNet DDP 2-rank xGMI rehearsal (eager + graph), full suite, resnet bench
set -o pipefail
out=gpurun_out/${1:-r2d}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread > $out/pytest_xgmi.log 2>&1
rc=$?; tail -3 $out/pytest_xgmi.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
grep -E "FAIL|passed|failed" $out/pytest_gpu.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --model resnet18 --steps 100 --warmup 10 > $out/bench_resnet.json 2> $out/bench.err && \
timeout -k 10 400 python -u bench.py --model resnet18 --gpus 2 --backend gloo --steps 30 --warmup 5 --no_scaling_ref > $out/bench_resnet_n2_gloo.json 2>> $out/bench.err
echo exit=$?
cat $out/bench_resnet.json $out/bench_resnet_n2_gloo.json

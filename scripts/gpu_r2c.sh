# bucket-plan flexibility: xGMI rehearsal tests (2 ranks on one GPU), engine tests, bench
set -o pipefail
out=gpurun_out/${1:-r2c}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_xgmi_gpu.py tests/test_engine_gpu.py -x -v --timeout 240 --timeout-method thread > $out/pytest_xgmi.log 2>&1
rc=$?; tail -3 $out/pytest_xgmi.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
tail -3 $out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --comm xgmi --steps 200 --warmup 20 --bucket_cap_mb 0.05 --first_bucket_mb 1e-6 > $out/bench_n2_b4.json 2> $out/bench.err
echo exit=$?
cat $out/bench_n2_b4.json

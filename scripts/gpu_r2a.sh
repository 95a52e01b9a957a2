# Round-2 check: new CLI/momentum tests, full GPU suite, self-launched 2-rank rehearsal bench.
set -o pipefail
out=gpurun_out/${1:-r2a}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_cli_gpu.py -x -v --timeout 200 --timeout-method thread > $out/pytest_cli.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --comm xgmi --steps 200 --warmup 20 > $out/bench_n2_gloo.json 2> $out/bench_n2_gloo.err && \
timeout -k 10 180 python -u bench.py > $out/bench.json 2> $out/bench.err
echo exit=$?

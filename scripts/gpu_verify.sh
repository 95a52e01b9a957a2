set -o pipefail
mkdir -p gpurun_out/v1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v1/pytest_gpu.log 2>&1 && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v1/smoke.log 2>&1 && \
timeout -k 10 180 python -u bench.py > gpurun_out/v1/bench.log 2>&1 && \
timeout -k 10 180 python -u bench.py --model resnet18 --steps 50 --warmup 10 > gpurun_out/v1/bench_resnet.log 2>&1
echo exit=$?

# One-call GPU check: pytest -m gpu, smoke(), both benches, and a rocprofv3 kernel-stats
# pass over the flagship (SimpleCNN) bench.  Output under gpurun_out/${1:-v1}.
set -o pipefail
out=gpurun_out/${1:-v1}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && \
timeout -k 10 180 python -u bench.py > $out/bench.log 2>&1 && \
timeout -k 10 180 python -u bench.py --model resnet18 --steps 200 --warmup 10 > $out/bench_resnet.log 2>&1 && \
timeout -k 10 180 python -u bench.py --batch_size 64 > $out/bench_b64.log 2>&1 && \
timeout -k 10 180 python -u bench.py --dtype fp32 > $out/bench_fp32.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --comm xgmi --steps 200 --warmup 20 > $out/bench_n2_rehearsal.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python -u bench.py --steps 200 --warmup 20 > $out/prof.log 2>&1
echo exit=$?
